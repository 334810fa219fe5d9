#!/bin/bash
# r03n: spectral GPU tests (register output path), A/B on C5/C3, PMC passes over C5
set -e
R=$(pwd)
PYTEST_K="spectral or c5 or c3 or noise" bash tools/gpu_tests.sh
NOTEST=1 CFGS="c5 c3" VARIANTS="noreg" STEPS=8 bash tools/gpu_ab.sh stft5
CFG=c5 BENCH_ARGS="--no-d2h" bash tools/gpu_pmc.sh pmc_r03n \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES"
python tools/pmc_summary.py pmc_r03n c5 > gpurun_out/pmc_r03n.txt 2>&1 || true
head -40 gpurun_out/pmc_r03n.txt
