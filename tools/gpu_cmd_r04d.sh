#!/bin/bash
# r04d: per-kernel A/B at equal planner: two-chain sine bank (famp0), fp64-frame grouped stages (kg2, kg3);
# the fp64 parity tests under kg3
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
SG_HIP_LIB=$R/soundgen_beta_amd/lib/exp_kg3.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "every_preset or extreme_calls or c4_calls" > gpurun_out/pytest_kg3.log 2>&1 || { tail -30 gpurun_out/pytest_kg3.log; exit 1; }
tail -2 gpurun_out/pytest_kg3.log
VARIANTS="famp0 kg2 kg3" KERNELS="sg_sine_bank sg_sine_bank_pairs sg_sine_bank_tall sg_sine_bank_tall_pairs sg_sine_bank_hp sg_fft_frames64" bash tools/gpu_kstat_ab.sh r04d_kab
