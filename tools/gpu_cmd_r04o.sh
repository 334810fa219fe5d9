#!/bin/bash
# r04o: PMC of the wavetable kernel on C2 (direct mode, default, and W mode SG_TAB_DIRECT=0):
# LDS bank conflicts, LDS / VALU issue, waits
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
G2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_ANY"
CFG=c2 BENCH_ARGS="--rms-calls 0" bash tools/gpu_pmc.sh r04o_dir "$G1" "$G2"
SG_TAB_DIRECT=0 CFG=c2 BENCH_ARGS="--rms-calls 0" bash tools/gpu_pmc.sh r04o_w "$G1" "$G2"
python tools/pmc_summary.py r04o_dir c2 4 > gpurun_out/r04o_dir.json
python tools/pmc_summary.py r04o_w c2 4 > gpurun_out/r04o_w.json
python - <<'PY'
import json
for t in ("dir", "w"):
    d = json.load(open("gpurun_out/r04o_%s.json" % t))["kernels"]
    for k, v in d.items():
        if "sg_sine_bank_tab" in k or "sg_harm_copy" in k:
            print(t, k, {c: round(x) for c, x in v.items() if c != "launches"})
PY
