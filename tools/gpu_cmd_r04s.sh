#!/bin/bash
# r04s: sg_mix occupancy A/B on C5: waves per SIMD capped at 6 / 8 (mixw6, mixw8), 4 samples
# per thread per chunk (mixe4), both (mixe4w8): kernel stats + the bench's RMS check
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=c5 VARIANTS="mixw6 mixw8 mixe4 mixe4w8" KERNELS="sg_mix sg_mix_hp" bash tools/gpu_kstat_ab.sh r04s
cd "$R"
for v in default mixw6 mixw8 mixe4 mixe4w8; do echo "$v $(grep -o '"rms_error_vs_oracle": [0-9.e-]*' gpurun_out/r04s_$v.log)"; done
