#!/bin/bash
# r04occ: sine-bank kernels capped for more waves per SIMD (sb8: sg_sine_bank 7 -> 8; tall6 /
# hp6: sg_sine_bank_tall / _hp 5 -> 6, small spills) vs default: C5 kernel stats + RMS
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=c5 VARIANTS="sb8 tall6 hp6" KERNELS="sg_sine_bank sg_sine_bank_tall sg_sine_bank_hp" bash tools/gpu_kstat_ab.sh r04occ
cd "$R"
for v in default sb8 tall6 hp6; do echo "$v $(grep -o '"rms_error_vs_oracle": [0-9.e-]*' gpurun_out/r04occ_$v.log)"; done
