#!/bin/bash
# r04fin8: sg_harm_finalize capped at 8 waves per SIMD (SGPRs 106 -> 78, spilled to VGPR lanes) vs default
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=c5 VARIANTS="fin8" KERNELS="sg_harm_finalize" bash tools/gpu_kstat_ab.sh r04fin8
cd "$R"
for v in default fin8; do echo "$v $(grep -o '"rms_error_vs_oracle": [0-9.e-]*' gpurun_out/r04fin8_$v.log)"; done
