#!/bin/bash
# r04v: sg_fft_frames64 threads per frame (128 / 512 / 1024 vs 256): C5 kernel stats + RMS
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=c5 VARIANTS="f64t128 f64t512 f64t1024" KERNELS="sg_fft_frames64 sg_ola" bash tools/gpu_kstat_ab.sh r04v
cd "$R"
for v in default f64t128 f64t512 f64t1024; do echo "$v $(grep -o '"rms_error_vs_oracle": [0-9.e-]*' gpurun_out/r04v_$v.log)"; done
