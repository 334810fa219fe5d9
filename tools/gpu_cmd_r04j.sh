#!/bin/bash
# r04j: wavetable kernel phases on C2 (diagnostic builds): d1 build only, s1/s2/s4 build
# only without twiddles / FFT stages / coefficients, s7 loads only, d2 no build, d4 no stores
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd "$R"
CFG=c2 VARIANTS="tab_d1 tab_s1 tab_s2 tab_s4 tab_s7 tab_d2 tab_d4" KERNELS="sg_sine_bank_tab" bash tools/gpu_kstat_ab.sh r04j
