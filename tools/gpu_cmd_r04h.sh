#!/bin/bash
# r04h: where the wavetable kernel's time goes on C2: kernel stats of diagnostic
# builds (tdiag1 build only, tdiag2 no build, tdiag3 no table reads, tdiag4 no stores)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=c2 VARIANTS="tdiag1 tdiag2 tdiag3 tdiag4" KERNELS="sg_sine_bank_tab sg_harm_copy" bash tools/gpu_kstat_ab.sh r04h
