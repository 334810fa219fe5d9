#!/bin/bash
# r04q: sg_mix tile size (2048 / 4096 vs 8192 samples per workgroup: fewer chunk loops, so
# fewer waits of a chunk's loads behind the previous chunk's stores) and sg_harm_finalize
# tiles per workgroup (1 / 2 vs 4): C5 kernel stats
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=c5 VARIANTS="mix2048 mix4096 fin1 fin2 pp8 pf8 pf16" KERNELS="sg_mix sg_harm_finalize sg_sine_bank_pairs sg_sine_bank_tall_pairs" bash tools/gpu_kstat_ab.sh r04q
for v in default mix2048 mix4096 fin1 fin2 pp8 pf8 pf16; do echo "$v $(grep -o '"rms_error_vs_oracle": [0-9.e-]*' gpurun_out/r04q_$v.log)"; done
