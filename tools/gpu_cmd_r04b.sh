#!/bin/bash
# r04b: full GPU suite (with the R shim tests), fp32-error vs rho study, default bench line,
# kernel stats with every kernel alone (SG_OVERLAP=0).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
echo "head $(cat .head_sha 2>/dev/null || echo unknown) + worktree" > gpurun_out/head.txt
bash tools/gpu_tests.sh
timeout -k 10 400 python tools/selector_study.py gpurun_out/selector_r04b.json 192 > gpurun_out/selector_r04b.log 2>&1
tail -28 gpurun_out/selector_r04b.log
timeout -k 10 400 python bench.py > gpurun_out/bench_r04b.json 2> gpurun_out/bench_r04b.err
cat gpurun_out/bench_r04b.json
bash tools/gpu_kstats.sh r04b
