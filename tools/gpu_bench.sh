#!/bin/bash
# The default bench (C5, 65,536 calls on one GPU) + GPU tests matching $PYTEST_K.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-r02}
if [ -n "$PYTEST_K" ]; then bash tools/gpu_tests.sh; fi
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py $BENCH_ARGS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
