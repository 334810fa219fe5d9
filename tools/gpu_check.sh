#!/bin/bash
# GPU tests, smoke, then the driver's bench command (each under its own limit;
# the chain stops at the first failure). Usage: gpu_check.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03}
if [ -z "$SKIP_TESTS" ]; then bash tools/gpu_tests.sh; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -30 gpurun_out/smoke_$TAG.log; exit 1; }
t0=$SECONDS
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py --gpus 1 --steps 20 --warmup 5 $BENCH_ARGS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
echo "bench wall $((SECONDS - t0)) s"
tail -2 gpurun_out/bench_$TAG.err
cat gpurun_out/bench_$TAG.json
