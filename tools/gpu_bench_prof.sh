#!/bin/bash
# Default bench line, then a rocprofv3 kernel-stats pass over device-resident C5 steps.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-bp}
timeout -k 10 500 python bench.py $BENCH_ARGS > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
cd /tmp
SG_OVERLAP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- python "$R/bench.py" --config ${CFG:-c5} --steps 4 --warmup 1 --device-steps 0 --no-cpu-baseline > "$R/gpurun_out/prof_$TAG.log" 2>&1 || { tail -30 "$R/gpurun_out/prof_$TAG.log"; exit 1; }
cut -d, -f1-5 "$R/gpurun_out/prof_$TAG/run_kernel_stats.csv" | head -14
