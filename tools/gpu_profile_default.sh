#!/bin/bash
# rocprofv3 kernel stats + HBM traffic PMC passes of the default bench workload.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02}
mkdir -p "$R/gpurun_out"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_ks" -o run -- python "$R/bench.py" --steps 3 --warmup 1 --device-steps 0 --no-cpu-baseline $BENCH_ARGS > "$R/gpurun_out/${TAG}_ks.log" 2>&1 || { tail -20 "$R/gpurun_out/${TAG}_ks.log"; exit 1; }
cut -d, -f1-5 "$R/gpurun_out/${TAG}_ks/run_kernel_stats.csv" | grep -v "at::native" | head -16
cd "$R"
PMC_TIMEOUT=400 CFG=${CFG:-c5} bash tools/gpu_traffic.sh ${TAG}_tr
