#!/bin/bash
# rocprofv3 kernel stats of the bench workload (no PMC), every kernel alone (SG_OVERLAP=0: the
# harmonic chain and the noise phase on one stream), so each launch's duration is its own and
# matches the bench's HIP-event roofline. Usage: gpu_kstats.sh TAG [bench args]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03}
shift || true
mkdir -p "$R/gpurun_out"
cd /tmp
export TMPDIR=/tmp
SG_OVERLAP=0 timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_ks" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --device-steps 0 --no-d2h --no-cpu-baseline "$@" > "$R/gpurun_out/${TAG}_ks.log" 2>&1 || { tail -20 "$R/gpurun_out/${TAG}_ks.log"; exit 1; }
cut -d, -f1-5 "$R/gpurun_out/${TAG}_ks/run_kernel_stats.csv" | grep -v "at::native" | head -24
