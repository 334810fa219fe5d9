#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, no tracing domains) over a short bench run.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp
export TMPDIR=/tmp
TAG=${1:-pmc}
shift || true
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/${TAG}_$i" -o run -- python "$R/bench.py" --config ${CFG:-c2} --steps 3 --warmup 1 --device-steps 0 --no-cpu-baseline $BENCH_ARGS > "$R/gpurun_out/${TAG}_$i.log" 2>&1 || { tail -20 "$R/gpurun_out/${TAG}_$i.log"; exit 1; }
done
