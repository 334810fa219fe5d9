#!/bin/bash
# HBM traffic per launch (MI355X guide, HBM/rocprofv3 section; 7 executes per pass:
# warmup 1 + 3 timed + 3 profiled steps): FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes (they do not fit one TCC group), no tracing
# domains; summarised by tools/pmc_summary.py.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp
export TMPDIR=/tmp
TAG=${1:-traffic}
CFG=${CFG:-c2}
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  SG_OVERLAP=0 timeout -s KILL ${PMC_TIMEOUT:-150} rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/${TAG}_$i" -o run -- python "$R/bench.py" --config $CFG --steps 3 --warmup 1 --device-steps 0 --no-cpu-baseline $BENCH_ARGS > "$R/gpurun_out/${TAG}_$i.log" 2>&1 || { tail -20 "$R/gpurun_out/${TAG}_$i.log"; exit 1; }
done
cd "$R"
python tools/pmc_summary.py $TAG $CFG 7 > gpurun_out/${TAG}_summary.json
cat gpurun_out/${TAG}_summary.json
