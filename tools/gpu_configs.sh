#!/bin/bash
# Bench + rocprofv3 kernel stats for the C3 / C4 configs.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
for cfg in ${CFGS:-c3 c4}; do
  timeout -k 10 500 python bench.py --config $cfg --steps 5 --warmup 2 --cpu-budget 10 > gpurun_out/bench_${cfg}_$TAG.json 2> gpurun_out/bench_${cfg}_$TAG.err || { tail -20 gpurun_out/bench_${cfg}_$TAG.err; exit 1; }
  cat gpurun_out/bench_${cfg}_$TAG.json
  cd /tmp
  SG_OVERLAP=0 timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${cfg}_$TAG" -o run -- python "$R/bench.py" --config $cfg --steps 3 --warmup 1 --device-steps 0 --no-cpu-baseline > "$R/gpurun_out/prof_${cfg}_$TAG.log" 2>&1 || { tail -20 "$R/gpurun_out/prof_${cfg}_$TAG.log"; exit 1; }
  cd "$R"
  cat gpurun_out/prof_${cfg}_$TAG/run_kernel_stats.csv | cut -d, -f1-5
done
