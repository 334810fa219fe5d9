#!/bin/bash
# Planning-time A/B (HEAD-of-round library vs the tree's) on C5 plans, then the default bench line.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-pab}
for i in 1 2; do
  for v in ${VARIANTS:-head} default; do
    if [ "$v" = default ]; then L=""; else L=$R/soundgen_beta_amd/lib/exp_$v.so; fi
    env ${L:+SG_HIP_LIB=$L} timeout -k 10 300 python tools/plan_ab.py ${NCALLS:-16384} >> gpurun_out/plan_ab_$TAG.log 2>&1 || { tail -20 gpurun_out/plan_ab_$TAG.log; exit 1; }
    tail -1 gpurun_out/plan_ab_$TAG.log
  done
done
if [ -n "$BENCH" ]; then
  timeout -k 10 500 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
  cat gpurun_out/bench_$TAG.json
fi
