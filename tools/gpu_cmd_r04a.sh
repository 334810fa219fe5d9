#!/bin/bash
# r04a: head validation: full GPU suite, smoke, default bench line, rocprof kernel stats.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
git_head=$(cat .head_sha 2>/dev/null || echo unknown)
echo "head $git_head" > gpurun_out/head.txt
bash tools/gpu_tests.sh
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_r04a.json 2> gpurun_out/bench_r04a.err
cat gpurun_out/bench_r04a.json
bash tools/gpu_kstats.sh r04a
