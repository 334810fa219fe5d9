#!/bin/bash
# rocprofv3 kernel stats of short bench runs, one per config: CFGS="c3 c4" tools/gpu_prof.sh tag
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp
export TMPDIR=/tmp
TAG=${1:-prof}
for cfg in ${CFGS:-c2}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_$cfg" -o run -- python "$R/bench.py" --config $cfg --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline > "$R/gpurun_out/${TAG}_$cfg.log" 2>&1 || { tail -20 "$R/gpurun_out/${TAG}_$cfg.log"; exit 1; }
  echo "== $cfg"; cut -d, -f1-4 "$R/gpurun_out/${TAG}_$cfg/run_kernel_stats.csv" | grep -v "at::native" | head -14
done
