#!/bin/bash
# rocprofv3 kernel stats of the default library and variants (tools/build_variant.sh)
# on one bench config: VARIANTS="a b" CFG=c5 BENCH_ARGS="--calls 8192" tools/gpu_ab_prof.sh tag
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-abp}
mkdir -p "$R/gpurun_out"
cd /tmp
export TMPDIR=/tmp
for v in default ${VARIANTS}; do
  if [ "$v" = default ]; then unset SG_HIP_LIB; else export SG_HIP_LIB=$R/soundgen_beta_amd/lib/exp_$v.so; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_$v" -o run -- python "$R/bench.py" --config ${CFG:-c5} --steps ${STEPS:-3} --warmup 1 --device-steps 0 --no-cpu-baseline $BENCH_ARGS > "$R/gpurun_out/${TAG}_$v.log" 2>&1 || { tail -20 "$R/gpurun_out/${TAG}_$v.log"; exit 1; }
  echo "== $v"; cut -d, -f1-4 "$R/gpurun_out/${TAG}_$v/run_kernel_stats.csv" | grep -v "at::native" | head -12
done
