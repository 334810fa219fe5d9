#!/bin/bash
# A/B of library variants (tools/build_variant.sh) on bench configs, after the
# GPU parity tests of the default library. VARIANTS="old wpe5" CFGS="c2 c4"
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ab}
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
  tail -2 gpurun_out/pytest_$TAG.log
fi
for cfg in ${CFGS:-c2}; do
  for v in default ${VARIANTS}; do
    if [ "$v" = default ]; then unset SG_HIP_LIB; else export SG_HIP_LIB=$R/soundgen_beta_amd/lib/exp_$v.so; fi
    timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-20} --warmup 3 --device-steps 0 --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab_${TAG}_${cfg}_$v.json 2> gpurun_out/ab_${TAG}_${cfg}_$v.err || { tail -20 gpurun_out/ab_${TAG}_${cfg}_$v.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], sys.argv[3], '%.3g samples/s' % d['value'], '%.3f ms/step' % d['ms_per_step'], r['kernel'], '%.1f us' % (r['avg_launch_ms']*1e3), 'frac %.3f' % r['frac'], 'rms %.2g' % d['rms_error_vs_oracle'])" gpurun_out/ab_${TAG}_${cfg}_$v.json $cfg $v
  done
done
