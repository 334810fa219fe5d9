#!/bin/bash
# Sweep of library variants x env settings on one config (after the GPU parity
# tests of the default library):  RUNS="default: ns4: default:SG_TASK_MAX=1024"
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${1:-sw}
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
  tail -1 gpurun_out/pytest_$TAG.log
fi
i=0
for run in ${RUNS:-default:}; do
  i=$((i+1))
  v=${run%%:*}; envs=${run#*:}
  if [ "$v" = default ]; then L=""; else L=$R/soundgen_beta_amd/lib/exp_$v.so; fi
  env ${L:+SG_HIP_LIB=$L} ${envs//,/ } timeout -k 10 300 python bench.py --config ${CFG:-c2} --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline > gpurun_out/sw_${TAG}_$i.json 2> gpurun_out/sw_${TAG}_$i.err || { tail -20 gpurun_out/sw_${TAG}_$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], '%.3g samples/s' % d['value'], '%.3f ms/step' % d['ms_per_step'], r['kernel'], '%.1f us' % (r['avg_launch_ms']*1e3), 'frac %.3f' % r['frac'], 'rms %.2g' % d['rms_error_vs_oracle'])" gpurun_out/sw_${TAG}_$i.json "$run"
done
