#!/bin/bash
# Parity tests (PYTEST_K) with the default library, then per-variant C5 kernel stats
# (rocprofv3 over device-resident steps of a reduced batch) and bench lines.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-abk}
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$PYTEST_K" > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
  tail -2 gpurun_out/pytest_$TAG.log
fi
for v in default ${VARIANTS}; do
  export SG_OVERLAP=${ABK_OVERLAP:-1}
  unset SG_EXEC_EACH
  case "$v" in
    default) unset SG_HIP_LIB ;;
    nooverlap) unset SG_HIP_LIB; export SG_OVERLAP=0 ;;
    each) unset SG_HIP_LIB; export SG_EXEC_EACH=1 ;;
    *) export SG_HIP_LIB=$R/soundgen_beta_amd/lib/exp_$v.so ;;
  esac
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/pk_${TAG}_$v" -o run -- python "$R/bench.py" --config c5 --calls ${CALLS:-16384} --steps 3 --warmup 1 --device-steps 0 --no-cpu-baseline > "$R/gpurun_out/pk_${TAG}_$v.log" 2>&1 || { tail -20 "$R/gpurun_out/pk_${TAG}_$v.log"; exit 1; }
  cd "$R"
  echo "== $v $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print('%.4g samples/s %.2f ms/step rms %.2g' % (d['value'], d['ms_per_step'], d['rms_error_vs_oracle']))" "$(ls gpurun_out/pk_${TAG}_$v.log)" 2>/dev/null || grep -o '"value": [0-9.e+]*' gpurun_out/pk_${TAG}_$v.log)"
  cut -d, -f1-4 "gpurun_out/pk_${TAG}_$v/run_kernel_stats.csv" | head -9 | tail -8
done
