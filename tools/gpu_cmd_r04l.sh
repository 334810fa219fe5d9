#!/bin/bash
# r04l: C2 with tables capped at N = 1024 (SG_TAB_LOGN=10: one launch with 4 workgroups per
# CU resident; the 2048-point spans on the recurrence) vs the default, kernel stats + bench
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
for t in 11; do
  SG_TAB_LOGN=$t SG_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r04l_$t" -o run -- python "$R/bench.py" --config c2 --steps 3 --warmup 1 --device-steps 0 --no-d2h --no-cpu-baseline --rms-calls 0 > "$R/gpurun_out/r04l_$t.log" 2>&1 || { tail -20 "$R/gpurun_out/r04l_$t.log"; exit 1; }
  echo "== logn $t"; grep -E '^"sg_sine_bank' "$R/gpurun_out/r04l_$t/run_kernel_stats.csv" | cut -d, -f1-4
  SG_TAB_LOGN=$t timeout -k 10 300 python "$R/bench.py" --config c2 --steps 30 --warmup 3 --device-steps 0 --no-cpu-baseline --rms-calls 64 > "$R/gpurun_out/r04l_c2_$t.json" 2> "$R/gpurun_out/r04l_c2_$t.err" || { tail -20 "$R/gpurun_out/r04l_c2_$t.err"; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('%.4g samples/s' % d['value'], '%.4f ms/step' % d['ms_per_step'], '%.1f us' % (r['avg_launch_ms']*1e3), 'frac %.3f' % r['frac'], 'rms %.2g' % d['rms_error_vs_oracle'])" "$R/gpurun_out/r04l_c2_$t.json"
done
