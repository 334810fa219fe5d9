#!/bin/bash
# r04g: wavetable path (sg_sine_bank_tab) parity, then C2 bench and C2 / C5 kernel
# stats with the table on (default) and off (SG_TABLE=0)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -s -k "sine_table or c2_tones or c2_full or planner_cases or ampl_anchors or harmonics or shard or amp_build" > gpurun_out/pytest_r04g.log 2>&1 || { grep -E "table rms" gpurun_out/pytest_r04g.log; tail -15 gpurun_out/pytest_r04g.log; exit 1; }
grep -E "table rms" gpurun_out/pytest_r04g.log; tail -2 gpurun_out/pytest_r04g.log
for t in 1 0; do
  SG_TABLE=$t timeout -k 10 300 python bench.py --config c2 --steps 30 --warmup 3 --device-steps 0 --no-cpu-baseline --rms-calls 64 > gpurun_out/r04g_c2_tab$t.json 2> gpurun_out/r04g_c2_tab$t.err || { tail -20 gpurun_out/r04g_c2_tab$t.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], '%.4g samples/s' % d['value'], '%.4f ms/step' % d['ms_per_step'], '%.1f us' % (r['avg_launch_ms']*1e3), 'frac %.3f' % r['frac'], 'rms %.2g' % d['rms_error_vs_oracle'])" gpurun_out/r04g_c2_tab$t.json tab$t
done
cd /tmp
for cfg in c2 c5; do
  for t in 1 0; do
    SG_TABLE=$t SG_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r04g_ks_${cfg}_$t" -o run -- python "$R/bench.py" --config $cfg --steps 3 --warmup 1 --device-steps 0 --no-d2h --no-cpu-baseline --rms-calls 0 > "$R/gpurun_out/r04g_ks_${cfg}_$t.log" 2>&1 || { tail -20 "$R/gpurun_out/r04g_ks_${cfg}_$t.log"; exit 1; }
    echo "== $cfg table=$t"; grep -E '^"sg_sine_bank' "$R/gpurun_out/r04g_ks_${cfg}_$t/run_kernel_stats.csv" | cut -d, -f1-4
  done
done
cd "$R"
CFG=c2 VARIANTS="tdiag1 tdiag2 tdiag3 tdiag4" KERNELS="sg_sine_bank_tab" bash tools/gpu_kstat_ab.sh r04g_diag
