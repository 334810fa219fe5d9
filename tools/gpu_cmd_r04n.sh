#!/bin/bash
# r04n: direct-output table jobs: parity subset, C2 bench (table on), kernel stats of the
# default and the build-only diagnostic (tab_d1)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -s -k "sine_table or c2_tones or c2_full or planner_cases or harmonics or ampl_anchors or edge or shard or api_plans" > gpurun_out/pytest_r04n.log 2>&1 || { grep -E "table rms" gpurun_out/pytest_r04n.log; tail -15 gpurun_out/pytest_r04n.log; exit 1; }
grep -E "table rms" gpurun_out/pytest_r04n.log; tail -1 gpurun_out/pytest_r04n.log
timeout -k 10 300 python bench.py --config c2 --steps 30 --warmup 3 --device-steps 0 --no-cpu-baseline --rms-calls 64 > gpurun_out/r04n_c2.json 2> gpurun_out/r04n_c2.err || { tail -20 gpurun_out/r04n_c2.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('%.4g samples/s' % d['value'], '%.4f ms/step' % d['ms_per_step'], '%.1f us' % (r['avg_launch_ms']*1e3), 'frac %.3f' % r['frac'], 'rms %.2g' % d['rms_error_vs_oracle'])" gpurun_out/r04n_c2.json
CFG=c2 VARIANTS="" KERNELS="sg_sine_bank_tab" bash tools/gpu_kstat_ab.sh r04n
