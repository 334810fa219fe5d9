#!/bin/bash
# r04r: direct table jobs with the candidate-sample max: parity subset (direct == W path
# bit for bit, table vs recurrence vs oracle), C2 bench, C2 kernel stats default vs cand0
# (full max pass)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -s -k "sine_table or c2_tones or c2_full or planner_cases or harmonics or ampl_anchors or edge" > gpurun_out/pytest_r04r.log 2>&1 || { tail -25 gpurun_out/pytest_r04r.log; exit 1; }
tail -1 gpurun_out/pytest_r04r.log
timeout -k 10 300 python bench.py --config c2 --steps 30 --warmup 3 --device-steps 0 --no-cpu-baseline --rms-calls 64 > gpurun_out/r04r_c2.json 2> gpurun_out/r04r_c2.err || { tail -20 gpurun_out/r04r_c2.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('%.4g samples/s' % d['value'], '%.4f ms/step' % d['ms_per_step'], '%.1f us' % (r['avg_launch_ms']*1e3), 'frac %.3f' % r['frac'], 'rms %.2g' % d['rms_error_vs_oracle'])" gpurun_out/r04r_c2.json
CFG=c2 VARIANTS="cand0" KERNELS="sg_sine_bank_tab sg_harm_copy sg_syl_max" bash tools/gpu_kstat_ab.sh r04r
