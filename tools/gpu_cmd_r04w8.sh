#!/bin/bash
# r04w8: validation at the head with sg_harm_finalize at 8 waves: the full GPU suite,
# smoke, the default bench line, C5 and C3 kernel stats, C3 bench
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "head $(cat .head_sha 2>/dev/null || echo unknown)" > gpurun_out/head.txt
bash tools/gpu_tests.sh
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r04w8.log 2>&1 || { tail -30 gpurun_out/smoke_r04w8.log; exit 1; }
tail -1 gpurun_out/smoke_r04w8.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r04w8.json 2> gpurun_out/bench_r04w8.err || { tail -20 gpurun_out/bench_r04w8.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('%.4g samples/s' % d['value'], 'dev %.4g' % d['value_device_resident'], '%.2f ms/step dev %.2f' % (d['ms_per_step'], d['ms_per_step_device_resident']), 'rms %.2g over %d' % (d['rms_error_vs_oracle'], d['rms_check']['calls']), 'frac %.3f' % d['roofline']['frac'])" gpurun_out/bench_r04w8.json
timeout -k 10 400 python bench.py --config c3 --steps 10 --warmup 2 --device-steps 10 --no-cpu-baseline --rms-calls 64 > gpurun_out/r04w8_c3.json 2> gpurun_out/r04w8_c3.err || { tail -20 gpurun_out/r04w8_c3.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('c3 %.4g samples/s' % d['value'], 'dev %.4g' % d['value_device_resident'], '%.3f ms/step dev %.3f' % (d['ms_per_step'], d['ms_per_step_device_resident']), 'rms %.2g/%d' % (d['rms_error_vs_oracle'], d['rms_check']['calls']))" gpurun_out/r04w8_c3.json
bash tools/gpu_kstats.sh r04w8_c5 > /dev/null
ls gpurun_out/r04w8_c5_ks
cd "$R"
CFG=c5 VARIANTS="sb8 tall6 hp6" KERNELS="sg_sine_bank sg_sine_bank_tall sg_sine_bank_hp" bash tools/gpu_kstat_ab.sh r04occ
cd "$R"
for v in default sb8 tall6 hp6; do echo "$v $(grep -o '"rms_error_vs_oracle": [0-9.e-]*' gpurun_out/r04occ_$v.log)"; done
