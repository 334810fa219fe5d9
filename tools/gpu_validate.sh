#!/bin/bash
# Validation of a head on the GPU box (one gpurun call):
#   gpurun --timeout 1200 -- 'bash tools/gpu_validate.sh r05a'
# the full GPU suite, smoke, the default bench line (C5, host- and device-resident, RMS vs the
# oracle), a C3 bench line and C5 per-kernel stats; outputs under gpurun_out/ named by the tag.
# Per-kernel A/Bs of build variants: tools/gpu_kstat_ab.sh (with tools/build_variant.sh).
# Write `git rev-parse HEAD > .head_sha` before the call so the log names the tree it ran.
set -e
TAG=${1:-val}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "head $(cat .head_sha 2>/dev/null || echo unknown)" > gpurun_out/head_$TAG.txt
bash tools/gpu_tests.sh | tail -3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -30 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('%.4g samples/s' % d['value'], 'dev %.4g' % d['value_device_resident'], '%.2f ms/step dev %.2f' % (d['ms_per_step'], d['ms_per_step_device_resident']), 'rms %.2g over %d' % (d['rms_error_vs_oracle'], d['rms_check']['calls']), 'frac %.3f' % d['roofline']['frac'])" gpurun_out/bench_$TAG.json
timeout -k 10 400 python bench.py --config c3 --steps 10 --warmup 2 --device-steps 10 --no-cpu-baseline --rms-calls 64 > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err || { tail -20 gpurun_out/${TAG}_c3.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('c3 %.4g samples/s' % d['value'], 'dev %.4g' % d['value_device_resident'], '%.3f ms/step dev %.3f' % (d['ms_per_step'], d['ms_per_step_device_resident']), 'rms %.2g/%d' % (d['rms_error_vs_oracle'], d['rms_check']['calls']))" gpurun_out/${TAG}_c3.json
timeout -k 10 400 python bench.py --node --steps 5 --warmup 2 --rms-calls 32 > gpurun_out/${TAG}_node.json 2> gpurun_out/${TAG}_node.err || { tail -20 gpurun_out/${TAG}_node.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('node %.4g samples/s' % d['value'], '%.2f ms/step' % d['ms_per_step'], 'plan %.2f s' % d['plan_s'], 'rms %.2g/%d' % (d['rms_error_vs_oracle'], d['rms_check']['calls']))" gpurun_out/${TAG}_node.json
bash tools/gpu_kstats.sh ${TAG}_c5 > /dev/null
ls gpurun_out/${TAG}_c5_ks
