#!/bin/bash
# r04z: round-4 validation at head: the full GPU suite, smoke, the default bench line,
# C5 kernel stats (SG_OVERLAP=0) -- then (r04z2) the head PMC passes
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "head $(cat .head_sha 2>/dev/null || echo unknown)" > gpurun_out/head.txt
bash tools/gpu_tests.sh
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r04z.log 2>&1 || { tail -30 gpurun_out/smoke_r04z.log; exit 1; }
tail -1 gpurun_out/smoke_r04z.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r04z.json 2> gpurun_out/bench_r04z.err || { tail -20 gpurun_out/bench_r04z.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('%.4g samples/s' % d['value'], 'dev %.4g' % d['value_device_resident'], '%.2f ms/step' % d['ms_per_step'], 'rms %.2g over %d' % (d['rms_error_vs_oracle'], d['rms_check']['calls']), 'frac %.3f' % d['roofline']['frac'])" gpurun_out/bench_r04z.json
bash tools/gpu_kstats.sh r04z_c5 > /dev/null
bash tools/gpu_kstats.sh r04z_c2 --config c2 > /dev/null
ls gpurun_out/r04z_c5_ks gpurun_out/r04z_c2_ks
