#!/bin/bash
# r04p: checkpoint after the wavetable work: full GPU suite + smoke, default C5 bench
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
git_head=$(cat .head_sha 2>/dev/null || echo unknown)
echo "head $git_head" > gpurun_out/head.txt
bash tools/gpu_tests.sh
timeout -k 10 600 python bench.py > gpurun_out/bench_r04p.json 2> gpurun_out/bench_r04p.err || { tail -20 gpurun_out/bench_r04p.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('%.4g samples/s' % d['value'], 'dev %.4g' % d['value_device_resident'], '%.2f ms/step' % d['ms_per_step'], 'rms %.2g over %d' % (d['rms_error_vs_oracle'], d['rms_check']['calls']))" gpurun_out/bench_r04p.json
