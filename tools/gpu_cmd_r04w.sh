#!/bin/bash
# r04w: C3 / C4 / C2 bench lines at the round-4 head (host- and device-resident, RMS check)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for cfg in c3 c4 c2; do
  timeout -k 10 400 python bench.py --config $cfg --steps 10 --warmup 2 --device-steps 10 --no-cpu-baseline --rms-calls 64 > gpurun_out/r04w_$cfg.json 2> gpurun_out/r04w_$cfg.err || { tail -20 gpurun_out/r04w_$cfg.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], '%.4g samples/s' % d['value'], 'dev %.4g' % d['value_device_resident'], '%.3f ms/step dev %.3f' % (d['ms_per_step'], d['ms_per_step_device_resident']), r['kernel'][:30], '%.3f ms' % r['avg_launch_ms'], 'frac %.3f' % r['frac'], 'rms %.2g/%d' % (d['rms_error_vs_oracle'], d['rms_check']['calls']))" gpurun_out/r04w_$cfg.json $cfg
done
