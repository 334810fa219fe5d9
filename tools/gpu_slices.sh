#!/bin/bash
# C2 step time vs the number of batch slices (sine bank of slice c+1 on the
# launch stream overlapping the finalize of slice c on the aux stream).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for k in ${SLICES:-1 2 4 8}; do
  SG_SLICES=$k timeout -k 10 300 python bench.py --config ${CFG:-c2} --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/slices_$k.json 2> gpurun_out/slices_$k.err || { tail -20 gpurun_out/slices_$k.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('slices', sys.argv[2], '%.3g samples/s' % d['value'], '%.3f ms/step' % d['ms_per_step'], '%.1f us sine' % (r['avg_launch_ms']*1e3), 'rms %.2g' % d['rms_error_vs_oracle'])" gpurun_out/slices_$k.json $k
done
