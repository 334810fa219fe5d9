#!/bin/bash
# r04u: the C5 headline (host-resident) with the runtime's copy engine choice forced:
# default vs HSA_ENABLE_SDMA=1 vs 0
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for e in default 1 0; do
  if [ "$e" = default ]; then unset HSA_ENABLE_SDMA; else export HSA_ENABLE_SDMA=$e; fi
  timeout -k 10 400 python bench.py --steps 8 --warmup 2 --device-steps 0 --no-cpu-baseline --rms-calls 0 > gpurun_out/r04u_$e.json 2> gpurun_out/r04u_$e.err || { tail -20 gpurun_out/r04u_$e.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.4g samples/s' % d['value'], '%.2f ms/step' % d['ms_per_step'])" gpurun_out/r04u_$e.json $e
done
