#!/bin/bash
# r03j: default bench line (new marshalling), stft A/B (13 carry pairs), kernel stats of the head
set -e
timeout -k 10 400 python bench.py > gpurun_out/bench_r03j.json 2> gpurun_out/bench_r03j.err
cat gpurun_out/bench_r03j.json
NOTEST=1 CFGS=c5 VARIANTS="cp13 cp13h" STEPS=8 bash tools/gpu_ab.sh stft2
R=$(pwd)
cd /tmp
SG_OVERLAP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_r03j" -o run -- python "$R/bench.py" --steps 4 --warmup 1 --device-steps 0 --no-cpu-baseline > "$R/gpurun_out/prof_r03j.log" 2>&1
cut -d, -f1-5 "$R/gpurun_out/prof_r03j/run_kernel_stats.csv" | head -14
