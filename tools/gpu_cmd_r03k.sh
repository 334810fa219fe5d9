#!/bin/bash
# r03k: GPU suite, smoke, default bench line, kernel stats of device-resident steps, C5 stft section stamps
set -e
R=$(pwd)
bash tools/gpu_tests.sh
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_r03k.json 2> gpurun_out/bench_r03k.err
cat gpurun_out/bench_r03k.json
cd /tmp
SG_OVERLAP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_r03k" -o run -- python "$R/bench.py" --steps 4 --warmup 1 --device-steps 0 --no-d2h --no-cpu-baseline > "$R/gpurun_out/prof_r03k.log" 2>&1
cut -d, -f1-5 "$R/gpurun_out/prof_r03k/run_kernel_stats.csv" | head -16
cd "$R"
SG_HIP_LIB=$R/soundgen_beta_amd/lib/exp_stamps.so timeout -k 10 300 python tools/stft_stamps.py c5 16384 > gpurun_out/stamps_r03k.json 2> gpurun_out/stamps_r03k.err
cat gpurun_out/stamps_r03k.json
