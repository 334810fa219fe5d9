#!/bin/bash
# r03o: D2H probe, GPU suite, smoke, default bench line, kernel stats (device-resident steps),
# fp64 grouped-stage variant: its GPU tests, then a per-kernel A/B
set -e
R=$(pwd)
timeout -k 10 120 python tools/d2h_probe.py > gpurun_out/d2h_r03o.json 2>&1 && cat gpurun_out/d2h_r03o.json
bash tools/gpu_tests.sh
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_r03o.json 2> gpurun_out/bench_r03o.err
cat gpurun_out/bench_r03o.json
SG_HIP_LIB=$R/soundgen_beta_amd/lib/exp_kg3.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "every_preset or c4_calls or fp64 or noise" > gpurun_out/pytest_kg3.log 2>&1 || { tail -30 gpurun_out/pytest_kg3.log; exit 1; }
tail -2 gpurun_out/pytest_kg3.log
cd /tmp
SG_OVERLAP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_r03o" -o run -- python "$R/bench.py" --steps 4 --warmup 1 --device-steps 0 --no-d2h --no-cpu-baseline > "$R/gpurun_out/prof_r03o.log" 2>&1
cut -d, -f1-5 "$R/gpurun_out/prof_r03o/run_kernel_stats.csv" | head -16
cd "$R"
VARIANTS="kg3 kg2" KERNELS="sg_fft_frames64 sg_stft_ola" bash tools/gpu_kstat_ab.sh kab_r03o
