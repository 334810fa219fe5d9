#!/bin/bash
# r03p: GPU suite, smoke, default bench line (head), D2H probe
set -e
bash tools/gpu_tests.sh
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_r03p.json 2> gpurun_out/bench_r03p.err
cat gpurun_out/bench_r03p.json
timeout -k 10 120 python tools/d2h_probe.py > gpurun_out/d2h_r03p.json 2>&1 && cat gpurun_out/d2h_r03p.json
