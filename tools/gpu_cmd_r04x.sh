#!/bin/bash
# r04x: measured threshold for the fp64 noise path (tools/noise_selector_study.py)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 900 python tools/noise_selector_study.py gpurun_out/r04x_noise_selector_study.json 256 4096 > gpurun_out/r04x.log 2>&1 || { tail -20 gpurun_out/r04x.log; exit 1; }
cat gpurun_out/r04x.log | tail -14
