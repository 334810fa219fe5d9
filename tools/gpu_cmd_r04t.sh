#!/bin/bash
# r04t: D2H into pinned host memory: the bandwidth bound of the host-resident headline,
# default runtime copy path vs SDMA forced on / off, 1-4 streams (tools/d2h_probe.py)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 180 python tools/d2h_probe.py > gpurun_out/r04t_default.json 2>&1 || { tail -5 gpurun_out/r04t_default.json; exit 1; }
echo "default $(tail -1 gpurun_out/r04t_default.json)"
HSA_ENABLE_SDMA=1 timeout -k 10 180 python tools/d2h_probe.py > gpurun_out/r04t_sdma1.json 2>&1 || { tail -5 gpurun_out/r04t_sdma1.json; exit 1; }
echo "sdma1 $(tail -1 gpurun_out/r04t_sdma1.json)"
HSA_ENABLE_SDMA=0 timeout -k 10 180 python tools/d2h_probe.py > gpurun_out/r04t_sdma0.json 2>&1 || { tail -5 gpurun_out/r04t_sdma0.json; exit 1; }
echo "sdma0 $(tail -1 gpurun_out/r04t_sdma0.json)"
