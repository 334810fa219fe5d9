#!/bin/bash
# r04final: the full GPU suite and smoke at the final round-4 head (kernels as validated in r04v2)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_tests.sh | tail -3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r04final.log 2>&1 || { tail -30 gpurun_out/smoke_r04final.log; exit 1; }
tail -1 gpurun_out/smoke_r04final.log
