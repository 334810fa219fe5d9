#!/bin/bash
# r04n2: the noise-threshold GPU test
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_precision_selector.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_r04n2.log 2>&1 || { tail -30 gpurun_out/pytest_r04n2.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_r04n2.log | tail -4
