#!/bin/bash
# GPU parity tests only (each test under its own 300 s limit; the run stops at the first failure).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
grep -E "PASSED|FAILED|SKIPPED|passed|failed" gpurun_out/pytest_gpu.log | tail -60
