set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PYTEST_K="${PYTEST_K:-envelope or c5}" bash tools/gpu_tests.sh
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/p3 -o run -- python $GRAFT_REPO_ROOT/bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/p3.log 2>&1
cut -d, -f1-5 $GRAFT_REPO_ROOT/gpurun_out/p3/run_kernel_stats.csv | head -20
