#!/bin/bash
# r04f: sine-bank parity subset at the new default (fast epilogue), then A/B:
# epi0 (per-lane epilogue), persist7 / persist14 (persistent long-task waves) on C2 and C5
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "c2_tones or planner_cases or c4_calls or every_preset or shard or amp_build or harmonics" > gpurun_out/pytest_r04f.log 2>&1 || { tail -30 gpurun_out/pytest_r04f.log; exit 1; }
tail -2 gpurun_out/pytest_r04f.log
NOTEST=1 VARIANTS="epi0 persist7 persist14" CFGS="c2" STEPS=30 BENCH_ARGS="--rms-calls 16" bash tools/gpu_ab.sh r04f
VARIANTS="epi0 persist7 persist14" KERNELS="sg_sine_bank sg_sine_bank_pairs sg_sine_bank_tall sg_sine_bank_tall_pairs sg_sine_bank_hp" bash tools/gpu_kstat_ab.sh r04f_kab
