#!/bin/bash
# r04c: full GPU suite at the SG_FAMP default, then A/B of the two-chain sine bank (exp_famp0)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
bash tools/gpu_tests.sh
NOTEST=1 VARIANTS="famp0" CFGS="c2 c5" STEPS=10 bash tools/gpu_ab.sh r04c
VARIANTS="famp0" KERNELS="sg_sine_bank sg_sine_bank_pairs sg_sine_bank_tall sg_sine_bank_tall_pairs sg_sine_bank_hp" bash tools/gpu_kstat_ab.sh r04c_kab
