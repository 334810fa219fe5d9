#!/bin/bash
# r03m: stft A/B of the prefetch placement on C5 and C3, stamps of pf4
set -e
R=$(pwd)
NOTEST=1 CFGS="c5 c3" VARIANTS="pf3 pf4" STEPS=8 bash tools/gpu_ab.sh stft4
SG_HIP_LIB=$R/soundgen_beta_amd/lib/exp_pf4s.so timeout -k 10 300 python tools/stft_stamps.py c5 16384 > gpurun_out/stamps_r03m.json 2> gpurun_out/stamps_r03m.err
cat gpurun_out/stamps_r03m.json
