#!/bin/bash
# r03l: spectral GPU tests on the packed untangle, stft A/B on C5 and C3, stamps
set -e
R=$(pwd)
PYTEST_K="spectral or c5 or c3 or noise or gathered" bash tools/gpu_tests.sh
NOTEST=1 CFGS="c5 c3" VARIANTS="prev cp13" STEPS=8 bash tools/gpu_ab.sh stft3
SG_HIP_LIB=$R/soundgen_beta_amd/lib/exp_stamps.so timeout -k 10 300 python tools/stft_stamps.py c5 16384 > gpurun_out/stamps_r03l.json 2> gpurun_out/stamps_r03l.err
cat gpurun_out/stamps_r03l.json
