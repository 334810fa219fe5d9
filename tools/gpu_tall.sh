#!/bin/bash
# fp32 Reinsch tall tasks: per-call RMS (first N C5 calls) with the default library and a variant, then the C5 A/B.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in default ${VARIANTS}; do
  if [ "$v" = default ]; then unset SG_HIP_LIB; else export SG_HIP_LIB=$R/soundgen_beta_amd/lib/exp_$v.so; fi
  timeout -k 10 400 python tools/c5_rms.py ${NCALLS:-200} > gpurun_out/rms_$v.log 2>&1 || { tail -20 gpurun_out/rms_$v.log; exit 1; }
  echo "== $v"; tail -13 gpurun_out/rms_$v.log
done
unset SG_HIP_LIB
NOTEST=1 CFGS="${CFGS:-c5}" STEPS=${STEPS:-4} bash tools/gpu_ab.sh ${TAG:-tall}
