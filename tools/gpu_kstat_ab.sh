#!/bin/bash
# Per-kernel A/B of library variants: rocprofv3 kernel stats over device-resident
# C5 steps for the default library and each VARIANTS entry (tools/build_variant.sh);
# prints the KERNELS rows of each.   VARIANTS="a b" KERNELS="sg_fft_frames64" bash tools/gpu_kstat_ab.sh tag
set -e
R=$(pwd)
TAG=${1:-kab}
cd /tmp
for v in default ${VARIANTS}; do
  if [ "$v" = default ]; then unset SG_HIP_LIB; else export SG_HIP_LIB=$R/soundgen_beta_amd/lib/exp_$v.so; fi
  SG_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_$v" -o run -- python "$R/bench.py" --config ${CFG:-c5} --steps 2 --warmup 1 --device-steps 0 --no-d2h --no-cpu-baseline > "$R/gpurun_out/${TAG}_$v.log" 2>&1 || { tail -20 "$R/gpurun_out/${TAG}_$v.log"; exit 1; }
  for k in ${KERNELS:-sg_stft_ola}; do
    echo "$v $(grep "^\"$k\"," "$R/gpurun_out/${TAG}_$v/run_kernel_stats.csv" | cut -d, -f1-4)"
  done
done
