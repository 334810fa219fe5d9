#!/bin/bash
# r04i: wavetable kernel granularity on C2: threads per workgroup (library
# variants thr256 / thr1024) and tasks per workgroup (SG_TAB_TASKS), kernel stats
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
run() {  # tag lib env...
  local tag=$1 lib=$2; shift 2
  if [ "$lib" = default ]; then unset SG_HIP_LIB; else export SG_HIP_LIB=$R/soundgen_beta_amd/lib/exp_$lib.so; fi
  env "$@" SG_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r04i_$tag" -o run -- python "$R/bench.py" --config c2 --steps 3 --warmup 1 --device-steps 0 --no-d2h --no-cpu-baseline --rms-calls 0 > "$R/gpurun_out/r04i_$tag.log" 2>&1 || { tail -20 "$R/gpurun_out/r04i_$tag.log"; exit 1; }
  echo "$tag $(grep '^"sg_sine_bank_tab"' "$R/gpurun_out/r04i_$tag/run_kernel_stats.csv" | cut -d, -f1-4)"
}
run default default SG_TAB_TASKS=64
run t32 default SG_TAB_TASKS=32
run t16 default SG_TAB_TASKS=16
run t8 default SG_TAB_TASKS=8
run thr256 thr256 SG_TAB_TASKS=64
run thr256_t16 thr256 SG_TAB_TASKS=16
run thr1024 thr1024 SG_TAB_TASKS=64
