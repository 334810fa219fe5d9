#!/bin/bash
# Instruction mix per kernel (SQ_INSTS_VALU_* by type, SALU, SMEM, LDS), two rocprofv3 --pmc
# passes (8 SQ counters each, no tracing domains) over device-resident steps of CFG:
#   gpurun -- 'bash tools/gpu_imix.sh TAG [CFG]'   -> gpurun_out/TAG_CFG_imix.json
# tools/imix_summary.py prints per-wave counts per kernel.
set -e
TAG=${1:?tag}
CFG=${2:-c5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F32"
G2="SQ_WAVES SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F64"
cd /tmp
i=0
for grp in "$G1" "$G2"; do
  i=$((i+1))
  SG_OVERLAP=0 timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/${TAG}_${CFG}im_$i" -o run -- python3 "$R/bench.py" --config $CFG --steps 1 --warmup 0 --device-steps 0 --no-d2h --no-cpu-baseline --rms-calls 0 > "$R/gpurun_out/${TAG}_${CFG}im_$i.log" 2>&1 || { tail -20 "$R/gpurun_out/${TAG}_${CFG}im_$i.log"; exit 1; }
done
cd "$R"
python3 tools/pmc_summary.py ${TAG}_${CFG}im $CFG > gpurun_out/${TAG}_${CFG}_imix.json
python3 tools/imix_summary.py gpurun_out/${TAG}_${CFG}_imix.json
