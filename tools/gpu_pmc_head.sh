#!/bin/bash
# PMC passes for bench.py's `issue` and `traffic` fields at a head:
#   gpurun -- 'bash tools/gpu_pmc_head.sh TAG [CFG]'   (CFG default c5)
# two SQ issue-counter passes and the FETCH_SIZE / WRITE_SIZE passes, each its own rocprofv3 run
# with no tracing domains; writes gpurun_out/TAG_CFG_pmc.json and TAG_CFG_traffic.json, which
# go to profiles/ (bench.py reads the newest by name).
set -e
TAG=${1:?tag}
CFG=${2:-c5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
# SQ_WAVE_CYCLES and SQ_BUSY_CU_CYCLES in both passes: achieved waves per SIMD is their ratio (bench.py
# pmc_from_profiles), and each pass's issue shares are taken against its own wave cycles
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
G2="SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU"
# LDS: conflict cycles against LDS instructions and against the LDS array's busy cycles
G3="SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"
cd /tmp
i=0
for grp in "$G1" "$G2" "$G3"; do
  i=$((i+1))
  SG_OVERLAP=0 timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/${TAG}_${CFG}sq_$i" -o run -- python3 "$R/bench.py" --config $CFG --steps 3 --warmup 1 --device-steps 0 --no-d2h --no-cpu-baseline --rms-calls 0 > "$R/gpurun_out/${TAG}_${CFG}sq_$i.log" 2>&1 || { tail -20 "$R/gpurun_out/${TAG}_${CFG}sq_$i.log"; exit 1; }
done
cd "$R"
python tools/pmc_summary.py ${TAG}_${CFG}sq $CFG 7 > gpurun_out/${TAG}_${CFG}_pmc.json
CFG=$CFG PMC_TIMEOUT=240 BENCH_ARGS="--no-d2h --rms-calls 0" bash tools/gpu_traffic.sh ${TAG}_${CFG}tr > /dev/null
cp gpurun_out/${TAG}_${CFG}tr_summary.json gpurun_out/${TAG}_${CFG}_traffic.json
ls gpurun_out | grep "^${TAG}_${CFG}_"
