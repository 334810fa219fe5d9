#!/bin/bash
# r04zb: head PMC passes after the noise threshold (C5) (no tracing domains, each pass its own run): C5 and C2 SQ issue
# counters (two passes each) and HBM traffic (FETCH_SIZE, WRITE_SIZE passes each)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"
G2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_ANY"
for cfg in c5; do
  cd /tmp
  i=0
  for grp in "$G1" "$G2"; do
    i=$((i+1))
    SG_OVERLAP=0 timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/r04zb_${cfg}sq_$i" -o run -- python3 "$R/bench.py" --config $cfg --steps 3 --warmup 1 --device-steps 0 --no-d2h --no-cpu-baseline --rms-calls 0 > "$R/gpurun_out/r04zb_${cfg}sq_$i.log" 2>&1 || { tail -20 "$R/gpurun_out/r04zb_${cfg}sq_$i.log"; exit 1; }
  done
  cd "$R"
  python tools/pmc_summary.py r04zb_${cfg}sq $cfg 7 > gpurun_out/r04zb_${cfg}_pmc.json
  CFG=$cfg PMC_TIMEOUT=240 BENCH_ARGS="--no-d2h --rms-calls 0" bash tools/gpu_traffic.sh r04zb_${cfg}tr > /dev/null
  cp gpurun_out/r04zb_${cfg}tr_summary.json gpurun_out/r04zb_${cfg}_traffic.json
done
ls gpurun_out | grep r04zb_
