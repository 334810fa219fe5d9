#!/bin/bash
# r04e: head profiles: C2 kernel stats + SQ pass; C5 SQ pass; C5 HBM traffic (FETCH / WRITE passes)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SALU"
bash tools/gpu_kstats.sh r04e_c2 --config c2
cd /tmp
export TMPDIR=/tmp
for cfg in c2 c5; do
  SG_OVERLAP=0 timeout -s KILL 200 rocprofv3 --pmc $SQ --output-format csv -d "$R/gpurun_out/r04e_${cfg}sq_1" -o run -- python3 "$R/bench.py" --config $cfg --steps 3 --warmup 1 --device-steps 0 --no-d2h --no-cpu-baseline --rms-calls 0 > "$R/gpurun_out/r04e_${cfg}sq_1.log" 2>&1 || { tail -20 "$R/gpurun_out/r04e_${cfg}sq_1.log"; exit 1; }
done
cd "$R"
python tools/pmc_summary.py r04e_c2sq c2 7 > gpurun_out/r04e_c2_pmc.json
python tools/pmc_summary.py r04e_c5sq c5 7 > gpurun_out/r04e_c5_pmc.json
CFG=c5 PMC_TIMEOUT=200 BENCH_ARGS="--no-d2h --rms-calls 0" bash tools/gpu_traffic.sh r04e_c5tr > /dev/null
ls gpurun_out
