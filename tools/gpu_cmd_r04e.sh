#!/bin/bash
# r04e: head profiles: C2 kernel stats + SQ pass; C5 SQ pass; C5 HBM traffic (FETCH / WRITE passes)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
for tm in 1024 2048 4096 512; do
  SG_TASK_MAX=$tm timeout -k 10 200 python bench.py --config c2 --steps 20 --warmup 3 --device-steps 10 --no-cpu-baseline --rms-calls 16 > gpurun_out/r04e_c2_tm$tm.json 2> gpurun_out/r04e_c2_tm$tm.err || { tail -20 gpurun_out/r04e_c2_tm$tm.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('task_max', sys.argv[2], '%.3f ms/step dev %.3f' % (d['ms_per_step'], d['ms_per_step_device_resident']), '%.1f us' % (r['avg_launch_ms']*1e3), 'frac %.3f' % r['frac'], 'rms %.2g' % d['rms_error_vs_oracle'])" gpurun_out/r04e_c2_tm$tm.json $tm
done
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
