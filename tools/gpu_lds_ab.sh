#!/bin/bash
# LDS counter pass per library variant (tools/build_variant.sh): SQ_LDS_BANK_CONFLICT
# (extra LDS-array cycles), SQ_LDS_IDX_ACTIVE (all LDS-array cycles), SQ_INSTS_LDS, over
# device-resident steps of CFG (default c5); prints per kernel conflicts per LDS
# instruction and the conflict share of the LDS-array cycles.
#   VARIANTS="r05" KERNELS="sg_stft_ola sg_stft_ola_noise" bash tools/gpu_lds_ab.sh TAG
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-lds}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
G="SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_LDS SQ_INSTS_VALU"
for v in default ${VARIANTS}; do
  if [ "$v" = default ]; then unset SG_HIP_LIB; else export SG_HIP_LIB=$R/soundgen_beta_amd/lib/exp_$v.so; fi
  SG_OVERLAP=0 timeout -s KILL 240 rocprofv3 --pmc $G --output-format csv -d "$R/gpurun_out/${TAG}_${v}_lds_1" -o run -- python3 "$R/bench.py" --config ${CFG:-c5} --steps 1 --warmup 0 --device-steps 0 --no-d2h --no-cpu-baseline --rms-calls 0 > "$R/gpurun_out/${TAG}_${v}_lds.log" 2>&1 || { tail -20 "$R/gpurun_out/${TAG}_${v}_lds.log"; exit 1; }
  (cd "$R" && python3 tools/pmc_summary.py ${TAG}_${v}_lds ${CFG:-c5} > gpurun_out/${TAG}_${v}_lds.json)
  python3 - "$R/gpurun_out/${TAG}_${v}_lds.json" "$v" ${KERNELS:-sg_stft_ola sg_stft_ola_noise} <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))["kernels"]
for k in sys.argv[3:]:
    acc = {}
    for key, e in d.items():
        if key.split(" ")[0] != k:
            continue
        for c, x in e.items():
            if c.startswith("SQ_"):
                acc[c] = acc.get(c, 0.0) + x * e["launches"]
    if not acc:
        continue
    ins = acc.get("SQ_INSTS_LDS", 0) or 1
    idx = acc.get("SQ_LDS_IDX_ACTIVE", 0) or 1
    print("%s %s conflict/inst %.3f conflict/idx_active %.3f unaligned/inst %.3f idx_active/busy_cu %.3f lds_inst/valu_inst %.3f"
          % (sys.argv[2], k, acc.get("SQ_LDS_BANK_CONFLICT", 0) / ins, acc.get("SQ_LDS_BANK_CONFLICT", 0) / idx,
             acc.get("SQ_LDS_UNALIGNED_STALL", 0) / ins, idx / (acc.get("SQ_BUSY_CU_CYCLES", 0) or 1),
             ins / (acc.get("SQ_INSTS_VALU", 0) or 1)))
EOF
done
