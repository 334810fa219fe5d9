"""Per-wave instruction mix per kernel from a tools/gpu_imix.sh summary (pmc_summary
JSON): each counter summed over the kernel's launches, divided by SQ_WAVES.
    python tools/imix_summary.py gpurun_out/TAG_CFG_imix.json [kernel ...]
"""
import json
import sys

d = json.load(open(sys.argv[1]))["kernels"]
want = sys.argv[2:]
acc = {}
for key, e in d.items():
    k = key.split(" ")[0]
    if want and k not in want:
        continue
    a = acc.setdefault(k, {})
    for c, x in e.items():
        if c.startswith("SQ_"):
            a[c] = a.get(c, 0.0) + x * e["launches"]
cols = ["SQ_INSTS_VALU", "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32",
        "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
        "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_CVT", "SQ_INSTS_SALU", "SQ_INSTS_SMEM",
        "SQ_INSTS_LDS"]
short = [c.replace("SQ_INSTS_", "").replace("VALU_", "") for c in cols]
print("%-26s %9s " % ("kernel (per wave)", "waves") + " ".join("%9s" % s for s in short))
for k, a in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_INSTS_VALU", 0)):
    w = a.get("SQ_WAVES", 0) or 1  # per-launch means x launches, like every counter
    print("%-26s %9.0f " % (k[:26], w) + " ".join("%9.1f" % (a.get(c, float("nan")) / w) for c in cols))
