"""Diagnostic: GPU path vs oracle RMS for C5 call i under argument variants.
python tools/c5_variant_rms.py n_calls i '{"label": {"arg": value|null}}'"""
import copy, os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import bench
from soundgen_beta_amd import batch, native
from oracle import oracle as O

n, i0 = int(sys.argv[1]), int(sys.argv[2])
base = bench.c5_calls(n)[i0]
print(base["preset"], json.dumps({k: v for k, v in base["args"].items()}, default=str)[:800])
variants = {"as is": {}, **(json.loads(sys.argv[3]) if len(sys.argv) > 3 else {})}
calls, labels = [], []
for lab, mod in variants.items():
    c = copy.deepcopy(base)
    for k, v in mod.items():
        if v is None:
            c["args"].pop(k, None)
        else:
            c["args"][k] = v
    calls.append(c)
    labels.append(lab)
ctx = native.Context(0)
plan = batch.Plan(calls, ctx)
plan.upload()
out = torch.empty(max(plan.total, 1), dtype=torch.float32, device="cuda")
plan.execute(out.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
for i, lab in enumerate(labels):
    if plan.status[i]:
        print("%-28s status %d %s" % (lab, plan.status[i], plan.message(i)))
        continue
    lo, L = int(plan.offsets[i]), int(plan.lengths[i])
    y = out[lo:lo + L].double().cpu().numpy()
    ref = bench.oracle_call(O, calls[i])
    if len(ref) != L:
        print("%-28s len %d vs oracle %d" % (lab, L, len(ref)))
        continue
    e = y - ref
    k = int(np.abs(e).argmax())
    print("%-28s rms %.3e maxabs %.2e at %d/%d (gpu %.4f oracle %.4f)" % (lab, np.sqrt(np.mean(e ** 2)), abs(e[k]), k, L, y[k], ref[k]))
