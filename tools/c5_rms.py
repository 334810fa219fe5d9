"""Per-call RMS of the GPU path vs the oracle over the first C5 calls (diagnostic).
python tools/c5_rms.py [n_calls]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import bench
from soundgen_beta_amd import batch, native
from oracle import oracle as O

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
calls = bench.c5_calls(n)
ctx = native.Context(0)
plan = batch.Plan(calls, ctx)
plan.upload()
out = torch.empty(max(plan.total, 1), dtype=torch.float32, device="cuda")
plan.execute(out.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
res = []
for i in range(n):
    if plan.status[i]:
        continue
    lo, L = int(plan.offsets[i]), int(plan.lengths[i])
    y = out[lo:lo + L].double().cpu().numpy()
    ref = bench.oracle_call(O, calls[i])
    if len(ref) != len(y):
        res.append((np.inf, i, calls[i]["preset"], "len %d vs %d" % (len(y), len(ref))))
        continue
    e = y - ref
    res.append((float(np.sqrt(np.mean(e ** 2))), i, calls[i]["preset"], "maxabs %.2e at %d/%d" % (np.abs(e).max(), int(np.abs(e).argmax()), L)))
res.sort(reverse=True)
for r in res[:12]:
    print("rms %.3e call %d %s %s" % r)
print("calls checked", len(res), "over 1e-5:", sum(r[0] > 1e-5 for r in res))
