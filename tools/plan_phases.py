"""Per-phase host timing of bench.py's plan loop on the GPU box: Plan() (descriptor
marshalling + sg_plan_batch), upload, release_host, for C5 chunks of 16,384 calls."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
import bench  # noqa: E402
from soundgen_beta_amd import batch, native  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
torch.zeros(1, device="cuda")
calls = bench.c5_calls(n)
ctx = native.Context(0)
for a in range(0, n, 16384):
    t0 = time.perf_counter()
    p = batch.Plan(calls[a:a + 16384], ctx)
    t1 = time.perf_counter()
    p.upload()
    t2 = time.perf_counter()
    p.release_host()
    t3 = time.perf_counter()
    print("chunk %d: plan %.2f s, upload %.2f s (%.1f GB device), release %.2f s" % (
        a, t1 - t0, t2 - t1, p.device_bytes() / 1e9, t3 - t2), flush=True)
t0 = time.perf_counter()
p = batch.Plan(calls[0:16384], None)
print("plan without ctx %.2f s" % (time.perf_counter() - t0), flush=True)
