"""D2H bandwidth into pinned host memory (what bounds bench.py's host-resident
headline): one 4 GB copy on one stream, the same split over 2 and 4 streams, and
a 4-way split issued on one stream. Prints GB/s per layout."""
import json
import time

import torch

dev = torch.device("cuda:0")
n = 1 << 30  # floats: 4 GiB
src = torch.empty(n, dtype=torch.float32, device=dev).fill_(1.0)
dst = torch.empty(n, dtype=torch.float32, pin_memory=True)
res = {}


def run(nstreams, parts, reps=3):
    streams = [torch.cuda.Stream(dev) for _ in range(nstreams)]
    best = 0.0
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for p in range(parts):
            a, b = p * n // parts, (p + 1) * n // parts
            with torch.cuda.stream(streams[p % nstreams]):
                dst[a:b].copy_(src[a:b], non_blocking=True)
        torch.cuda.synchronize()
        best = max(best, 4.0 * n / (time.perf_counter() - t) / 1e9)
    return best


for ns, parts in ((1, 1), (1, 4), (2, 2), (4, 4), (2, 8)):
    res["%d streams, %d parts" % (ns, parts)] = round(run(ns, parts), 1)
print(json.dumps({"d2h_GBps_pinned": res}))
