"""GPU outputs of chosen C5 calls under the fp64 filter policies, saved for
offline error analysis against the oracle (diagnostic).

    python tools/call_diag.py OUT.npz INDEX [INDEX ...]
    python tools/call_diag.py --scan STRIDE   (every STRIDE-th call: the 15 worst RMS)

INDEX is a call of the 65,536-call C5 batch (bench.c5_calls). Each call is
synthesized alone with the default policy (fp64 filter above SG_HP_RHO) and
with every filtered bout on the fp64 path; the npz holds y_default_<i>,
y_hp_<i> and the oracle's ref_<i>."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
from oracle import oracle as O  # noqa: E402
from soundgen_beta_amd import batch, native  # noqa: E402


def main(out, idx):
    calls = bench.c5_calls(65536)
    L = native.lib()
    res = {}
    for i in idx:
        c = calls[i]
        ref = bench.oracle_call(O, c)
        res["ref_%d" % i] = ref
        for name, mode in (("default", 1), ("hp", 2)):
            L.sg_set_fp64_policy(mode, 300.0)
            y = batch.synthesize([c])[0]
            res["y_%s_%d" % (name, i)] = np.asarray(y, np.float64)
            r = float(np.sqrt(np.mean((y - ref) ** 2))) if len(y) == len(ref) else float("inf")
            print("call %d %s %s rms %.3e" % (i, c["preset"], name, r), flush=True)
    L.sg_set_fp64_policy(1, 300.0)
    np.savez_compressed(out, **res)


def scan(stride):
    from concurrent.futures import ThreadPoolExecutor
    calls = bench.c5_calls(65536)[::stride]
    outs = batch.synthesize(calls)
    refs = []
    with ThreadPoolExecutor(16) as ex:
        for k in range(0, len(calls), 256):  # a progress line per 256 calls
            refs += list(ex.map(lambda c: bench.oracle_call(O, c), calls[k:k + 256]))
            print("scan: oracle %d/%d" % (len(refs), len(calls)), flush=True)
    rows = []
    for i, (y, ref) in enumerate(zip(outs, refs)):
        r = float(np.sqrt(np.mean((y - ref) ** 2))) if len(y) == len(ref) else float("inf")
        rows.append((r, i * stride, calls[i]["preset"]))
    rows.sort(reverse=True)
    for r, i, p in rows[:15]:
        print("scan rms %.3e call %d %s" % (r, i, p))
    by = {}
    for r, i, p in rows:
        by[p] = max(by.get(p, 0.0), r)
    print("worst per preset:", " ".join("%s %.1e" % kv for kv in sorted(by.items(), key=lambda kv: -kv[1])))


if __name__ == "__main__":
    if sys.argv[1] == "--scan":
        scan(int(sys.argv[2]))
    else:
        main(sys.argv[1], [int(a) for a in sys.argv[2:]])
