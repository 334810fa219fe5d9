"""Planning C5 calls whose draws come from ONE stream through callbacks (how the R
shim binds R's RNG) against planning them with injected draws (verdict r04 item 5).
CPU only: no device is touched.

    python tools/callback_planning.py [calls]

Prints seconds for: injected draws (parallel parts), one RRng stream through
callbacks (serial: a stream is sequential), and the node path (sg_node_plan_batch:
a serial recording pass in call order, then the shards planned in parallel from each
call's recorded draws)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from soundgen_beta_amd import batch, native  # noqa: E402
from soundgen_beta_amd.rrng import RRng  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    calls = bench.c5_calls(n)
    for _ in range(2):  # the second plan reuses the first one's host blocks (as the bench's later chunks do)
        t = time.perf_counter()
        p = batch.Plan(calls, None)
        t_inj = time.perf_counter() - t
        p.close()
    args = [c["args"] for c in calls]
    g = RRng(7)
    t = time.perf_counter()
    p = batch.Plan([{"kind": "soundgen", "args": a, "rng": g} for a in args], None)
    t_cb = time.perf_counter() - t
    ok = int((p.status == 0).sum())
    p.close()
    g = RRng(7)
    node = native.Node([0, 0])
    t = time.perf_counter()
    q = batch.NodePlan([{"kind": "soundgen", "args": a, "rng": g} for a in args], node)
    t_node = time.perf_counter() - t
    q.close()
    node.close()
    print(f"{n} C5 calls: injected draws {t_inj:.2f} s; one callback stream, serial {t_cb:.2f} s "
          f"({t_cb / t_inj:.1f}x, {ok} planned); node record + parallel replay {t_node:.2f} s "
          f"({t_node / t_inj:.1f}x); host threads {os.cpu_count()}", flush=True)


if __name__ == "__main__":
    main()
