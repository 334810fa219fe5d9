"""Planner stage times of one C5 chunk on this host (no GPU use): SG_PLAN_PROF=1
makes the library print its per-stage totals (parts on N threads, merge,
finalize_plan, finalize_spec, inclusive per-scope CPU seconds).
   SG_PLAN_PROF=1 python tools/plan_stages.py [calls] [repeats]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from soundgen_beta_amd import batch  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    calls = bench.c5_calls(n)
    for r in range(reps):
        t = time.perf_counter()
        m = batch.Marshalled(calls)
        t1 = time.perf_counter()
        p = batch.Plan(None, None, m)
        t2 = time.perf_counter()
        p.close()
        t3 = time.perf_counter()
        print(f"rep {r}: marshal {t1 - t:.3f} s plan {t2 - t1:.3f} s close {t3 - t2:.3f} s", flush=True)


if __name__ == "__main__":
    main()
