"""Multi-GPU load balance of the C5 batch, predicted on the CPU.

Plans the 65,536-call C5 batch with the product planner (CPU only), takes each
call's actual device work from the plan (sg_plan_call_work: sine-bank (sample,
row) terms, nominal FFT flops; output samples), prices it with the per-unit
kernel times of dist.py (W_ROW, W_FLOP, W_SAMPLE), and reports the max/mean rank
load at N = 2, 4, 8 for:
  lpt_analytic  dist.shard's assignment (LPT over dist.call_cost, arguments only)
  round_robin   call i -> rank i mod N
  lpt_actual    LPT over the planned cost (a lower bound for LPT)
Writes profiles/<tag>_dist_balance.json. Unmeasured on hardware: the driver's
8-GPU scaling run is the measurement.

    python tools/dist_balance.py [tag] [calls]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(tag="r03", n_calls=65536):
    import bench
    from soundgen_beta_amd import batch
    from soundgen_beta_amd import dist as sgd
    n_calls = int(n_calls)
    calls = bench.c5_calls(n_calls)
    t0 = time.perf_counter()
    rows, flops, samples = [], [], []
    for a in range(0, n_calls, 16384):
        p = batch.Plan(calls[a:a + 16384], None)
        r, f = p.call_work()
        rows.append(r)
        flops.append(f)
        samples.append(p.lengths.astype(np.float64))
        p.close()
    rows, flops, samples = np.concatenate(rows), np.concatenate(flops), np.concatenate(samples)
    plan_s = time.perf_counter() - t0
    actual = rows * sgd.W_ROW + flops * sgd.W_FLOP + samples * sgd.W_SAMPLE
    analytic = np.array([sgd.call_cost(c) for c in calls])
    res = {"workload": "C5, %d calls (bench.c5_calls)" % n_calls, "plan_s_cpu": plan_s,
           "weights_ns": {"row": sgd.W_ROW, "flop": sgd.W_FLOP, "sample": sgd.W_SAMPLE},
           "total_cost_ms": float(actual.sum()) / 1e6,
           "corr_analytic_vs_planned": float(np.corrcoef(analytic, actual)[0, 1]), "N": {}}
    for N in (2, 4, 8):
        out = {}
        for name, owner in (("lpt_analytic", sgd.lpt_assign(analytic, N)),
                            ("round_robin", np.arange(n_calls) % N),
                            ("lpt_actual", sgd.lpt_assign(actual, N))):
            load = np.array([actual[owner == r].sum() for r in range(N)])
            smp = np.array([samples[owner == r].sum() for r in range(N)])
            out[name] = {"max_over_mean": float(load.max() / load.mean()),
                         "samples_max_over_mean": float(smp.max() / smp.mean())}
        res["N"][str(N)] = out
    dst = os.path.join(ROOT, "profiles", "%s_dist_balance.json" % tag)
    with open(dst, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
