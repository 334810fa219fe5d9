"""fp32 pre-filter noise error against the planner's noise conditioning estimate (GPU).

C3 calls (breathing noise under a vowel filter) and a C5 sample are synthesized
with every noise on the fp32 kernels (SG_HP_RHO_NOISE=1e30; the formant filter
keeps its default policy); each call's RMS error against the oracle is written
next to its noise conditioning rho_noise (batch.Plan.noise_conditioning), so the
fp64 noise threshold can be set from measured errors:
    python tools/noise_selector_study.py out.json [n_c3] [n_c5]
"""
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

os.environ["SG_HP_RHO_NOISE"] = "1e30"  # read once, at the planner's first noise decision
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out_path, n_c3=256, n_c5=4096):
    import bench
    from oracle import oracle as O
    from soundgen_beta_amd import batch
    O.lib()
    calls = bench.c3_calls(n_c3) + bench.c5_calls(n_c5)[::4]
    plan = batch.Plan(calls, None)
    rho_n = plan.noise_conditioning()
    rho_f = plan.conditioning()
    outs = batch.synthesize(calls, device=0)

    def ref(c):
        try:
            return bench.oracle_call(O, c)
        except Exception:  # noqa: BLE001
            return None
    with ThreadPoolExecutor(bench.host_cores()) as ex:
        refs = list(ex.map(ref, calls))
    rows = []
    for i, c in enumerate(calls):
        r, y = refs[i], outs[i]
        e = (float(np.sqrt(np.mean((np.asarray(y, np.float64) - r) ** 2)))
             if r is not None and not isinstance(y, Exception) and len(y) == len(r) else None)
        rows.append({"i": i, "preset": c.get("preset", "c3"), "rho_noise": float(rho_n[i]), "rho_filter": float(rho_f[i]),
                     "err_fp32_noise": e})
    bad = [r for r in rows if r["err_fp32_noise"] is not None and r["err_fp32_noise"] > 1e-5]
    lo = min((r["rho_noise"] for r in bad), default=None)
    summary = {"calls": len(rows), "over_1e-5": len(bad), "min_rho_noise_over_1e-5": lo,
               "max_err_by_rho_noise": {str(t): max((r["err_fp32_noise"] for r in rows
                                                     if r["err_fp32_noise"] is not None and r["rho_noise"] <= t),
                                                    default=None) for t in (30, 60, 100, 150, 200, 300, 1e9)}}
    json.dump({"summary": summary, "rows": rows}, open(out_path, "w"), indent=0)
    print(json.dumps(summary))
    for r in sorted(rows, key=lambda r: -(r["err_fp32_noise"] or 0))[:12]:
        print(r)


if __name__ == "__main__":
    main(sys.argv[1], *(int(a) for a in sys.argv[2:]))
