"""fp32 formant-filter error against the planner's conditioning estimate (GPU).

Random calls with extreme formant / rolloff / lip / stochastic-formant settings
(tests/test_precision_selector.py's generator) plus a C5 sample are synthesized
with the fp64 path disabled (sg_set_fp64_policy(0): every filter in fp32) and
with the default policy; each call's RMS error against the oracle is written
next to the planner's estimate rho (batch.Plan.conditioning) and window length,
so the threshold can be set from measured errors:
    python tools/selector_study.py out.json [n_random]
"""
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main(out_path, n_random=192):
    import bench
    from oracle import oracle as O
    from soundgen_beta_amd import batch, native
    from test_precision_selector import _extreme_calls
    O.lib()
    calls = []
    for seed in range(n_random // 24):
        calls += _extreme_calls(24, 100 + seed)
    c5 = bench.c5_calls(2000)[::10]
    calls += c5
    plan = batch.Plan(calls, None)
    rho = plan.conditioning()
    hp = plan.precision()[0]
    wl = [int(round(c["args"].get("windowLength", 50) * 44100 / 1000 / 2)) * 2 for c in calls]
    L = native.lib()
    outs = {}
    for pol in (0, 1):
        assert L.sg_set_fp64_policy(pol, native.HP_RHO_DEFAULT) == 0
        try:
            outs[pol] = batch.synthesize(calls, device=0)
        finally:
            L.sg_set_fp64_policy(1, native.HP_RHO_DEFAULT)

    def ref(c):
        try:
            return bench.oracle_call(O, c)
        except Exception:  # noqa: BLE001
            return None
    with ThreadPoolExecutor(bench.host_cores()) as ex:
        refs = list(ex.map(ref, calls))
    rows = []
    for i, c in enumerate(calls):
        r = refs[i]
        e = {}
        for pol in (0, 1):
            y = outs[pol][i]
            e[pol] = (float(np.sqrt(np.mean((np.asarray(y, np.float64) - r) ** 2)))
                      if r is not None and not isinstance(y, Exception) and len(y) == len(r) else None)
        rows.append({"i": i, "preset": c.get("preset", "random"), "wl": wl[i], "rho": float(rho[i]),
                     "hp_bouts": int(hp[i]), "err_fp32": e[0], "err_default": e[1]})
    json.dump({"rows": rows}, open(out_path, "w"), indent=0)
    bad = [r for r in rows if r["err_default"] is not None and r["err_default"] > 1e-5]
    print("calls %d, default policy over 1e-5: %d" % (len(rows), len(bad)))
    for r in sorted(rows, key=lambda r: -(r["err_fp32"] or 0))[:25]:
        print(r)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 192)
