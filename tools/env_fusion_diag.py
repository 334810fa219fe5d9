"""Envelope-fusion diagnosis on the GPU: the test batch of
tests/test_gpu_parity.py::test_evaluated_envelope_columns_byte_equal synthesized
with sg_set_envelope_fusion 0 (all materialised), 1 (filter columns evaluated),
2 (noise columns evaluated) and 3; per mode the calls that differ from mode 0,
their largest absolute difference relative to the call's peak, and their kind."""
import json
import sys

import numpy as np

sys.path.insert(0, ".")
import bench  # noqa: E402
from soundgen_beta_amd import batch, native  # noqa: E402
from soundgen_beta_amd.rrng import RRng  # noqa: E402


def main():
    def make():  # R-stream generators are consumed by planning: fresh ones per plan
        c = bench.c5_calls(300)[::3] + bench.c3_calls(8)
        return c + [{"kind": "soundgen", "args": {"sylLen": 250, "samplingRate": 16000, "addSilence": 0,
                                                  "formants": "a", "noiseAnchors": {"time": [0, 250], "value": [-25, -15]}},
                     "rng": RRng(40 + i)} for i in range(3)]
    calls = make()
    L = native.lib()
    p = batch.Plan(make())
    fp64 = p.precision()[0]
    p.close()
    outs = {}
    for mode in (0, 1, 2, 3):
        L.sg_set_envelope_fusion(mode)
        try:
            outs[mode] = batch.synthesize(make())
        finally:
            L.sg_set_envelope_fusion(3)
    rep = {}
    for mode in (1, 2, 3):
        bad = []
        for i, (a, b) in enumerate(zip(outs[0], outs[mode])):
            if a.tobytes() != b.tobytes():
                pk = float(np.max(np.abs(a))) or 1.0
                d = np.abs(a.astype(np.float64) - b.astype(np.float64))
                bad.append({"call": i, "len": len(a), "max_rel": float(d.max() / pk), "n_diff": int((d > 0).sum()),
                            "first": int(np.argmax(d > 0)), "fp64": int(fp64[i]),
                            "preset": str(calls[i].get("preset", calls[i]["args"].get("formants", "")))[:40]})
        rep[mode] = {"n_calls": len(calls), "n_differ": len(bad), "calls": bad[:12]}
        print(mode, len(bad), "of", len(calls), bad[:4], flush=True)
    json.dump(rep, open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/env_fusion_diag.json", "w"), indent=1)


if __name__ == "__main__":
    main()
