"""Golden vectors (tests/golden/, restatement-derived — see make_golden.py):
CPU: the oracle reproduces them exactly (regression pin);
GPU: the HIP path matches them within the north-star tolerance."""
import ast
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "harmonics_golden.npz")
TOL = 1e-5  # RMS on the normalised waveform (BASELINE.json north star)


def _cases():
    z = np.load(GOLDEN)  # allow_pickle stays False
    names = sorted({k.split("__")[0] for k in z.files})
    for n in names:
        normals = z[n + "__normals"] if n + "__normals" in z.files else None
        yield n, z[n + "__pitch"], ast.literal_eval(str(z[n + "__params"])), normals, z[n + "__y"]


def test_oracle_reproduces_golden(oracle):
    for name, pitch, params, normals, y in _cases():
        got = oracle.generate_harmonics(pitch, normals=normals, **params)
        assert len(got) == len(y), name
        np.testing.assert_array_equal(got, y, err_msg=name)


@pytest.mark.gpu
def test_hip_matches_golden():
    from soundgen_beta_amd import batch
    cases = list(_cases())
    calls = [{"kind": "harmonics", "pitch": p, "params": prm, "normals": nrm} for _, p, prm, nrm, _ in cases]
    outs = batch.synthesize(calls)
    for (name, _, _, _, y), got in zip(cases, outs):
        assert len(got) == len(y), name
        rms = float(np.sqrt(np.mean((got.astype(np.float64) - y) ** 2)))
        assert rms <= TOL, (name, rms)
