"""Regenerate tests/golden/*.npz — restatement-derived golden vectors.

R is absent from the build container, so these vectors come
from the C oracle (oracle/sg_oracle.c, itself checked against the NumPy twin in
tests/test_oracle.py); they pin the HIP path and guard the oracle against
regressions. tools/r_golden.R writes the same cases from real R where R exists.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import oracle as O  # noqa: E402

rng = np.random.default_rng(20261015)
NORMALS = rng.standard_normal(4000)

CASES = {
    # R/source.R:167-172: pitch = getSmoothContour(200 -> 300, len = 3500), samplingRate = 16000
    "roxygen_harmonics": (np.linspace(0, 1, 3500) * 100 + 200, dict(samplingRate=16000), None),
    "tone_150_16k": (np.full(1750, 150.0), dict(samplingRate=16000, rolloff=-12, rolloffOct=-12, pitchFloor=50), None),
    "subharm_16k": (np.full(3500, 320.0), dict(samplingRate=16000, nonlinBalance=100, subFreq=110, subDep=90,
                                              jitterDep=1, shimmerDep=10), NORMALS),
}


def main():
    out = {}
    for name, (pitch, params, normals) in CASES.items():
        y = O.generate_harmonics(pitch, normals=normals, **params)
        out[name + "__pitch"] = pitch
        out[name + "__y"] = y
        out[name + "__params"] = np.array(repr(params))
        if normals is not None:
            out[name + "__normals"] = normals
    np.savez_compressed(os.path.join(HERE, "harmonics_golden.npz"), **out)
    print("wrote", len(CASES), "cases")


if __name__ == "__main__":
    main()
