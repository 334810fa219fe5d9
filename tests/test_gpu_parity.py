"""GPU parity: the HIP path (libsoundgen_hip.so through the C-ABI) vs the CPU
oracle on the same inputs and injected random draws.
Tolerance: RMS <= 1e-5 on the normalised waveform (BASELINE.json north star);
sample counts bit-exact."""
import numpy as np
import pytest

from test_planner import CASES, NORMALS, UNIFORMS

pytestmark = pytest.mark.gpu

C2 = dict(samplingRate=44100, temperature=0, nonlinBalance=0, rolloff=-12, rolloffOct=-12, rolloffKHz=-6,
          pitchFloor=50)
TOL = 1e-5


def _rms(a, b):
    return float(np.sqrt(np.mean((np.asarray(a, np.float64) - b) ** 2)))


def test_c2_tones_batch(oracle):
    from soundgen_beta_amd import batch
    rng = np.random.Generator(np.random.PCG64(20261015))
    f0 = np.exp(rng.uniform(np.log(80), np.log(400), 24))
    calls = [{"kind": "harmonics", "pitch": np.full(3500, f), "params": C2} for f in f0]
    outs = batch.synthesize(calls)
    for c, y in zip(calls, outs):
        ref = oracle.generate_harmonics(c["pitch"], **c["params"])
        assert len(y) == len(ref)
        assert _rms(y, ref) <= TOL


def test_planner_cases_one_batch(oracle):
    """Every planner case (vibrato, subharmonic epochs + crossfades, jitter,
    shimmer, temperature random walks, 16 kHz, near-ceiling f0) in ONE batch."""
    from soundgen_beta_amd import batch
    calls = [{"kind": "harmonics", "pitch": p, "params": prm, "normals": NORMALS, "uniforms": UNIFORMS}
             for _, p, prm in CASES]
    outs = batch.synthesize(calls)
    worst = 0.0
    for (name, p, prm), y in zip(CASES, outs):
        ref = oracle.generate_harmonics(p, normals=NORMALS, uniforms=UNIFORMS, **prm)
        assert len(y) == len(ref), name
        r = _rms(y, ref)
        worst = max(worst, r)
        assert r <= TOL, (name, r)
    print("worst rms", worst)


def test_ampl_anchors_and_contours(oracle):
    from soundgen_beta_amd import batch
    t = np.linspace(0, 1, 3500)
    calls = [
        {"kind": "harmonics", "pitch": np.full(3500, 180.0), "params": C2,
         "amplAnchors": {"time": [0, 1], "value": [110, 60]}},
        {"kind": "harmonics", "pitch": 300 - 120 * t ** 2, "params": C2},
        {"kind": "harmonics", "pitch": 220 * 2 ** (0.5 * np.sin(2 * np.pi * 3 * t)), "params": C2},
        {"kind": "harmonics", "pitch": 150 + 100 * t, "params": dict(samplingRate=16000)},
    ]
    for c, y in zip(calls, batch.synthesize(calls)):
        ref = oracle.generate_harmonics(c["pitch"], amplAnchors=c.get("amplAnchors"), **c["params"])
        assert len(y) == len(ref)
        assert _rms(y, ref) <= TOL


def test_edge_single_and_empty_batches(oracle):
    from soundgen_beta_amd import batch
    c = {"kind": "harmonics", "pitch": np.full(40, 500.0), "params": C2}  # very short: few glottal cycles
    out = batch.synthesize([c])
    ref = oracle.generate_harmonics(c["pitch"], **c["params"])
    assert len(out[0]) == len(ref) and _rms(out[0], ref) <= TOL
    assert batch.synthesize([]) == []
