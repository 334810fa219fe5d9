"""GPU parity: HIP path vs the CPU oracle on the same inputs.
Tolerance: RMS <= 1e-5 on the normalised waveform (BASELINE.json north star),
sample counts bit-exact."""
import numpy as np
import pytest

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


def test_pitch_contours(oracle):
    from soundgen_beta_amd import batch
    t = np.linspace(0, 1, 3500)
    pitches = [150 + 100 * t, 300 - 120 * t ** 2, 220 * 2 ** (0.5 * np.sin(2 * np.pi * 3 * t)), np.full(700, 1000.0)]
    calls = [{"kind": "harmonics", "pitch": p, "params": C2} for p in pitches]
    calls.append({"kind": "harmonics", "pitch": pitches[0], "params": dict(samplingRate=16000)})
    for c, y in zip(calls, batch.synthesize(calls)):
        ref = oracle.generate_harmonics(c["pitch"], **c["params"])
        assert len(y) == len(ref)
        assert _rms(y, ref) <= TOL
