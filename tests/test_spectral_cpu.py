"""CPU: host parts of the spectral path — soundgen() planning: every output
length (syllables, pauses, noise trims, istft lengths, bouts, silence)
bit-exact with the oracle. (getSpectralEnvelope's matrix is computed on the
GPU: tests/test_gpu_spectral.py.)"""
import numpy as np
import pytest

from soundgen_beta_amd import api, batch

U = np.random.default_rng(1).uniform(size=3_000_000)
N = np.random.default_rng(2).standard_normal(200_000)

FORMANTS_A = {"f1": {"time": 0, "freq": 860, "amp": 30, "width": 120},
              "f2": {"time": 0, "freq": 1280, "amp": 40, "width": 120},
              "f3": {"time": 0, "freq": 2900, "amp": 25, "width": 200}}
MOVING = {"f1": {"time": [0, 1], "freq": [700, 300], "amp": [30, 30], "width": [100, 100]},
          "f2": {"time": [0, .5, 1], "freq": [1200, 1800, 2400], "amp": [40, 40, 40], "width": [120, 120, 150]}}


SOUNDGEN_CASES = {
    # C1 parity pin: presets$M1$Vowel1 defaults, sylLen 1000 @16 kHz, 2-anchor pitch
    "c1_pin": dict(sylLen=1000, samplingRate=16000, temperature=0, addSilence=0, pitchAnchors=[100, 150]),
    "c3_vowel_breathing": dict(sylLen=2000, samplingRate=44100, temperature=0, addSilence=0, windowLength=50,
                               overlap=75, formants="a", pitchAnchors=[120, 200],
                               noiseAnchors={"time": [0, 2000], "value": [-25, -25]}, formantsNoise=None),
    "multi_syl_bouts": dict(sylLen=500, samplingRate=16000, temperature=0, pitchAnchors=[300, 250], nSyl=3,
                            repeatBout=2, pauseLen=100),
    "post_noise_am": dict(sylLen=700, samplingRate=22050, temperature=0, pitchAnchors=[180, 140],
                          noiseAnchors={"time": [-50, 700], "value": [-10, -30]}, formantsNoise="s",
                          amDep=40, amFreq=25, amShape=0.3),
    "moving_formants_global_ampl": dict(sylLen=800, samplingRate=16000, temperature=0, pitchAnchors=[150, 220],
                                        formants=MOVING, amplAnchorsGlobal={"time": [0, 1], "value": [110, 80]},
                                        nSyl=2, pauseLen=150),
    "stochastic": dict(sylLen=400, samplingRate=16000, temperature=0.1, pitchAnchors=[200, 260], nSyl=2,
                       nonlinBalance=60, subDep=80, jitterDep=1, shimmerDep=5),
    "noise_only": dict(sylLen=300, samplingRate=16000, temperature=0, pitchAnchors=None,
                       noiseAnchors={"time": [0, 300], "value": [-20, -20]}),
    # loess contours (3-10 anchors): the default 4-anchor pitch, amplitude and noise anchors
    "default_pitch_loess": dict(sylLen=300, samplingRate=16000, temperature=0, addSilence=0),
    "loess_ampl_noise": dict(sylLen=600, samplingRate=16000, temperature=0, addSilence=0,
                             pitchAnchors={"time": [0, .2, .7, 1], "value": [140, 210, 180, 120]},
                             amplAnchors={"time": [0, .4, 1], "value": [110, 90, 120]},
                             noiseAnchors={"time": [0, 200, 400, 600], "value": [-40, -20, -25, -30]}),
}


@pytest.mark.parametrize("name", sorted(SOUNDGEN_CASES))
def test_soundgen_plan_lengths_match_oracle(oracle, name):
    kw = SOUNDGEN_CASES[name]
    p = batch.Plan([{"kind": "soundgen", "args": kw, "normals": N, "uniforms": U}], None)
    assert p.status[0] == 0, p.message(0)
    y = oracle.soundgen(normals=N, uniforms=U, **kw)
    assert p.lengths[0] == len(y)


def test_c5_plan_lengths_match_oracle(oracle):
    """C5 preset calls (bench.c5_calls): every planned length equals the oracle's,
    including presets with separately filtered noise, nSyl > 1 and temperature > 0
    (the draw order decides the lengths), and the failures are the documented ones."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    calls = bench.c5_calls(40)
    plan = batch.Plan(calls, None)
    for i, c in enumerate(calls):
        assert plan.status[i] == 0, (i, c["preset"], plan.message(i))
        assert plan.lengths[i] == len(bench.oracle_call(oracle, c)), (i, c["preset"])


def test_c4_c5_plan_nothing_refused():
    """Every C4 call and 1024 C5 calls plan (no SG_E_UNSUPPORTED): zero-width
    loess neighbourhoods take R's span + 0.1 retry, odd windows are planned."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    for calls in (bench.c4_calls(512), bench.c5_calls(1024)):
        plan = batch.Plan(calls, None)
        bad = np.nonzero(plan.status)[0]
        assert len(bad) == 0, [(int(i), plan.message(int(i))) for i in bad[:5]]
