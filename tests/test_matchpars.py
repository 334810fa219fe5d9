"""compareSounds / getMelSpec / wigglePars / matchPars (soundgen_beta_amd/matchpars.py,
R/matchPars.R) on hand-derived cases (CPU), and the batched matchPars loop on
the GPU (its candidates equal per-call soundgen()). R is absent and the dtw
package is not vendored: similarity values are parity unpinned against R."""
import json
import math
import os

import numpy as np
import pytest

from soundgen_beta_amd import matchpars as MP
from soundgen_beta_amd import rrng

HERE = os.path.dirname(os.path.abspath(__file__))


def test_defaults_match_reference_rda():
    """MATCHPARS_DEFAULTS is the package's `defaults` list (data/defaults.rda; the
    first of a duplicated name, as R's `[` returns)."""
    d = json.load(open(os.path.join(HERE, "golden", "rda_fixtures.json")))["data/defaults.rda"]["defaults"]
    # the fixture keeps the LAST of a duplicated name (windowLength 40 then 50, samplingRate
    # 16000 twice; R/presets.R:117-144); defaults['windowLength'] in R is the first, 40
    assert d["windowLength"] == [50.0] and MP.MATCHPARS_DEFAULTS["windowLength"] == 40
    for k in d:
        if k == "windowLength":
            continue
        want = d[k]
        got = MP.MATCHPARS_DEFAULTS[k]
        if isinstance(want, list) and len(want) == 1:
            want = want[0]
        if want is None or (isinstance(want, list) and want == [None]):
            assert got is None, k
        elif isinstance(want, dict):
            for c, vals in want.items():
                if isinstance(vals, dict):  # a formant
                    for cc, vv in vals.items():
                        assert np.allclose(np.atleast_1d(got[c][cc]), vv), (k, c, cc)
                else:
                    assert np.allclose(np.atleast_1d(got[c]), vals), (k, c)
        else:
            assert math.isclose(float(got), float(want)), (k, got, want)


def test_mel_filterbank_hand_case():
    """fft2melmx (Slaney): triangles between consecutive mel edges, peak 2 / (f3 - f1)."""
    w = MP.fft2melmx(64, 16000, 10)
    assert w.shape == (10, 64)
    edges = MP._mel2hz(np.arange(12) / 11 * MP._hz2mel(8000.0))
    f = np.arange(64) / 64 * 16000
    for i in range(10):
        assert np.all(w[i][(f <= edges[i]) | (f >= edges[i + 2])] == 0)
        assert w[i].max() <= 2 / (edges[i + 2] - edges[i]) + 1e-15
    # hz2mel / mel2hz: linear below 1 kHz (200/3 Hz per mel), log above, inverse of each other
    assert math.isclose(float(MP._hz2mel(1000.0)), 15.0) and math.isclose(float(MP._mel2hz(MP._hz2mel(3000.0))), 3000.0)


def test_get_mel_spec_shape_and_range():
    sr = 16000
    t = np.arange(sr) / sr
    x = np.sin(2 * np.pi * 440 * t) * np.hanning(sr)
    spec = MP.get_mel_spec(x, sr)
    assert spec.shape[0] == 200  # nbands = 100 windowLength / 20
    # frames: seq(1, length - winpts, by = steppts): winpts 640, step 320
    assert spec.shape[1] <= len(range(1, sr - 640 + 1, 320))
    assert spec.min() == 0.0 and spec.max() == 1.0
    # a sine's energy sits in the band around 440 Hz
    edges = MP._mel2hz(np.arange(202) / 201 * MP._hz2mel(8000.0))
    band = int(np.argmax(spec.mean(axis=1)))
    assert edges[band] <= 440 <= edges[band + 2]


def test_compare_sounds_identity_and_order():
    """A sound compared with itself scores 1 (cor, cosine, pixel, dtw); a different
    pitch scores lower; the summary is the mean of the methods."""
    sr = 16000
    t = np.arange(int(0.5 * sr)) / sr
    a = np.sin(2 * np.pi * 200 * t) + 0.5 * np.sin(2 * np.pi * 400 * t)
    b = np.sin(2 * np.pi * 300 * t) + 0.5 * np.sin(2 * np.pi * 600 * t)
    same = MP.compare_sounds(a, None, a, sr, summary=False)
    for m in ("cor", "cosine", "pixel"):
        assert math.isclose(same[m], 1.0, rel_tol=1e-12), (m, same[m])
    assert math.isclose(same["dtw"], 1.0, abs_tol=1e-12)
    diff = MP.compare_sounds(a, None, b, sr, summary=False)
    assert all(diff[m] < same[m] for m in same)
    s = MP.compare_sounds(a, None, b, sr, summary=True)
    assert math.isclose(s, np.mean(list(diff.values())), rel_tol=1e-12)
    # penalizeLengthDif: a longer candidate is padded with NA columns that count as 0
    longer = np.concatenate([a, a])
    p = MP.compare_sounds(a, None, longer, sr, method=("pixel",), summary=True)
    q = MP.compare_sounds(a, None, longer, sr, method=("pixel",), summary=True, penalizeLengthDif=False)
    assert p < q


def test_dtw_symmetric2_hand_cases():
    # identical: 0; a constant offset c over n points: n c (diagonal steps count 2 d) / 2n
    x = np.array([0.0, 1.0, 2.0, 3.0])
    assert MP.dtw_normalized(x, x) == 0.0
    assert math.isclose(MP.dtw_normalized(x, x + 0.5), (0.5 + 2 * 0.5 * 3) / 8)
    # a repeated sample is absorbed by a horizontal step at zero cost
    assert MP.dtw_normalized(np.array([0.0, 1.0, 2.0]), np.array([0.0, 1.0, 1.0, 2.0])) == 0.0


def test_match_columns_central_na():
    m = np.arange(6, dtype=float).reshape(2, 3)
    # matchLengths(1:3, 6, 'central', NA): c(NA x 6, 1:3, NA x 6)[5:10] -> NA NA 1 2 3 NA
    out = MP._match_columns(m, 6)
    assert np.isnan(out[:, :2]).all() and np.isnan(out[:, 5]).all()
    assert np.array_equal(out[:, 2:5], m)


def test_wiggle_pars_draw_order_and_bounds():
    """wigglePars with R's RNG: deterministic per seed, mutated values inside the
    permittedValues bounds, integers rounded (rolloffParabHarm), anchors keep
    their first and last times."""
    pars = {"sylLen": 300.0, "rolloffParabHarm": 3.0, "pitchAnchors": {"time": [0, .5, 1], "value": [100, 150, 120]}}
    outs = []
    for _ in range(2):
        D = MP._Draws(rrng.RRng(7))
        outs.append([MP.wiggle_pars(D, pars, ["sylLen", "rolloffParabHarm", "pitchAnchors"], .75, .5)
                     for _ in range(20)])
    assert outs[0] == outs[1]
    for p in outs[0]:
        assert 20 <= p["sylLen"] <= 5000
        assert p["rolloffParabHarm"] == round(p["rolloffParabHarm"]) and 1 <= p["rolloffParabHarm"] <= 20
        pa = p["pitchAnchors"]
        assert pa["time"][0] == 0 and pa["time"][-1] == 1
        assert all(50 <= v <= 3500 for v in pa["value"])
    assert any(p != pars for p in outs[0])


def test_revsort_ties_like_r():
    # R: sample(c('nothing', 'remove', 'add'), 1, prob = c(.9, .05, .05)) orders the tie remove/add
    # as revsort leaves it; u <= .9 -> nothing
    p, perm = [0.9, 0.05, 0.05], [1, 2, 3]
    MP._revsort(p, perm)
    assert p == [0.9, 0.05, 0.05] and perm[0] == 1 and sorted(perm[1:]) == [2, 3]


@pytest.mark.gpu
def test_match_pars_batch_equals_single_calls():
    """One generation of matchPars: the pop mutants synthesized as one GPU batch equal
    per-call soundgen() with the same parameters (draw-free: temperature 0)."""
    from soundgen_beta_amd import api, batch
    sr = 16000
    target = api.soundgen(sylLen=400, pitchAnchors={"time": [0, 1], "value": [150, 220]}, temperature=0,
                          samplingRate=sr, addSilence=0)
    init = {"sylLen": 300, "pitchAnchors": {"time": [0, 1], "value": [120, 180]}, "temperature": 0, "addSilence": 0}
    res = MP.match_pars(target, sr, pars=["sylLen", "pitchAnchors"], init=init, maxIter=6, pop=4,
                        rng=rrng.RRng(3), method=("cor", "cosine", "pixel"))
    assert res["evaluated"] >= 5 and res["history"][0]["sim"] <= res["history"][-1]["sim"]
    D = MP._Draws(rrng.RRng(11))
    muts = [MP.wiggle_pars(D, dict(init, samplingRate=sr), ["sylLen", "pitchAnchors"], .25, .1) for _ in range(4)]
    ys = batch.synthesize([{"kind": "soundgen", "args": MP._soundgen_args(m)} for m in muts])
    for m, y in zip(muts, ys):
        ref = api.soundgen(**MP._soundgen_args(m))
        assert len(ref) == len(y) and np.array_equal(np.float32(ref), np.float32(y))


def _mel_batch_calls(sr, n, seed):
    rng = np.random.default_rng(seed)
    calls = []
    for i in range(n):
        f0 = float(np.exp(rng.uniform(np.log(90), np.log(500))))
        calls.append({"kind": "soundgen", "args": {
            "sylLen": float(rng.uniform(150, 900)), "samplingRate": sr, "temperature": 0, "addSilence": 0,
            "pitchAnchors": {"time": [0, 1], "value": [f0, f0 * float(rng.uniform(0.7, 1.5))]},
            "formants": str(rng.choice(list("aoieu"))), "rolloff": float(rng.uniform(-18, -6)),
            "noiseAnchors": {"time": [0, 300], "value": [float(rng.uniform(-40, -10))] * 2}},
            "uniforms": rng.uniform(size=200000)})
    return calls


@pytest.mark.gpu
@pytest.mark.parametrize("sr,wl,ov", [(16000, 40, 50), (44100, 40, 50), (22050, 25, 70)])
def test_mel_spec_gpu_equals_numpy(sr, wl, ov):
    """getMelSpec on the GPU (sg_mel_spec) vs the numpy restatement: same columns kept, <= 1e-9."""
    from soundgen_beta_amd import api
    y = api.soundgen(sylLen=700, samplingRate=sr, temperature=0, addSilence=50,
                     pitchAnchors={"time": [0, 1], "value": [140, 260]}, formants="ai")
    got = MP.get_mel_spec_gpu(y, sr, windowLength=wl, overlap=ov)
    want = MP.get_mel_spec(y, sr, windowLength=wl, overlap=ov)
    assert got.shape == want.shape
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("penalize", [True, False])
def test_compare_sounds_batch_gpu_equals_numpy(penalize):
    """compareSounds for a generation of 40 candidates in HBM (one launch sequence,
    sg_compare_sounds_batch) vs the numpy compare_sounds per candidate: every
    method (cor, cosine, pixel, dtw) and the summary within 1e-6; candidates both
    shorter and longer than the target (matchColumns' NA padding on either side)."""
    from soundgen_beta_amd import api, batch
    sr = 16000
    target = api.soundgen(sylLen=500, samplingRate=sr, temperature=0, addSilence=0,
                          pitchAnchors={"time": [0, 1], "value": [150, 220]}, formants="ae")
    tspec = MP.get_mel_spec(target, sr)
    calls = _mel_batch_calls(sr, 40, 5)
    data, offs, lens = batch.synthesize_packed(calls, 0)
    assert (lens > 0).all()
    got, summ = MP.compare_sounds_batch(tspec, data, offs, lens, sr, penalizeLengthDif=penalize)
    host = data.cpu().numpy()
    ncols = set()
    for i in range(len(calls)):
        y = host[offs[i]:offs[i] + lens[i]].astype(np.float64)
        want = MP.compare_sounds(None, tspec, y, sr, summary=False, penalizeLengthDif=penalize)
        ncols.add(np.sign(MP.get_mel_spec(y, sr).shape[1] - tspec.shape[1]))
        for m in ("cor", "cosine", "pixel", "dtw"):
            assert abs(got[m][i] - want[m]) <= 1e-6, (i, m, got[m][i], want[m])
        vals = [v for v in want.values() if not math.isnan(v)]
        assert abs(summ[i] - np.mean(vals)) <= 1e-6
    assert ncols >= {-1, 1}  # shorter and longer candidates both exercised
