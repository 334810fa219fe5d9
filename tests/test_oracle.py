"""CPU: the C oracle (oracle/sg_oracle.c) against the independent NumPy twin
(tests/np_twin.py) and against known answers derived from the reference's
own roxygen examples. R is absent, so these pin the oracle's
restatement, not R itself ("parity unpinned" vs R)."""
import numpy as np
import pytest

import np_twin as T


def test_glottal_cycles_roxygen_example(oracle):
    # soundgen:::getGlottalCycles(seq(150, 200, length.out = 350), samplingRate = 3500)
    # R/utilities_soundgen.R:473-476
    p = T.seq_len(150, 200, 350)
    got = oracle.glottal_cycles(p, 3500)
    assert np.array_equal(got, T.glottal_cycles(p, 3500))
    assert got[0] == 1 and np.all(np.diff(got) >= 2)


@pytest.mark.parametrize("n", [2, 3, 4, 7, 25])
def test_spline_fmm(oracle, n):
    rng = np.random.default_rng(n)
    x = np.cumsum(rng.uniform(0.5, 3, n))
    y = rng.normal(size=n)
    for m in (5, 17, 200):
        np.testing.assert_allclose(oracle.spline(x, y, m), T.spline(x, y, m), rtol=1e-11, atol=1e-11)


def test_spline_reproduces_cubic(oracle):
    # FMM end conditions make the spline exact for a cubic
    x = np.array([1.0, 2.5, 4, 6, 7.5, 9])
    y = 0.3 * x ** 3 - 2 * x ** 2 + x - 4
    u = T.seqint_len(1, 9, 50)
    np.testing.assert_allclose(oracle.spline(x, y, 50), 0.3 * u ** 3 - 2 * u ** 2 + u - 4, rtol=1e-10)


def test_approx(oracle):
    x = np.array([1.0, 4, 9, 10, 30])
    y = np.array([2.0, -1, 0.5, 7, 3])
    for n in (2, 3, 31, 100):
        np.testing.assert_allclose(oracle.approx(x, y, n), T.approx(x, y, n), rtol=1e-14, atol=1e-14)


# getRolloff roxygen examples, R/sourceSpectrum.R:32-70
ROLLOFF_EXAMPLES = [
    dict(pitch_per_gc=[150, 800, 3000], rolloff=-12, rolloffOct=0, rolloffKHz=0),
    dict(pitch_per_gc=[150, 800, 3000], rolloff=-12, rolloffOct=-3, rolloffKHz=0),
    dict(pitch_per_gc=[150, 800, 3000], rolloff=-12, rolloffOct=-3, rolloffKHz=-6),
    dict(pitch_per_gc=[150, 800, 3000], rolloff=-6, rolloffOct=0, rolloffKHz=-3),
    dict(pitch_per_gc=[400], rolloff=-12, rolloffOct=0, rolloffKHz=0, rolloffParab=10, rolloffParabHarm=1),
    dict(pitch_per_gc=[400], rolloff=-12, rolloffOct=0, rolloffKHz=0, rolloffParab=10, rolloffParabHarm=2),
    dict(pitch_per_gc=[400], rolloff=-12, rolloffOct=0, rolloffKHz=0, rolloffParab=20, rolloffParabHarm=4),
    dict(pitch_per_gc=[400], rolloff=-12, rolloffOct=0, rolloffKHz=0, rolloffParab=-20, rolloffParabHarm=7),
    # "only harmonics below 2000 Hz are affected" (R/sourceSpectrum.R:67-69)
    dict(pitch_per_gc=[150, 600], rolloff=-12, rolloffOct=-2, rolloffKHz=-6, rolloffParab=-20, rolloffParabCeiling=2000),
    dict(pitch_per_gc=[150, 333, 700, 1500], rolloff=-12, rolloffOct=-2, rolloffKHz=-6, rolloffParab=15,
         rolloffParabCeiling=1000),
]


@pytest.mark.parametrize("ex", ROLLOFF_EXAMPLES)
def test_get_rolloff_examples(oracle, ex):
    kw = dict(rolloff=ex["rolloff"], rolloffOct=ex["rolloffOct"], rolloffKHz=ex["rolloffKHz"],
              rolloffParab=ex.get("rolloffParab", 0), rolloffParabHarm=ex.get("rolloffParabHarm", 2),
              rolloffParabCeiling=ex.get("rolloffParabCeiling"))
    got = oracle.get_rolloff(ex["pitch_per_gc"], nHarmonics=100, samplingRate=16000, **kw)
    want = T.get_rolloff(ex["pitch_per_gc"], 100, kw["rolloff"], kw["rolloffOct"], kw["rolloffKHz"], 200, -120,
                         16000, kw["rolloffParab"], kw["rolloffParabHarm"], kw["rolloffParabCeiling"])
    from soundgen_beta_amd import api  # the product planner's getRolloff (host helper)
    np.testing.assert_array_equal(api.getRolloff(ex["pitch_per_gc"], nHarmonics=100, samplingRate=16000, **kw), got)
    assert got.shape == want.shape
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-300)
    # every column is normalised to a maximum of exactly 1 (0 dB)
    assert np.all(got.max(axis=0) == 1.0)


def test_rolloff_drops_and_renumbers_rows(oracle):
    # harmonics above Nyquist are -Inf -> 0 and dropped (R/sourceSpectrum.R:182-183)
    got = oracle.get_rolloff([3000], nHarmonics=100, samplingRate=16000)
    assert got.shape[0] == 2  # 3000, 6000 < 8000; 9000 > Nyquist


def test_find_zero_crossing_and_cross_fade(oracle):
    rng = np.random.default_rng(7)
    for k in range(40):
        a = np.sin(np.linspace(0, rng.uniform(3, 40), rng.integers(3, 400)) + rng.uniform(0, 6)) + rng.normal(0, .1)
        for loc in (1, len(a) // 2, len(a)):
            assert oracle.find_zero_crossing(a, loc) == T.find_zero_crossing(a, loc)
        b = np.sin(np.linspace(0, rng.uniform(3, 40), rng.integers(3, 400)) + rng.uniform(0, 6))
        for sr in (16000, 44100):
            np.testing.assert_allclose(oracle.cross_fade(a, b, sr), T.cross_fade(a, b, sr), rtol=0, atol=1e-15)


def test_cross_fade_onto_scalar_zero(oracle):
    # waveform = 0; crossFade(0, epoch) prepends c(0, 0) and trims the epoch to
    # its first upward zero crossing (R/source.R:386, :420-423)
    e = np.sin(np.linspace(-1, 30, 500))
    out = oracle.cross_fade(np.array([0.0]), e, 44100)
    zc = T.find_zero_crossing(e, 1)
    assert len(out) == 2 + len(e) - zc
    assert out[0] == 0 and out[1] == 0


def test_clumper_example(oracle):
    # soundgen:::clumper(s = c(1,3,2,2,2,0,0,4,4,1,1,1,1,1,3,3), minLength = 3)  R/utilities_math.R:549-554
    s = np.array([1, 3, 2, 2, 2, 0, 0, 4, 4, 1, 1, 1, 1, 1, 3, 3], float)
    out = oracle.clumper(s, 3)
    assert len(out) == len(s)
    runs = np.split(out, np.nonzero(np.diff(out))[0] + 1)
    assert all(len(r) >= 3 for r in runs)


def test_vocal_fry_epochs_example(oracle):
    # getVocalFry(rolloff, pitch_per_gc = c(400, 500, 600, 700), subFreq = 200,
    # subDep = 150, shortestEpoch = 100 / 0), R/subharmonics.R:99-107
    ppg = np.array([400.0, 500, 600, 700])
    R = oracle.get_rolloff(ppg, nHarmonics=20, samplingRate=16000)
    ep, mats = oracle.vocal_fry(R, ppg, subFreq=200, subDep=150, shortestEpoch=100)
    # nSub = round(f0 / subFreq) - 1 = (1, 1, 2, 3); clumper with minLength
    # round(100 / (1000 / f0)) >= 40 > 4 cycles collapses to the median 2
    assert ep == [(1, 4)]
    mult, A = mats[0]
    np.testing.assert_allclose(mult[:3], [1 / 3, 2 / 3, 1.0], rtol=1e-14)
    ep0, mats0 = oracle.vocal_fry(R, ppg, subFreq=200, subDep=150, shortestEpoch=0)
    assert ep0 == [(1, 2), (3, 3), (4, 4)]


PITCHES = {
    "roxygen_200_300": T.seq_len(200, 300, 3500),   # R/source.R:167-172 (linear getSmoothContour)
    "flat_110": np.full(3500, 110.0),
    "flat_370": np.full(1750, 370.0),
    "sweep": 150 + 100 * np.linspace(0, 1, 3500) ** 2,
}


@pytest.mark.parametrize("name", sorted(PITCHES))
@pytest.mark.parametrize("sr", [16000, 44100])
def test_generate_harmonics_simple_vs_twin(oracle, name, sr):
    p = PITCHES[name]
    kw = dict(samplingRate=sr, temperature=0, nonlinBalance=0)
    got = oracle.generate_harmonics(p, **kw)
    want = T.generate_harmonics_simple(p, sr=sr)
    assert len(got) == len(want)
    assert float(np.sqrt(np.mean((got - want) ** 2))) < 1e-9


def test_istft_stft_vs_numpy(oracle):
    rng = np.random.default_rng(3)
    # odd wl (windowLength_points = floor(L / 2) of a short sound): wl %/% 2 bins,
    # a (wl - 1)-point inverse recycled against the wl-point window, fractional hops
    for wl in (64, 440, 800, 65, 441, 2203):
        nr, nc = wl // 2, 7
        z = rng.normal(size=(nr, nc)) + 1j * rng.normal(size=(nr, nc))
        np.testing.assert_allclose(oracle.istft(z, 75, wl), T.istft(z, 75, wl), rtol=1e-9, atol=1e-12)
        wave = rng.normal(size=wl * 4)
        step = np.arange(1, len(wave) - wl, wl * 0.25, dtype=float)
        np.testing.assert_allclose(oracle.stft(wave, wl, step), T.stft(wave, wl, step), rtol=1e-9, atol=1e-12)


def test_fft_any_length(oracle):
    rng = np.random.default_rng(11)
    for n in (1, 2, 7, 19, 29, 440, 1102, 2204):
        x = rng.normal(size=n) + 1j * rng.normal(size=n)
        np.testing.assert_allclose(oracle.fft(x), np.fft.fft(x), rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(oracle.fft(x, inverse=True), np.fft.ifft(x) * n, rtol=1e-9, atol=1e-9)


def test_loess_vs_twin(oracle):
    """loess restatement (C oracle) vs the independent NumPy twin on random
    3-10 point data and spans; parity vs R itself is unpinned."""
    rng = np.random.default_rng(11)
    checked = 0
    for _ in range(150):
        n = int(rng.integers(3, 11))
        x = np.sort(rng.choice(np.arange(1, 800), n, replace=False)).astype(float)
        y = rng.normal(size=n) * 10
        span = float(rng.uniform(0.45, 1.6))
        z = np.linspace(x[0], x[-1], 61)
        try:
            a = oracle.loess(x, y, span, z)
        except Exception:  # degenerate neighbourhood (nf = 1 at a data point)
            with pytest.raises(FloatingPointError):  # the twin's predict() stops too
                T.loess(x, y, span, z)
            continue
        np.testing.assert_allclose(a, T.loess(x, y, span, z), rtol=0, atol=1e-9 * max(1, np.abs(y).max()))
        checked += 1
    assert checked > 100


@pytest.mark.parametrize("anchors,L,sr,kw", [
    ({"time": [0, .1, .9, 1], "value": [100, 150, 135, 100]}, 1050, 3500, dict(pitch=True, floor=50, ceiling=3500)),
    ({"time": [0, .3, .6, 1], "value": [0, 40, 10, 20]}, 5000, 16000, dict(floor=0)),
    ({"time": [0, 200, 500, 900, 1000], "value": [-30, -10, -40, -20, -25]}, 16000, 16000, dict(floor=-120, ceiling=40)),
    # zero-width neighbourhoods (floor(n span) = 1): R's span + 0.1 retry
    # (R/smoothContours.R:135-143); the vignette's own example
    # (vignettes/sound_generation.Rmd:129-132), 2 s: span 0.518 -> 0.718
    ({"time": [0, .1, 1], "value": [350, 700, 350]}, 7000, 3500, dict(pitch=True, floor=50, ceiling=3500)),
    ({"time": [0, .5, 1], "value": [150, 420, 300]}, 10500, 3500, dict(pitch=True, floor=50, ceiling=3500)),
    ({"time": [0, .2, .7, 1], "value": [90, 250, 180, 120]}, 14000, 3500, dict(pitch=True, floor=50, ceiling=3500)),
])
def test_smooth_contour_loess_vs_twin(oracle, anchors, L, sr, kw):
    a = oracle.smooth_contour(anchors, L, thisIsPitch=kw.get("pitch", False), valueFloor=kw.get("floor"),
                              valueCeiling=kw.get("ceiling"), samplingRate=sr)
    b = T.smooth_contour_loess(anchors["time"], anchors["value"], L, sr, **kw)
    np.testing.assert_allclose(a, b, rtol=1e-11, atol=1e-9)
