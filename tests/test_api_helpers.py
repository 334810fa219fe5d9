"""The exported hot-path helpers of the API mirror (NAMESPACE: getSmoothContour,
crossFade, addVectors; findZeroCrossing is their internal) against the oracle's
restatements (R/smoothContours.R:53-227, R/utilities_soundgen.R:255-375,
R/utilities_math.R:500-525) and the roxygen examples. CPU only: all are host
functions in the reference too."""
import numpy as np
import pytest

from soundgen_beta_amd import api


@pytest.mark.parametrize("case", [
    dict(anchors={"time": [0, .1, .9, 1], "value": [100, 150, 135, 100]}, len=500, thisIsPitch=True),
    dict(anchors={"time": [0, .3, .5, .9, 1], "value": [-20, 0, -5, 3, -30]}, len=777, method="spline"),
    dict(anchors={"time": [0, 1], "value": [1, 5]}, len=10),
    dict(anchors={"time": [0], "value": [3]}, len=7),
    dict(anchors={"time": [0, .2, .4, .6, .8, 1], "value": [0, 5, 2, 9, 1, 4]}, len=300, valueFloor=1,
         valueCeiling=8),
    dict(anchors={"time": [0, 50, 120, 300], "value": [200, 400, 250, 210]}, len=None, thisIsPitch=True,
         samplingRate=16000),
    # len = NULL (R/smoothContours.R:92-96): times in ms, not starting at 0; loess span
    # from the anchors' duration; spline over the raw times
    dict(anchors={"time": [20, 95, 130, 333], "value": [200, 400, 250, 210]}, len=None, samplingRate=22050),
    dict(anchors={"time": [20, 95, 130, 333, 400], "value": [1, 4, 2, 8, 3]}, len=None, method="spline",
         samplingRate=44100),
])
def test_get_smooth_contour_vs_oracle(oracle, case):
    got = api.getSmoothContour(**case)
    want = oracle.smooth_contour(**case)
    assert got is not None and got.shape == want.shape
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-12)


def test_get_smooth_contour_floor_refits_vs_oracle(oracle):
    """Anchors dipping below valueFloor drive the loess refit loop (span / 1.1 while a
    value of 1..len falls below the floor, R/smoothContours.R:144-151): the planner's
    per-cell bound must pick the same span as the oracle's point-by-point test."""
    rng = np.random.default_rng(11)
    n_refit = 0
    for trial in range(300):
        n = int(rng.integers(3, 11))
        t = np.sort(rng.uniform(0, 1, n))
        t[0], t[-1] = 0, 1
        v = rng.normal(0, 3, n) if trial % 2 else rng.uniform(-5, 40, n)
        case = dict(anchors={"time": list(t), "value": list(v)}, len=int(rng.integers(5, 3000)), valueFloor=0.0)
        got = api.getSmoothContour(**case)
        want = oracle.smooth_contour(**case)
        n_refit += bool(np.min(v) < 0)
        assert got.shape == want.shape, trial
        np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-12, err_msg=str(trial))
    assert n_refit > 50


def test_get_smooth_contour_na():
    assert api.getSmoothContour(None, len=100) is None
    assert api.getSmoothContour({"time": [0, 1], "value": [1, 2]}, len=0) is None
    assert api.getSmoothContour({"time": [5, 5], "value": [1, 2]}) is None  # len = NULL, zero duration


def test_get_smooth_contour_len_null_uses_the_anchor_duration(oracle):
    """len = NULL differs from the len it implies: the loess span is taken from
    the anchors' duration, not from floor(duration sr / 1000) / sr (the API used
    to pass the floored len, a rounding deviation from R)."""
    # 365.47 ms: floor(4 span) = 2 from the anchors' duration, 3 from 5847 / 16 kHz
    a = {"time": [0, 137.3, 261.9, 365.47], "value": [3, 9, 1, 4]}
    sr = 16000
    n = int(np.floor(365.47 * sr / 1000))
    null = api.getSmoothContour(a, len=None, samplingRate=sr)
    given = api.getSmoothContour(a, len=n, samplingRate=sr)
    assert len(null) == len(given) == n
    np.testing.assert_allclose(null, oracle.smooth_contour(a, None, samplingRate=sr), rtol=1e-12, atol=1e-12)
    assert not np.allclose(null, given, rtol=0, atol=1e-12)


def test_find_zero_crossing_vs_oracle(oracle):
    a = np.sin(np.arange(1, 101) / 2)  # the roxygen example
    for loc in range(0, 102):
        assert api.findZeroCrossing(a, loc) == oracle.find_zero_crossing(a, loc), loc
    rng = np.random.default_rng(3)
    for _ in range(50):
        b = rng.normal(size=int(rng.integers(1, 40)))
        for loc in range(1, b.size + 1):
            assert api.findZeroCrossing(b, loc) == oracle.find_zero_crossing(b, loc)


def test_cross_fade_vs_oracle(oracle):
    rng = np.random.default_rng(7)
    for n1, n2, sr in [(300, 400, 16000), (1000, 50, 44100), (5, 8, 16000), (2000, 2000, 8000)]:
        a1 = np.sin(np.arange(n1) / 7.0) + 0.1 * rng.normal(size=n1)
        a2 = np.sin(np.arange(n2) / 5.0 + 1) + 0.1 * rng.normal(size=n2)
        got = api.crossFade(a1, a2, sr)
        want = oracle.cross_fade(a1, a2, sr)
        assert got.shape == want.shape
        np.testing.assert_array_equal(got, want)


def test_add_vectors_roxygen_examples():
    v1, v2, v3 = np.arange(1, 7.0), np.full(3, 100.0), np.full(15, 100.0)
    # insertionPoint > 1 pads v2 with insertionPoint zeros (R/utilities_math.R:507-510)
    np.testing.assert_array_equal(api.addVectors(v1, v2, 5), [1, 2, 3, 4, 5, 106, 100, 100])
    np.testing.assert_array_equal(api.addVectors(v1, v2, -4), [100, 100, 100, 0, 0, 1, 2, 3, 4, 5, 6])
    np.testing.assert_array_equal(api.addVectors(v2, v1, -4), [1, 2, 3, 4, 5, 106, 100, 100])
    assert api.addVectors(v1, v3, -4).size == 15
    np.testing.assert_array_equal(api.addVectors(v2, v3, 7)[:10], [100, 100, 100, 0, 0, 0, 0, 100, 100, 100])
    np.testing.assert_array_equal(api.addVectors([1, np.nan], [np.nan, 2], 1), [1, 2])
