"""The output writer (seewave::savewav as soundgen(savePath = ...) and morph()
call it, R/soundgen.R:856, R/morph.R:205): tuneR::writeWave's file layout (CPU)
and the 16-bit conversion on the GPU vs the numpy restatement of
tuneR::normalize / seewave::rescale (oracle.savewav_pcm), sample for sample."""
import os
import struct

import numpy as np
import pytest


def _expected_file(pcm, sr):
    """tuneR::writeWave(extensible = TRUE) of a mono 16-bit Wave, field by field
    (tuneR_1.3.2.tar.gz::tuneR/R/writeWave.R)."""
    n = len(pcm)
    b = n * 2
    h = b"RIFF" + struct.pack("<i", b + 72) + b"WAVE" + b"fmt " + struct.pack("<i", 40)
    h += struct.pack("<hhiihh", -2, 1, sr, sr * 2, 2, 16)  # 65534 as a signed 16-bit write
    h += struct.pack("<hhi", 22, 16, 1) + struct.pack("<h", 1) + bytes([0, 0, 0, 0, 16, 0, 128, 0, 0, 170, 0, 56, 155, 113])
    h += b"fact" + struct.pack("<ii", 4, n) + b"data" + struct.pack("<i", b)
    return h + np.asarray(pcm, "<i2").tobytes()


def test_wav_file_layout(tmp_path):
    from soundgen_beta_amd import api
    pcm = np.array([0, 1, -1, 32767, -32768, 12345], dtype=np.int16)
    p = str(tmp_path / "x.wav")
    api.write_wav(p, pcm, 44100)
    assert open(p, "rb").read() == _expected_file(pcm, 44100)
    api.write_wav(p, pcm[:0], 16000)
    assert open(p, "rb").read() == _expected_file(pcm[:0], 16000)


def test_oracle_normalize_known_answer(oracle):
    # x = (0, .5, -.25, 1): mean .3125, max 1 -> level 1; centered extremes -.5625, .6875 -> m = .6875
    got = oracle.savewav_pcm([0, .5, -.25, 1])
    xc = np.array([-.3125, .1875, -.5625, .6875])
    assert list(got) == list(np.rint(1.0 * xc / .6875 * 32767).astype(int))
    assert got[3] == 32767
    # max > 1: level 1; all-equal input: m = 0, no scaling, zeros
    assert list(oracle.savewav_pcm([2.0, 2.0, 2.0])) == [0, 0, 0]
    # level = max(wave) <= 1 scales the peak below full scale
    y = oracle.savewav_pcm([0.0, 0.25, 0.5])
    assert y[2] == round(0.5 * 0.25 / 0.25 * 32767)
    # seewave::rescale(x, -1, 1) then as.integer: values in (-1, 1) truncate to 0, the top to 1
    assert list(oracle.savewav_pcm([0, .3, 1], rescale=(-1, 1))) == [-1, 0, 1]


@pytest.mark.gpu
def test_savewav_pcm_matches_restatement(oracle, tmp_path):
    from soundgen_beta_amd import api
    rng = np.random.default_rng(7)
    waves = [rng.uniform(-1, 1, 20001), 3 * rng.standard_normal(1500), 0.3 * np.sin(np.arange(4410) / 7.0),
             np.full(100, 0.25), np.zeros(64), 1e-9 * rng.standard_normal(500), rng.uniform(-1, 1, 7)]
    for i, w in enumerate(waves):
        p = str(tmp_path / ("w%d.wav" % i))
        got = api.savewav(w, f=16000, filename=p)
        want = oracle.savewav_pcm(w)
        assert np.array_equal(got, want), i
        assert open(p, "rb").read() == _expected_file(want, 16000)
    w = rng.uniform(-1, 1, 3000)
    got = api.savewav(w, f=22050, filename=str(tmp_path / "r.wav"), rescale=(-20000, 20000))
    assert np.array_equal(got, oracle.savewav_pcm(w, rescale=(-20000, 20000)))
    with pytest.raises(Exception):
        api.savewav(w, f=22050, filename=str(tmp_path / "bad.wav"), rescale=(1, 2))


@pytest.mark.gpu
def test_batch_wav_output_matches_restatement(oracle, tmp_path):
    """soundgen(savePath = ...) over a batch: every call's file holds the
    restated 16-bit conversion of that call's synthesized waveform."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from soundgen_beta_amd import batch
    calls = bench.c5_calls(48)
    paths = [str(tmp_path / ("c%d.wav" % i)) for i in range(len(calls))]
    pcm = batch.synthesize_to_wav(calls, paths, 44100)
    ys = batch.synthesize(calls)
    for i, (p, y) in enumerate(zip(pcm, ys)):
        want = oracle.savewav_pcm(np.asarray(y, np.float64))
        assert np.array_equal(p, want), i
        assert open(paths[i], "rb").read() == _expected_file(want, 44100)


@pytest.mark.gpu
def test_savewav_gpu_vs_r_printed(tmp_path):
    """The GPU conversion (sg_pcm_stats + sg_pcm_convert) of tuneR's x1 =
    sine(660, pcm = TRUE, bit = 8, duration = 500) gives the samples R printed for
    normalize(x1, "16", center = TRUE, level = 1, rescale = TRUE)
    (tuneRTest.Rout.save:325-326; tests/golden/r_pins.json), the conversion
    seewave::savewav applies when max(wave) > 1."""
    import json
    import math
    from soundgen_beta_amd import api
    pins = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "r_pins.json")))
    s = np.array([math.sin(2 * math.pi * 660 * k / 44100) for k in range(500)])
    x1 = np.rint(s / np.max(np.abs(s)) * 127 + 127)
    got = api.savewav(x1, f=44100, filename=str(tmp_path / "x1.wav"))
    assert list(got[:10]) == pins["tuneR"]["x13_normalize16_rescale"]
