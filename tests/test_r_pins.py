"""R-computed values held by the reference's vendored test suites pin the R-base
numerics the oracle, the host planner and the NumPy twin restate
(tests/golden/r_pins.json, built by tests/golden/make_r_fixtures.py):

- signal_0.7-6 savedTests.Rdata: interp1 'spline' = splinefun(x, y) (FMM, the
  spline behind upsample R/utilities_soundgen.R:410, jitter R/source.R:285,
  random walks R/utilities_math.R:318 and contours R/smoothContours.R:117);
  interp1 'linear' (approx's formula, R/source.R:403-405); ifft(fft(.)).
- tuneR_1.3.2 tuneRTest.Rout.save: normalize(x1, unit = "16", center = TRUE,
  level = 1, rescale = TRUE), the conversion seewave::savewav applies.
- tuneR Testfiles/16bit_PCM_mono_ex.wav and the reference's own
  inst/shiny/soundgen_main/www/efc0saw1.wav: writeWave's extensible layout.
CPU only; the GPU conversion is pinned in test_wav.py against the same values."""
import base64
import json
import math
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

import np_twin

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "soundgen_beta_amd", "csrc")
PINS = json.load(open(os.path.join(HERE, "golden", "r_pins.json")))
SIG = PINS["signal"]
SPLINE = sorted(k for k, v in SIG.items() if v.get("method") == "spline")
LINEAR = sorted(k for k, v in SIG.items() if v.get("method") == "linear")


def _in_range(c):
    x, xi = np.asarray(c["x"]), np.asarray(c["xi"], float)
    return (xi >= x.min()) & (xi <= x.max())


def _close(got, want, rtol=1e-14, atol=1e-15):
    got, want = np.asarray(got, float), np.asarray(want, float)
    return np.all(np.abs(got - want) <= atol + rtol * np.abs(want)), int(np.sum(got == want))


@pytest.mark.parametrize("name", SPLINE)
def test_oracle_fmm_spline_vs_r(oracle, name):
    """splinefun(x, y)(xi) as R computed it; extrapolated points (Test142) use
    the last knot's cubic, as stats' spline_eval does."""
    c = SIG[name]
    want = np.asarray(c["R"], float)
    keep = ~np.isnan(want)
    got = oracle.spline_at(c["x"], c["y"], np.asarray(c["xi"], float)[keep])
    ok, exact = _close(got, want[keep])
    assert ok, (name, np.max(np.abs(got - want[keep])))
    print(name, "bit-exact", exact, "of", int(keep.sum()))


@pytest.mark.parametrize("name", LINEAR)
def test_oracle_approx_vs_r_linear(oracle, name):
    """interp1 'linear' inside [x1, xn] computes approx's y_i + dy (v - x_i) / dx."""
    c = SIG[name]
    want = np.asarray(c["R"], float)
    keep = _in_range(c) & ~np.isnan(want)
    got = oracle.approx_at(c["x"], c["y"], np.asarray(c["xi"], float)[keep])
    ok, exact = _close(got, want[keep])
    assert ok, (name, np.max(np.abs(got - want[keep])))
    # outside the range approx(rule = 1) gives NA, as interp1 without extrap does
    out = ~_in_range(c)
    if out.any() and not c["extrap"]:
        assert np.isnan(oracle.approx_at(c["x"], c["y"], np.asarray(c["xi"], float)[out])).all()
        assert np.isnan(want[out]).all()


def test_twin_fmm_spline_vs_r():
    """The NumPy twin's FMM coefficients reproduce R's splinefun values."""
    for name in SPLINE:
        c = SIG[name]
        x, y = np.asarray(c["x"], float), np.asarray(c["y"], float)
        want = np.asarray(c["R"], float)
        xi = np.asarray(c["xi"], float)
        keep = ~np.isnan(want)
        b, cc, d = np_twin.fmm_coef(x, y)
        i = np.clip(np.searchsorted(x, xi[keep], side="right") - 1, 0, len(x) - 1)
        dx = xi[keep] - x[i]
        got = y[i] + dx * (b[i] + dx * (cc[i] + dx * d[i]))
        ok, _ = _close(got, want[keep], rtol=1e-13, atol=1e-14)
        assert ok, (name, np.max(np.abs(got - want[keep])))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_planner_rmath_vs_r(tmp_path):
    """The host planner's fmm_spline / Spline::eval and approx1 (sg_rmath.h,
    compiled with g++) against R's values."""
    exe = str(tmp_path / "rmath_pins")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I" + CSRC, "-I" + os.path.join(HERE, "..", "include"),
                    os.path.join(HERE, "cpp", "rmath_pins.cpp"), os.path.join(CSRC, "sg_scratch.cpp"), "-o", exe], check=True, timeout=300)
    lines, keys = [], []
    for name in SPLINE + LINEAR:
        c = SIG[name]
        want = np.asarray(c["R"], float)
        keep = ~np.isnan(want) if name in SPLINE else (_in_range(c) & ~np.isnan(want))
        xi = np.asarray(c["xi"], float)[keep]
        f = lambda v: " ".join(repr(float(t)) for t in v)  # noqa: E731
        lines.append("%s %d %s %s %d %s" % ("S" if name in SPLINE else "L", len(c["x"]), f(c["x"]), f(c["y"]),
                                            len(xi), f(xi)))
        keys.append((name, want[keep]))
    r = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    outs = r.stdout.strip().split("\n")
    assert len(outs) == len(keys)
    for (name, want), line in zip(keys, outs):
        got = np.array([float(v) for v in line.split()])
        ok, _ = _close(got, want)
        assert ok, (name, np.max(np.abs(got - want)))


@pytest.mark.parametrize("name", ["Test136", "Test137", "Test138"])
def test_oracle_fft_vs_r(oracle, name):
    """R's fft (any n, unnormalised, +i inverse): ifft(fft(a) * fft(b)) / n."""
    c = SIG[name]
    a = np.asarray(c["a"], complex)
    fa = oracle.fft(a)
    prod = fa * oracle.fft(np.asarray(c["b"], complex)) if c["b"] else fa
    got = oracle.fft(prod, inverse=True) / len(a)
    want = np.asarray(c["R_re"]) + 1j * np.asarray(c["R_im"])
    assert np.max(np.abs(got - want)) <= 4e-15, (name, got, want)


def _x1():
    """tuneR sine(660, pcm = TRUE, bit = 8, duration = 500) (tuneRTest.R:4)."""
    s = np.array([math.sin(2 * math.pi * 660 * k / 44100) for k in range(500)])
    m = np.max(np.abs(s))
    return np.rint(1 * s / m * 127 + 127)


def test_savewav_restatement_vs_r(oracle):
    """savewav(x1) = normalize(x1, "16", level = 1, rescale = TRUE) since max(x1) > 1
    (seewave.r:5220-5223): the first 10 samples R printed."""
    got = oracle.savewav_pcm(_x1())
    assert list(got[:10]) == PINS["tuneR"]["x13_normalize16_rescale"]


def test_savewav_norescale_vs_r():
    """normalize(x1, "16", rescale = FALSE): m = 128 for an 8-bit Wave (tuneR
    normalize.R) -- restated here only to confirm the input x1 itself."""
    x = _x1()
    xc = x - math.fsum(x) / len(x)
    got = np.rint(1 * xc / 128 * 32767).astype(int)
    assert list(got[:10]) == PINS["tuneR"]["x14_normalize16_norescale"]


def test_wav_writer_vs_tuner_file(tmp_path):
    """tuneR's own writeWave(extensible = TRUE) file, byte for byte: its samples
    written by sg_wav_write reproduce the whole file."""
    from soundgen_beta_amd import api
    raw = base64.b64decode(PINS["wav"]["16bit_PCM_mono_ex.wav"])
    sr = struct.unpack("<i", raw[24:28])[0]
    pcm = np.frombuffer(raw[80:], "<i2")
    p = str(tmp_path / "t.wav")
    api.write_wav(p, pcm, sr)
    assert open(p, "rb").read() == raw


def test_wav_header_vs_reference_shiny_file(tmp_path):
    """The header seewave::savewav wrote for the reference's own
    inst/shiny/soundgen_main/www/efc0saw1.wav equals ours for the same length and rate."""
    from soundgen_beta_amd import api
    h = base64.b64decode(PINS["wav"]["efc0saw1.wav"]["header"])
    size = PINS["wav"]["efc0saw1.wav"]["size"]
    sr = struct.unpack("<i", h[24:28])[0]
    n = (size - 80) // 2
    p = str(tmp_path / "s.wav")
    api.write_wav(p, np.zeros(n, np.int16), sr)
    assert open(p, "rb").read()[:80] == h
