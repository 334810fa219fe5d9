"""Builds tests/golden/r_pins.json: R-computed values that the reference's own
vendored test suites hold, used to pin the oracle's R-base numerics.

Sources (read as data from the vendored tarballs; nothing is executed):
- packrat/src/signal/signal_0.7-6.tar.gz::signal/tests/savedTests.Rdata with the
  inputs of signal/tests/signal.R:4-26 (regenerated here with the platform libm,
  as R does):
    Test136-138  ifft(fft(.))                        R base fft, any n (signal/R/filter.R:183)
    Test141/146/150/154/158/162/169/180/181
                 interp1(., 'linear')                 s * dy + y (signal/R/interp1.R)
    Test142/147/151/155/159/163/171/176/179
                 interp1(., 'spline') = splinefun(x, y)(xi), method "fmm" (stats splines.c)
- packrat/src/tuneR/tuneR_1.3.2.tar.gz::tuneR/tests/tuneRTest.Rout.save:325-326, 337-338:
  the printed first 10 samples of normalize(x1, unit = "16", center = TRUE,
  level = 1, rescale = TRUE / FALSE), x1 = sine(660, pcm = TRUE, bit = 8,
  duration = 500) (tuneRTest.R:4). rescale = TRUE is the conversion
  seewave::savewav applies (seewave.r:5220-5223) when max(wave) > 1.
- tuneR/tests/Testfiles/16bit_PCM_mono_ex.wav (writeWave(extensible = TRUE)
  output, kept whole: 4,080 bytes) and the header of the reference's
  inst/shiny/soundgen_main/www/efc0saw1.wav (written by seewave::savewav).

    python tests/golden/make_r_fixtures.py [/root/reference]
"""
import base64
import io
import json
import math
import os
import sys
import tarfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "tools"))

LINEAR = [141, 146, 150, 154, 158, 162, 169, 180, 181]
SPLINE = [142, 147, 151, 155, 159, 163, 171, 176, 179]
FFT = [136, 137, 138]


def r_seq_len(a, b, n):
    """seq(a, b, length.out = n): from, from + i * by, to (R's seq.default)."""
    if n == 1:
        return [a]
    by = (b - a) / (n - 1)
    return [a] + [a + i * by for i in range(1, n - 1)] + [b]


def r_seq_by(a, b, by):
    n = int((b - a) / by + 1e-10)
    return [a + i * by for i in range(n + 1)]


def sinv(v):
    return [math.sin(x) for x in v]


def signal_inputs():
    """signal/tests/signal.R:9-22 (only the vectors the interp1 tests use)."""
    x9 = sinv([2 * math.pi * k / 5 for k in range(11)])
    x10 = r_seq_len(0.0, 11.0, 500)
    x12 = [0.0, 4.0, 5.0, 6.0, 8.0, 10.0]
    x13 = sinv([2 * math.pi * t / 5 for t in r_seq_len(0.0, 10.0, 500)])
    x16 = [float(k) for k in list(range(0, 5)) + list(range(6, 11))]
    x17 = [float(k) for k in list(range(0, 2)) + list(range(3, 11))]
    x18 = sinv([2 * math.pi * k / 5 for k in range(6)])
    x20 = sinv([2 * math.pi * t / 5 for t in r_seq_by(0.0, 10.0, 0.05)])
    x21 = r_seq_by(1.0, 4.0, 2.0)
    r010 = [float(k) for k in range(11)]
    r05 = [float(k) for k in range(6)]

    def f(xs):
        return sinv([2 * math.pi * x / 5 for x in xs])

    # (x, y, xi, extrap) per test, signal.R:200-240
    cases = {
        141: (r010, x9, x10, True), 142: (r010, x9, x10, True),
        146: (x12, f(x12), x13, False), 147: (x12, f(x12), x13, False),
        150: (x16, f(x16), x13, False), 151: (x16, f(x16), x13, False),
        154: (r010, x9, x13, False), 155: (r010, x9, x13, False),
        158: (x17, f(x17), x13, False), 159: (x17, f(x17), x13, False),
        162: (r010, x9, x20, False), 163: (r010, x9, x20, False),
        169: (r05, x18, r05, False), 171: (r05, x18, r05, False),
        176: ([1.0, 2.0, 3.0], [1.0, 2.0, 3.0], [1.4], False),
        179: ([1.0, 3.0, 5.0], [1.0, 3.0, 5.0], [1.4], False),
        180: (x21, x21, [0.0, 1.0, 1.4, 3.0, 4.0], False),
        181: ([1.0, 2.0], [1.0, 2.0], [1.4], False),
    }
    return cases


def _member(tar_path, name):
    with tarfile.open(tar_path) as t:
        return t.extractfile(name).read()


def main(ref="/root/reference"):
    from read_rda import read_rda
    import tempfile
    sig = os.path.join(ref, "packrat/src/signal/signal_0.7-6.tar.gz")
    tun = os.path.join(ref, "packrat/src/tuneR/tuneR_1.3.2.tar.gz")
    with tempfile.NamedTemporaryFile(suffix=".Rdata") as tf:
        tf.write(_member(sig, "signal/tests/savedTests.Rdata"))
        tf.flush()
        saved = read_rda(tf.name)
    out = {"source": __doc__.split("\n\n")[0], "signal": {}, "tuneR": {}, "wav": {}}
    cases = signal_inputs()
    for k in LINEAR + SPLINE:
        x, y, xi, extrap = cases[k]
        want = saved["savedTest%d" % k]
        if isinstance(want, dict):
            want = want["values"]
        out["signal"]["Test%d" % k] = {"method": "linear" if k in LINEAR else "spline", "x": x, "y": y, "xi": xi,
                                       "extrap": extrap, "R": want}
    ffts = {136: ([1, 2, 3, 4], None), 137: ([1, 2, 3, 0], [1, 2, 0, 0]), 138: ([1, -2, 0], [1, 2, 0])}
    for k in FFT:
        a, b = ffts[k]
        want = saved["savedTest%d" % k]
        out["signal"]["Test%d" % k] = {"method": "ifft(fft(a) * fft(b))" if b else "ifft(fft(a))", "a": a, "b": b,
                                       "R_re": [z.real for z in want], "R_im": [z.imag for z in want]}
    rout = _member(tun, "tuneR/tests/tuneRTest.Rout.save").decode().splitlines()

    def printed(tag):
        i = next(j for j, l in enumerate(rout) if l.startswith("> %s@left[1:10]" % tag))
        return [int(v) for v in rout[i + 1].split()[1:]]
    out["tuneR"] = {
        "x1": "sine(660, pcm = TRUE, bit = 8, duration = 500): round(sin(2 pi 660 (0:499) / 44100) / m * 127 + 127), "
              "m = max|sin| (tuneR/R/Waveforms.R:39-47, postWaveform :17-27, normalize.R)",
        "x13_normalize16_rescale": printed("x13"),
        "x14_normalize16_norescale": printed("x14"),
        "lines": "tuneRTest.Rout.save:325-326, :337-338",
    }
    wav = _member(tun, "tuneR/tests/Testfiles/16bit_PCM_mono_ex.wav")
    out["wav"]["16bit_PCM_mono_ex.wav"] = base64.b64encode(wav).decode()
    shiny = open(os.path.join(ref, "inst/shiny/soundgen_main/www/efc0saw1.wav"), "rb").read()
    out["wav"]["efc0saw1.wav"] = {"header": base64.b64encode(shiny[:80]).decode(), "size": len(shiny)}
    dst = os.path.join(HERE, "r_pins.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=0)
    print(dst)


if __name__ == "__main__":
    main(*sys.argv[1:])
