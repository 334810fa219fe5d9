"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the CPU oracle
(oracle/_build/libsg_oracle.so, built from oracle/sg_oracle.c by oracle/Makefile).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module. The product path (soundgen_beta_amd) never does.
Parity status: see the header of sg_oracle.c ("parity unpinned" vs R).
"""
import ctypes as C
import os
import subprocess

import numpy as np

from soundgen_beta_amd import _abi, rargs

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.environ.get("SG_ORACLE_LIB") or os.path.join(_HERE, "_build", "libsg_oracle.so")  # override: sanitizer build
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        dp = C.POINTER(C.c_double)
        dpp = C.POINTER(dp)
        i64 = C.c_int64
        i64p = C.POINTER(C.c_int64)
        L.or_last_error.restype = C.c_char_p
        L.or_free.argtypes = [C.c_void_p]
        L.or_generate_harmonics.argtypes = [dp, i64, C.POINTER(_abi.sg_harm_params), _abi.sg_anchors,
                                            C.POINTER(_abi.sg_random), dpp, i64p]
        L.or_soundgen.argtypes = [C.POINTER(_abi.sg_soundgen_args), C.POINTER(_abi.sg_random), dpp, i64p]
        L.or_generate_noise.argtypes = [i64, _abi.sg_anchors, C.c_double, C.c_double, C.c_int32, C.c_double,
                                        C.c_double, C.c_double, dp, C.c_int32, C.POINTER(_abi.sg_random), dpp]
        L.or_spectral_envelope.argtypes = [C.c_int32, C.c_int32, C.POINTER(_abi.sg_formants), C.c_double,
                                           C.c_double, _abi.sg_anchors, C.c_double, C.c_double, C.c_double,
                                           C.c_double, C.c_double, C.c_double, C.c_double, C.c_double,
                                           C.c_double, C.c_double, C.POINTER(_abi.sg_random), dp]
        L.or_formant_filter.argtypes = [dp, i64, dp, C.c_int32, C.c_int32, C.c_double, dpp, i64p]
        L.or_istft.argtypes = [dp, dp, i64, i64, C.c_double, i64, dpp, i64p]
        L.or_stft.argtypes = [dp, i64, i64, dp, i64, dp, dp]
        L.or_fft.argtypes = [dp, dp, i64, C.c_int, dp, dp]
        L.or_get_rolloff.argtypes = [dp, C.c_int32, C.c_int32] + [C.c_double] * 9 + [dp, C.POINTER(C.c_int32)]
        L.or_glottal_cycles.argtypes = [dp, i64, C.c_double, dp]
        L.or_glottal_cycles.restype = i64
        L.or_spline.argtypes = [dp, dp, i64, i64, dp]
        L.or_approx.argtypes = [dp, dp, i64, i64, dp]
        L.or_spline_at.argtypes = [dp, dp, i64, dp, i64, dp]
        L.or_approx_at.argtypes = [dp, dp, i64, dp, i64, dp]
        L.or_find_zero_crossing.argtypes = [dp, i64, i64]
        L.or_find_zero_crossing.restype = i64
        L.or_clumper.argtypes = [dp, i64, dp, i64]
        L.or_cross_fade.argtypes = [dp, i64, dp, i64, C.c_double, C.c_double, dp]
        L.or_cross_fade.restype = i64
        L.or_vocal_fry_epochs.argtypes = [dp, i64, dp, i64, C.c_double, C.c_double, C.c_double, C.c_double,
                                          i64p, i64p, i64p, i64, dp, dp]
        L.or_smooth_contour.argtypes = [dp, dp, i64, i64, C.c_int, C.c_int, C.c_int, C.c_double, C.c_int,
                                        C.c_double, C.c_double, dp]
        L.or_loess.argtypes = [dp, dp, C.c_int, C.c_double, dp, i64, dp]
        _lib = L
    return _lib


class OracleError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s: %s" % (_abi.SG_ERR_NAMES.get(code, code), msg))
        self.code = code


def _check(rc):
    if rc < 0:
        raise OracleError(rc, lib().or_last_error().decode())
    return rc


def _take(ptr, n):
    a = np.ctypeslib.as_array(ptr, shape=(n,)).copy() if n > 0 else np.zeros(0)
    lib().or_free(ptr)
    return a


def _f64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


def generate_harmonics(pitch, amplAnchors=None, normals=None, uniforms=None, rng=None, **kw):
    h = rargs.Holder()
    p = rargs.fill_harm_params(kw)
    pitch = h.arr(pitch)
    rnd = h.random(normals, uniforms, rng)
    out = C.POINTER(C.c_double)()
    n = C.c_int64()
    _check(lib().or_generate_harmonics(_abi.dptr(pitch), len(pitch), C.byref(p),
                                        h.anchors(rargs.as_anchors(amplAnchors)), C.byref(rnd),
                                        C.byref(out), C.byref(n)))
    return _take(out, n.value)


def soundgen(normals=None, uniforms=None, rng=None, **kw):
    h = rargs.Holder()
    a = rargs.fill_soundgen_args(h, kw)
    rnd = h.random(normals, uniforms, rng)
    out = C.POINTER(C.c_double)()
    n = C.c_int64()
    _check(lib().or_soundgen(C.byref(a), C.byref(rnd), C.byref(out), C.byref(n)))
    return _take(out, n.value)


def generate_noise(len, noiseAnchors, rolloffNoise=-6, attackLen=10, windowLength_points=1024,
                   samplingRate=16000, overlap=75, throwaway=-120, filterNoise=None, uniforms=None, rng=None):
    h = rargs.Holder()
    rnd = h.random(None, uniforms, rng)
    fn, fnc = None, 0
    if filterNoise is not None:
        filterNoise = np.asarray(filterNoise, dtype=np.float64)
        if filterNoise.ndim == 1:
            filterNoise = filterNoise[:, None]
        fnc = filterNoise.shape[1]
        fn = h.arr(filterNoise.T.ravel())  # column-major
    out = C.POINTER(C.c_double)()
    _check(lib().or_generate_noise(int(len), h.anchors(rargs.as_anchors(noiseAnchors)), rolloffNoise,
                                   attackLen, int(windowLength_points), samplingRate, overlap, throwaway,
                                   _abi.dptr(fn), fnc, C.byref(rnd), C.byref(out)))
    return _take(out, int(len))


def spectral_envelope(nr, nc, formants=None, formantDep=1, rolloffLip=6, mouthAnchors=None,
                      mouthOpenThres=0, openMouthBoost=0, vocalTract=None, temperature=0, formDrift=.3,
                      formDisp=.2, formantDepStoch=30, smoothLinearFactor=1, samplingRate=16000,
                      speedSound=35400, normals=None, uniforms=None, rng=None):
    h = rargs.Holder()
    F = h.formants(rargs.as_formants(formants))
    rnd = h.random(normals, uniforms, rng)
    out = np.zeros(nr * nc)
    vt = float("nan") if vocalTract is None else float(vocalTract)
    _check(lib().or_spectral_envelope(nr, nc, C.byref(F), formantDep, rolloffLip,
                                      h.anchors(rargs.as_anchors(mouthAnchors)), mouthOpenThres,
                                      openMouthBoost, vt, temperature, formDrift, formDisp,
                                      formantDepStoch, smoothLinearFactor, samplingRate, speedSound,
                                      C.byref(rnd), _abi.dptr(out)))
    return out.reshape(nc, nr).T  # nr x nc


def formant_filter(sound, env, windowLength_points, overlap=75):
    sound = _f64(sound)
    env = np.asarray(env, dtype=np.float64)
    if env.ndim == 1:
        env = env[:, None]
    envc = _f64(env.T.ravel())
    out = C.POINTER(C.c_double)()
    n = C.c_int64()
    _check(lib().or_formant_filter(_abi.dptr(sound), len(sound), _abi.dptr(envc), env.shape[1],
                                   int(windowLength_points), overlap, C.byref(out), C.byref(n)))
    return _take(out, n.value)


def istft(z, ovlp, wl):
    z = np.asarray(z)
    nr, nc = z.shape
    re = _f64(np.real(z).T.ravel())
    im = _f64(np.imag(z).T.ravel())
    out = C.POINTER(C.c_double)()
    n = C.c_int64()
    _check(lib().or_istft(_abi.dptr(re), _abi.dptr(im), nr, nc, ovlp, wl, C.byref(out), C.byref(n)))
    return _take(out, n.value)


def stft(wave, wl, step):
    wave = _f64(wave)
    step = _f64(step)
    nr, nc = wl // 2, len(step)
    re, im = np.zeros(nr * nc), np.zeros(nr * nc)
    _check(lib().or_stft(_abi.dptr(wave), len(wave), wl, _abi.dptr(step), nc, _abi.dptr(re), _abi.dptr(im)))
    return (re + 1j * im).reshape(nc, nr).T


def fft(x, inverse=False):
    x = np.asarray(x, dtype=np.complex128)
    re, im = _f64(x.real), _f64(x.imag)
    ore, oim = np.zeros(len(x)), np.zeros(len(x))
    lib().or_fft(_abi.dptr(re), _abi.dptr(im), len(x), int(inverse), _abi.dptr(ore), _abi.dptr(oim))
    return ore + 1j * oim


def get_rolloff(pitch_per_gc, nHarmonics=100, rolloff=-12, rolloffOct=-2, rolloffParab=0,
                rolloffParabHarm=2, rolloffKHz=-6, baseline=200, throwaway=-120, samplingRate=16000,
                rolloffParabCeiling=None):
    p = _f64(np.atleast_1d(pitch_per_gc))
    out = np.zeros(nHarmonics * len(p))
    rows = C.c_int32()
    ceil = float("nan") if rolloffParabCeiling is None else float(rolloffParabCeiling)
    _check(lib().or_get_rolloff(_abi.dptr(p), len(p), nHarmonics, rolloff, rolloffOct, rolloffParab,
                                rolloffParabHarm, ceil, rolloffKHz, baseline, throwaway, samplingRate,
                                _abi.dptr(out), C.byref(rows)))
    H = rows.value
    return out[:H * len(p)].reshape(len(p), H).T


def glottal_cycles(pitch, samplingRate):
    p = _f64(pitch)
    out = np.zeros(len(p) + 1)
    n = lib().or_glottal_cycles(_abi.dptr(p), len(p), samplingRate, _abi.dptr(out))
    return out[:n].astype(np.int64)


def spline(x, y, n):
    x, y = _f64(x), _f64(y)
    out = np.zeros(n)
    lib().or_spline(_abi.dptr(x), _abi.dptr(y), len(x), n, _abi.dptr(out))
    return out


def approx(x, y, n):
    x, y = _f64(x), _f64(y)
    out = np.zeros(n)
    _check(lib().or_approx(_abi.dptr(x), _abi.dptr(y), len(x), n, _abi.dptr(out)))
    return out


def spline_at(x, y, u):
    """splinefun(x, y, method = "fmm")(u)."""
    x, y, u = _f64(x), _f64(y), _f64(u)
    out = np.zeros(len(u))
    lib().or_spline_at(_abi.dptr(x), _abi.dptr(y), len(x), _abi.dptr(u), len(u), _abi.dptr(out))
    return out


def approx_at(x, y, v):
    """approx(x, y, xout = v)$y (linear, rule = 1: NaN outside [x1, xn])."""
    x, y, v = _f64(x), _f64(y), _f64(v)
    out = np.zeros(len(v))
    lib().or_approx_at(_abi.dptr(x), _abi.dptr(y), len(x), _abi.dptr(v), len(v), _abi.dptr(out))
    return out


def find_zero_crossing(a, location):
    a = _f64(a)
    r = lib().or_find_zero_crossing(_abi.dptr(a), len(a), int(location))
    return None if r == 0 else int(r)


def clumper(s, minLength):
    s = _f64(s).copy()
    ml = _f64(np.atleast_1d(minLength))
    lib().or_clumper(_abi.dptr(s), len(s), _abi.dptr(ml), len(ml))
    return s


def cross_fade(a1, a2, samplingRate, crossLen=15):
    a1, a2 = _f64(a1), _f64(a2)
    out = np.zeros(len(a1) + len(a2) + 2)
    n = lib().or_cross_fade(_abi.dptr(a1), len(a1), _abi.dptr(a2), len(a2), samplingRate, crossLen,
                            _abi.dptr(out))
    return out[:n]


def vocal_fry(rolloff, pitch_per_gc, subFreq=100, subDep=100, throwaway=-120, shortestEpoch=300):
    """getVocalFry() with scalar subFreq/subDep: returns (epochs, [(mult, A)])."""
    R = np.asarray(rolloff, dtype=np.float64)
    H, G = R.shape
    Rc = _f64(R.T.ravel())
    p = _f64(pitch_per_gc)
    me = 4096
    st, en, nr = (np.zeros(me, dtype=np.int64) for _ in range(3))
    mult = np.zeros(H * 64 * 8 + 16)
    amp = np.zeros(H * 64 * G * 8 + 16)
    i64p = C.POINTER(C.c_int64)
    ne = _check(lib().or_vocal_fry_epochs(_abi.dptr(Rc), H, _abi.dptr(p), G, subFreq, subDep, throwaway,
                                          shortestEpoch, st.ctypes.data_as(i64p), en.ctypes.data_as(i64p),
                                          nr.ctypes.data_as(i64p), me, _abi.dptr(mult), _abi.dptr(amp)))
    res, mo, ao = [], 0, 0
    for e in range(ne):
        k, g = int(nr[e]), int(en[e] - st[e] + 1)
        res.append((mult[mo:mo + k].copy(), amp[ao:ao + k * g].reshape(g, k).T.copy()))
        mo += k
        ao += k * g
    return list(zip(st[:ne].tolist(), en[:ne].tolist())), res


def smooth_contour(anchors, len, thisIsPitch=False, method="loess", valueFloor=None, valueCeiling=None,
                   samplingRate=16000):
    """getSmoothContour(anchors, len, ...) (R/smoothContours.R:53-227)."""
    t = _f64(anchors["time"])
    v = _f64(anchors["value"])
    # len None: R's len = NULL (times in ms, len = floor(duration_ms sr / 1000))
    n_out = int(np.floor((t.max() - t.min()) * samplingRate / 1000)) if len is None else int(len)
    out = np.zeros(max(n_out, 0))
    _check(lib().or_smooth_contour(_abi.dptr(t), _abi.dptr(v), t.size, -1 if len is None else n_out,
                                   int(bool(thisIsPitch)),
                                   0 if method == "loess" else 1, int(valueFloor is not None),
                                   float(valueFloor or 0.0), int(valueCeiling is not None),
                                   float(valueCeiling or 0.0), float(samplingRate), _abi.dptr(out)))
    return out


def loess(x, y, span, z):
    """loess(y ~ x, span = span) then predict at z (R 3.4 stats defaults, 1-D)."""
    x, y, z = _f64(x), _f64(y), _f64(z)
    out = np.zeros(len(z))
    _check(lib().or_loess(_abi.dptr(x), _abi.dptr(y), len(x), float(span), _abi.dptr(z), len(z), _abi.dptr(out)))
    return out


def savewav_pcm(wave, rescale=None):
    """The 16-bit samples seewave::savewav writes (seewave.r:5192-5229 ->
    tuneR::normalize(unit = "16", level), tuneR/R/normalize.R; or seewave::rescale
    + writeWave's as.integer), restated in numpy float64. mean() is R's
    long-double mean; here the exact sum (math.fsum) divided by n."""
    import math
    x = np.asarray(wave, dtype=np.float64)
    if rescale is not None:
        nrange = rescale[1] - rescale[0]
        y = (x - x.min()) * nrange / (x.max() - x.min()) - nrange / 2
        return np.trunc(y).astype(np.int16)
    mx = float(x.max())
    level = mx if mx <= 1 else 1.0
    xc = x - math.fsum(x) / len(x)
    m = max(abs(float(xc.min())), abs(float(xc.max())))
    if m > 1.5e-8:
        xc = level * xc / m
    return np.rint(xc * 32767).astype(np.int16)
