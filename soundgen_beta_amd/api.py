"""R-level API mirror: soundgen(), generateHarmonics(), getRolloff().

Same names, argument meanings, defaults and error behaviour as the reference
(R/soundgen.R:208, R/source.R:173, R/sourceSpectrum.R:71); every synthesis
runs on the GPU through libsoundgen_hip.so. Random draws are injected
(`normals`, `uniforms`: R's rnorm()/runif() draws in the reference order).
"""
import ctypes as C
import os

import numpy as np

from . import _abi, native, rargs


def _ctx(device):
    return native.default_context(device)


def _run_one(call, device):
    """Plan ONE call once (its draws are consumed once, in the reference order),
    size the output from the plan, execute on the GPU and copy to the host."""
    from . import batch
    ctx = _ctx(device)
    plan = batch.Plan([call], ctx)
    try:
        if plan.status[0] != 0:
            raise native.SoundgenError(int(plan.status[0]), plan.message(0))
        out = np.zeros(max(plan.total, 1))
        native.check(native.lib().sg_execute_to_host(ctx.ptr, plan.ptr, _abi.dptr(out)), ctx.ptr)
        return out[:int(plan.lengths[0])].copy()
    finally:
        plan.close()


def generateHarmonics(pitch, amplAnchors=rargs.NA, normals=None, uniforms=None, rng=None, device=0, **kw):
    """generateHarmonics(pitch, ...) — R/source.R:173-471."""
    return _run_one({"kind": "harmonics", "pitch": np.asarray(pitch, dtype=np.float64), "params": kw,
                     "amplAnchors": amplAnchors, "normals": normals, "uniforms": uniforms, "rng": rng}, device)


def soundgen(normals=None, uniforms=None, rng=None, device=0, **kw):
    """soundgen(...) — R/soundgen.R:208-862. Returns the waveform (float64)."""
    return _run_one({"kind": "soundgen", "args": kw, "normals": normals, "uniforms": uniforms, "rng": rng}, device)


def generateNoise(len, noiseAnchors=None, rolloffNoise=-6, attackLen=10, windowLength_points=1024,
                  samplingRate=16000, overlap=75, throwaway=-120, filterNoise=None, uniforms=None, rng=None,
                  device=0):
    """generateNoise() — R/source.R:57-138 (runif draws injected or from `rng`)."""
    if noiseAnchors is None:
        noiseAnchors = {"time": [0, 300], "value": [-120, -120]}
    h = rargs.Holder()
    rnd = h.random(None, uniforms, rng)
    fn, fnc = None, 0
    if filterNoise is not None:
        filterNoise = np.asarray(filterNoise, dtype=np.float64)
        if filterNoise.ndim == 1:
            filterNoise = filterNoise[:, None]
        fnc = filterNoise.shape[1]
        fn = h.arr(filterNoise.T.ravel())  # column-major nr x nc
    out = np.zeros(int(len))
    ctx = _ctx(device)
    native.check(native.lib().sg_generate_noise(ctx.ptr, int(len), h.anchors(rargs.as_anchors(noiseAnchors)),
                                                rolloffNoise, attackLen, int(windowLength_points), samplingRate,
                                                overlap, throwaway, _abi.dptr(fn), fnc, C.byref(rnd),
                                                _abi.dptr(out)), ctx.ptr)
    return out


def getSpectralEnvelope(nr, nc, formants=None, formantDep=1, rolloffLip=6, mouthAnchors=None, mouthOpenThres=0,
                        openMouthBoost=0, vocalTract=None, temperature=0, formDrift=.3, formDisp=.2,
                        formantDepStoch=30, smoothLinearFactor=1, samplingRate=16000, speedSound=35400,
                        normals=None, uniforms=None, rng=None, device=0):
    """getSpectralEnvelope() — R/sourceSpectrum.R:261-566; returns nr x nc."""
    h = rargs.Holder()
    F = h.formants(rargs.as_formants(formants))
    rnd = h.random(normals, uniforms, rng)
    out = np.zeros(int(nr) * int(nc))
    vt = float("nan") if vocalTract is None else float(vocalTract)
    # tracks and draws on the host, the nr x nc matrix on the GPU (sg_spec_env, fp32)
    ctx = _ctx(device)
    native.check(native.lib().sg_spectral_envelope(ctx.ptr, int(nr), int(nc), C.byref(F), formantDep, rolloffLip,
                                                   h.anchors(rargs.as_anchors(mouthAnchors)), mouthOpenThres,
                                                   openMouthBoost, vt, temperature, formDrift, formDisp,
                                                   formantDepStoch, smoothLinearFactor, samplingRate, speedSound,
                                                   C.byref(rnd), _abi.dptr(out)), ctx.ptr)
    return out.reshape(int(nc), int(nr)).T


def formantFilter(sound, env, windowLength_points, overlap=75, device=0):
    """The formant filter of soundgen(): seewave::stft x env -> istft -> /max
    (R/soundgen.R:743-807). env: nr x nc (nc == 1: stationary)."""
    h = rargs.Holder()
    sound = h.arr(sound)
    env = np.asarray(env, dtype=np.float64)
    if env.ndim == 1:
        env = env[:, None]
    envc = h.arr(env.T.ravel())
    wl = int(windowLength_points)
    cap = len(sound) + 2 * wl
    out = np.zeros(cap)
    n = C.c_int64()
    ctx = _ctx(device)
    native.check(native.lib().sg_formant_filter(ctx.ptr, _abi.dptr(sound), len(sound), _abi.dptr(envc), env.shape[1],
                                                wl, overlap, _abi.dptr(out), cap, C.byref(n)), ctx.ptr)
    return out[:n.value].copy()


def savewav(wave, f=None, filename=None, rescale=None, device=0):
    """seewave::savewav(wave, f, filename, rescale) as soundgen(savePath = ...)
    and morph(savePath = ...) call it (R/soundgen.R:856, R/morph.R:205): the
    16-bit conversion (tuneR::normalize(unit = "16", level = min(max(wave), 1)),
    or seewave::rescale) runs on the GPU in R's fp64 arithmetic, the file is
    tuneR::writeWave's WAVE_FORMAT_EXTENSIBLE layout. Returns the int16 samples."""
    if f is None:
        raise TypeError("savewav(): the sampling rate f is required for a numeric vector")
    if filename is None:
        raise TypeError("savewav(): filename is required (R would deparse the argument name)")
    x = np.ascontiguousarray(np.asarray(wave, dtype=np.float64).ravel())
    pcm = np.zeros(len(x), dtype=np.int16)
    rs = None if rescale is None else np.ascontiguousarray(np.asarray(rescale, dtype=np.float64)[:2])
    ctx = _ctx(device)
    native.check(native.lib().sg_savewav_pcm(ctx.ptr, _abi.dptr(x), len(x), _abi.dptr(rs) if rs is not None else None,
                                             pcm.ctypes.data_as(C.POINTER(C.c_int16))), ctx.ptr)
    write_wav(filename, pcm, f)
    return pcm


def write_wav(filename, pcm, f):
    """The file of tuneR::writeWave(Wave(pcm, samp.rate = f, bit = 16)) (extensible header)."""
    pcm = np.ascontiguousarray(np.asarray(pcm, dtype=np.int16))
    native.check(native.lib().sg_wav_write(os.fsencode(filename), pcm.ctypes.data_as(C.POINTER(C.c_int16)), len(pcm),
                                           int(f)))


def getRolloff(pitch_per_gc=(440,), nHarmonics=100, rolloff=-12, rolloffOct=-2, rolloffParab=0,
               rolloffParabHarm=2, rolloffParabCeiling=None, rolloffKHz=-6, baseline=200, throwaway=-120,
               samplingRate=16000, plot=False):
    """getRolloff() — R/sourceSpectrum.R:71-186 (host helper; H x nGC matrix)."""
    p = np.ascontiguousarray(np.atleast_1d(np.asarray(pitch_per_gc, dtype=np.float64)))
    out = np.zeros(nHarmonics * len(p))
    rows = C.c_int32()
    ceil = float("nan") if rolloffParabCeiling is None else float(rolloffParabCeiling)
    rc = native.lib().sg_get_rolloff(_abi.dptr(p), len(p), nHarmonics, rolloff, rolloffOct, rolloffParab,
                                     rolloffParabHarm, ceil, rolloffKHz, baseline, throwaway, samplingRate,
                                     _abi.dptr(out), C.byref(rows))
    native.check(rc)
    H = rows.value
    return out[:H * len(p)].reshape(len(p), H).T.copy()


def getSmoothContour(anchors=None, len=None, thisIsPitch=False, method="loess", valueFloor=None,
                     valueCeiling=None, samplingRate=16000):
    """getSmoothContour() — R/smoothContours.R:53-227 (exported; host helper through the
    planner's own contour code). anchors: {"time": ..., "value": ...}, a numeric vector
    (time spread over 0..1), or NA/None. len None: anchors' time is the duration in ms
    and len = floor(duration_ms * samplingRate / 1000), the times kept in ms and the
    loess span taken from that duration, as R/smoothContours.R:92-96 does (len = -1
    at the C ABI). Returns a float64 array, or None where R returns NA."""
    an = rargs.as_anchors(anchors)
    if an is None:
        return None
    t, v = an
    cap = int(np.floor((np.max(t) - np.min(t)) * samplingRate / 1000)) if len is None else int(len)
    if cap <= 0:
        return None
    len = -1 if len is None else cap
    h = rargs.Holder()
    s = h.anchors(an)
    out = np.zeros(cap)
    n = C.c_int64()
    L = native.lib()
    rc = L.sg_get_smooth_contour(s, len, int(bool(thisIsPitch)), 1 if method == "spline" else 0,
                                 int(valueFloor is not None), float(valueFloor or 0.0),
                                 int(valueCeiling is not None), float(valueCeiling or 0.0), float(samplingRate),
                                 _abi.dptr(out), C.byref(n))
    native.check(rc)
    return out[:n.value].copy() if n.value else None


def findZeroCrossing(ampl, location):
    """findZeroCrossing(ampl, location) — R/utilities_soundgen.R:255-295: the index
    (1-based) of the upward zero crossing nearest to `location`, None for NA."""
    a = np.asarray(ampl, dtype=np.float64)
    n = a.size
    location = int(location)
    if n < 1 or location < 1 or location > n:
        return None
    if n == 1 and location == 1:
        return location
    zl = zr = None
    i = location
    if location > 1:
        while i > 1:
            if a[i - 1] > 0 and a[i - 2] < 0:
                zl = i - 1
                break
            i -= 1
    if location < n:
        i = location
    while i < n - 1:  # R: i keeps the left search's value when location == len
        if a[i] > 0 and a[i - 1] < 0:
            zr = i
            break
        i += 1
    if zl is None and zr is None:
        return None
    if zl is None:
        return zr
    if zr is None:
        return zl
    return zl if abs(zl - location) <= abs(zr - location) else zr


def crossFade(ampl1, ampl2, samplingRate, crossLen=15, crossLenPoints=None):
    """crossFade() — R/utilities_soundgen.R:328-375: both waveforms cut at their zero
    crossings, then joined by a linear cross-fade over crossLenPoints samples."""
    a1 = np.asarray(ampl1, dtype=np.float64)
    a2 = np.asarray(ampl2, dtype=np.float64)
    zc1 = findZeroCrossing(a1, a1.size)
    if zc1 is not None:
        a1 = np.concatenate([a1[:zc1], [0.0]])
    zc2 = findZeroCrossing(a2, 1)
    if zc2 is not None:
        a2 = a2[zc2:]
    if crossLenPoints is None:
        cl = min(np.floor(crossLen * samplingRate / 1000), a1.size - 1, a2.size - 1)
    else:
        cl = min(crossLenPoints, a1.size - 1, a2.size - 1)
    if cl < 2:
        return np.concatenate([a1, a2])
    cl = int(cl)
    # seq(0, 1, length.out = cl) as R computes it
    multipl = np.arange(cl, dtype=np.float64) * (1.0 / (cl - 1))
    multipl[-1] = 1.0
    idx1 = a1.size - cl
    cross = multipl[::-1] * a1[idx1:] + multipl * a2[:cl]
    return np.concatenate([a1[:idx1], cross, a2[cl:]])


def addVectors(v1, v2, insertionPoint):
    """addVectors() — R/utilities_math.R:500-525 (exported): v2 added into v1 from
    index insertionPoint (1-based, may be <= 0), both zero-padded, NA as 0."""
    a = np.nan_to_num(np.asarray(v1, dtype=np.float64), nan=0.0)
    b = np.nan_to_num(np.asarray(v2, dtype=np.float64), nan=0.0)
    ip = int(insertionPoint)
    if ip > 1:
        b = np.concatenate([np.zeros(ip), b])
    elif ip < 1:
        a = np.concatenate([np.zeros(1 - ip), a])
    d = b.size - a.size
    if d > 0:
        a = np.concatenate([a, np.zeros(d)])
    elif d < 0:
        b = np.concatenate([b, np.zeros(-d)])
    return a + b
