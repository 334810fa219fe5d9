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
