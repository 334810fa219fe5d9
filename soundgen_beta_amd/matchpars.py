"""compareSounds() and a batched matchPars() loop (R/matchPars.R:81-311, :313-416,
getMelSpec :510-560; wigglePars :436-508), the batch drivers SURVEY §8(f) ranks
after morph().

- getMelSpec: tuneR 1.3.2 melfcc(spec_out = TRUE)$aspectrum restated in numpy
  (tuneR_1.3.2.tar.gz::tuneR/R/melfcc.R, powspec.R, audspec.R, fft2melmx.R,
  hz2mel.R, mel2hz.R; signal 0.7-6 specgram.R and hamming.R): pre-emphasis
  0.97, hamming-windowed |FFT|^2 of round(wintime sr) points zero-padded to
  the next power of two, Slaney mel filterbank of 100 windowLength / 20 bands
  (audspec's nfft is (nfreqs - 1) 2, a quirk kept), then soundgen's frame
  stripping (colMeans > 2^(throwaway / 10)) and log01.
- compareSounds: per column cor / cosine / pixel / dtw of the two spectra
  (matchColumns pads the shorter with NA, central), averaged as R does.
- On the GPU (sg_mel.hip, the product path of match_pars): get_mel_spec_gpu and
  compare_sounds_batch run both for a whole generation of candidates in HBM in
  one launch sequence (fp64 FFT frames, mel bands, kept columns, then one
  wavefront per column for cor / cosine / pixel / dtw). The numpy functions
  below (get_mel_spec, compare_sounds) are the host restatement the GPU tests
  compare against.
  dtw: the dtw package's default (symmetric2 steps, Euclidean local distance,
  normalizedDistance = distance / (n + m)) computed by the library
  (sg_dtw_symmetric2); the dtw package is not vendored: parity unpinned.
- matchPars: R's hill climbing -- mutate the parameters (wigglePars, R's RNG
  through rrng.RRng), synthesize, keep a mutant that improves the similarity by
  more than minExpectedDelta, stop after maxIter non-improving candidates in a
  row. Each generation's `pop` mutants are planned and synthesized as ONE GPU
  batch (pop = 1 is R's loop draw for draw). The starting point comes from the
  caller (`init`): R derives it from analyze() / segment() /
  phonTools::findformants(), the acoustic-analysis stack that is out of scope
  (SURVEY §2).
Parity: restated from the sources; no R here, so the similarity values are
checked against hand-derived cases (tests/test_matchpars.py).
"""
import copy
import ctypes as C
import math

import numpy as np

from . import native, rargs, rcall

_PAR_ROUND = ("repeatBout", "nSyl", "rolloffParabHarm")
# permittedValues rows (default, low, high, step) wigglePars reads (R/presets.R:22-79)
_PV = dict(rargs.PERMITTED_VALUES, pitchDeltas=(0, -24, 24, 1))

# the package's `defaults` list (R/presets.R:84-144; data/defaults.rda), the start of
# matchPars (defaults[pars]); duplicated names (samplingRate, windowLength) resolve
# to their first occurrence, as R's `[` does
MATCHPARS_DEFAULTS = dict(
    repeatBout=1, nSyl=1, sylLen=300, pauseLen=200, temperature=0.025, maleFemale=0, creakyBreathy=0,
    nonlinBalance=0, nonlinDep=50, jitterDep=3, jitterLen=1, vibratoFreq=5, vibratoDep=0, shimmerDep=0,
    attackLen=50, rolloff=-12, rolloffOct=-12, rolloffParab=0, rolloffParabHarm=3, rolloffKHz=-6, rolloffLip=6,
    formantDep=1, formantDepStoch=30, vocalTract=15.5, subFreq=100, subDep=100, shortestEpoch=300, amDep=0,
    amFreq=30, amShape=0, rolloffNoise=-14, samplingRate=16000, windowLength=40, windowLength_points=512,
    overlap=75, addSilence=100, pitchFloor=25, pitchCeiling=3500, pitchSamplingRate=3500, throwaway=-120,
    pitchAnchors={"time": [0, .1, .9, 1], "value": [100, 150, 135, 100]},
    pitchAnchorsGlobal={"time": [0, 1], "value": [0, 0]},
    noiseAnchors={"time": [0, 300], "value": [-120, -120]},
    mouthAnchors={"time": [0, 1], "value": [.5, .5]},
    amplAnchors={"time": [0, 1], "value": [120, 120]},
    amplAnchorsGlobal={"time": [0, 1], "value": [120, 120]},
    formants={"f1": {"time": 0, "freq": 860, "amp": 30, "width": 120},
              "f2": {"time": 0, "freq": 1280, "amp": 40, "width": 120},
              "f3": {"time": 0, "freq": 2900, "amp": 25, "width": 200}},
    formantsNoise=None, vowelString=None,
)


# ---------------------------------------------------------------- R draws
class _Draws:
    """R's rnorm / runif / sample / rbinom semantics over an rrng.RRng."""

    def __init__(self, rng):
        self.rng = rng

    def unif(self):
        return float(self.rng.random())

    def rnorm1(self, mean, sd):
        if sd == 0 or not math.isfinite(mean):  # nmath rnorm: no draw
            return float(mean)
        return float(mean + sd * self.rng.standard_normal())

    def unif_index(self, n):  # R 3.4 sample(): floor(n unif_rand())
        return int(math.floor(n * self.unif()))

    def rbinom1(self, p):  # rbinom(1, 1, p), nmath rbinom.c inversion for size 1
        if p == 0:
            return 0
        if p == 1:
            return 1
        u = self.unif()
        return int(u >= 1 - p) if p <= 0.5 else int(u < p)

    def sample_prob1(self, prob):
        """sample(x, 1, prob = prob) (ProbSampleNoReplace after revsort, R 3.4)."""
        tot = float(sum(prob))
        p = [x / tot for x in prob]
        perm = list(range(1, len(p) + 1))
        _revsort(p, perm)
        rT, mass, j = self.unif(), 0.0, 0
        for j in range(len(p) - 1):
            mass += p[j]
            if rT <= mass:
                break
        else:
            j = len(p) - 1
        return perm[j]


def _revsort(a, ib):
    """R's sort.c revsort (heapsort into decreasing order, ties as R orders them)."""
    n = len(a)
    if n <= 1:
        return
    A = [None] + a
    B = [None] + ib
    l, ir = (n >> 1) + 1, n
    while True:
        if l > 1:
            l -= 1
            ra, ii = A[l], B[l]
        else:
            ra, ii = A[ir], B[ir]
            A[ir], B[ir] = A[1], B[1]
            ir -= 1
            if ir == 1:
                A[1], B[1] = ra, ii
                break
        i, j = l, l << 1
        while j <= ir:
            if j < ir and A[j] > A[j + 1]:
                j += 1
            if ra > A[j]:
                A[i], B[i] = A[j], B[j]
                i = j
                j += j
            else:
                j = ir + 1
        A[i], B[i] = ra, ii
    a[:] = A[1:]
    ib[:] = B[1:]


def rnorm_bounded(D, n, mean, sd, low=None, high=None, roundToInteger=False):
    """rnorm_bounded(), R/utilities_math.R:187-231."""
    mean = list(np.atleast_1d(np.asarray(mean, float)))
    sd = list(np.atleast_1d(np.asarray(sd, float)))
    lo = -math.inf if low is None else low
    hi = math.inf if high is None else high
    mean = [min(max(m, lo), hi) for m in mean]
    if len(mean) < n:
        mean = [mean[0]] * n
    if len(sd) < n:
        sd = [sd[0]] * n
    rnd = (lambda v: float(np.round(v))) if roundToInteger else (lambda v: v)
    if all(s == 0 for s in sd):
        return [rnd(m) for m in mean]
    out = [rnd(D.rnorm1(mean[i], sd[i])) for i in range(n)]
    for i in range(n):
        while out[i] < lo or out[i] > hi:
            out[i] = rnd(D.rnorm1(mean[i], sd[i]))
    return out


def wiggle_anchors(D, df, temperature, temp_coef, low, high, wiggleAllRows=False):
    """wiggleAnchors(), R/utilities_soundgen.R:634-735: df is a dict of equally long
    columns (a data.frame); returns the wiggled copy."""
    cols = list(df)
    X = np.array([np.atleast_1d(np.asarray(df[c], float)) for c in cols]).T  # rows x cols
    if np.isnan(X).any():
        return None
    nrow, ncol = X.shape
    action = D.sample_prob1([1 - temperature, temperature / 2, temperature / 2])  # nothing, remove, add
    if action == 3:
        if nrow == 1:
            idx = list(range(1, ncol))
            means, sds = X[0, idx], X[0, idx] * temperature * temp_coef
            new = _rnorm_bounded_cols(D, means, sds, [low[i] for i in idx], [high[i] for i in idx])
            X = np.vstack([X, np.concatenate([[1.0], new])])
            X[0, 0] = 0.0
        else:
            a1 = D.unif_index(nrow) + 1
            direction = -1 if D.unif_index(2) == 0 else 1
            a2 = a1 - direction if (a1 + direction < 1 or a1 + direction > nrow) else a1 + direction
            i1, i2 = min(a1, a2), max(a1, a2)
            new = X[i1 - 1:i2].mean(axis=0)
            X = np.vstack([X[:i1], new[None, :], X[i2 - 1:]])
    elif action == 2:
        if wiggleAllRows:
            k = D.unif_index(nrow) + 1
            X = np.delete(X, k - 1, axis=0)
        elif nrow > 2:
            k = 2 + D.unif_index(nrow - 2)  # sampleModif(2:(nrow - 1), 1)
            X = np.delete(X, k - 1, axis=0)
    nrow = X.shape[0]
    orig = None if wiggleAllRows else (X[0, 0], X[-1, 0])
    if nrow == 1:
        ranges = X[0].copy()
    else:
        ranges = np.abs(X.max(axis=0) - X.min(axis=0))
        z = ranges == 0
        ranges[z] = np.abs(X[0, z])
    for i in range(ncol):
        X[:, i] = rnorm_bounded(D, nrow, X[:, i], ranges[i] * temperature * temp_coef, low[i], high[i], False)
    if orig is not None:
        X[0, 0], X[-1, 0] = orig
    return {c: list(X[:, i]) for i, c in enumerate(cols)}


def _rnorm_bounded_cols(D, means, sds, lows, highs):
    """rnorm_bounded with per-element bounds (wiggleAnchors' new anchor)."""
    means = [min(max(m, lo), hi) for m, lo, hi in zip(means, lows, highs)]
    if all(s == 0 for s in sds):
        return list(means)
    out = [D.rnorm1(m, s) for m, s in zip(means, sds)]
    for i in range(len(out)):
        while out[i] < lows[i] or out[i] > highs[i]:
            out[i] = D.rnorm1(means[i], sds[i])
    return out


def wiggle_pars(D, parList, parsToWiggle, probMutation, stepVariance):
    """wigglePars(), R/matchPars.R:436-508."""
    parList = copy.deepcopy(parList)
    pv = _PV
    if len(parsToWiggle) > 1:
        idx = [D.rbinom1(probMutation) for _ in parsToWiggle]
        mutate = [p for p, m in zip(parsToWiggle, idx) if m == 1]
        if not mutate:
            mutate = [parsToWiggle[D.unif_index(len(parsToWiggle))]]
    else:
        mutate = list(parsToWiggle)
    for p in mutate:
        v = parList.get(p)
        if isinstance(v, (int, float)) and not isinstance(v, bool):
            lo, hi = pv[p][1], pv[p][2]
            r = abs(v) if v != 0 else hi - lo
            parList[p] = rnorm_bounded(D, 1, v, r * stepVariance, lo, hi, p in _PAR_ROUND)[0]
        elif isinstance(v, dict):
            if p in ("formants", "formantsNoise"):
                for f in list(v):
                    v[f] = wiggle_anchors(D, _df(v[f]), stepVariance, 1, (0, 50, -120, 1), (1, 8000, 120, 2000))
            else:
                allrows = False
                if p == "pitchAnchors":
                    low, high = (0, pv["pitchFloor"][0]), (1, pv["pitchCeiling"][0])
                elif p in ("amplAnchors", "amplAnchorsGlobal"):
                    low, high = (0, 0), (1, -pv["throwaway"][0])
                elif p == "noiseAnchors":
                    low, high = (-math.inf, pv["throwaway"][0]), (math.inf, 40)
                    allrows = True
                else:  # pitchAnchorsGlobal: permittedValues['pitchDeltas', ...]
                    low, high = (0, pv["pitchDeltas"][1]), (1, pv["pitchDeltas"][2])
                parList[p] = wiggle_anchors(D, _df(v), stepVariance, 1, low, high, allrows)
    return parList


def _df(f):
    """A formant / anchor list as an R data.frame: columns recycled to the longest,
    formant columns in R's order (time, freq, amp, width)."""
    order = [k for k in ("time", "freq", "amp", "width", "value") if k in f] + [k for k in f if k not in
                                                                               ("time", "freq", "amp", "width", "value")]
    cols = {k: list(np.atleast_1d(np.asarray(f[k], float))) for k in order}
    n = max(len(c) for c in cols.values())
    return {k: [c[i % len(c)] for i in range(n)] for k, c in cols.items()}


# ---------------------------------------------------------------- mel spectrum
def _hz2mel(f):
    f = np.asarray(f, float)
    f_sp, brkfrq = 200 / 3, 1000.0
    brkpt = brkfrq / f_sp
    logstep = math.exp(math.log(6.4) / 27)
    return np.where(f < brkfrq, f / f_sp, brkpt + np.log(np.maximum(f, 1e-300) / brkfrq) / math.log(logstep))


def _mel2hz(z):
    z = np.asarray(z, float)
    f_sp, brkfrq = 200 / 3, 1000.0
    brkpt = brkfrq / f_sp
    logstep = math.exp(math.log(6.4) / 27)
    return np.where(z < brkpt, f_sp * z, brkfrq * np.exp(math.log(logstep) * (z - brkpt)))


def fft2melmx(nfft, sr, nfilts, width=1.0, minfreq=0.0, maxfreq=None):
    """tuneR fft2melmx (Slaney mel, constamp = FALSE): nfilts x nfft weights."""
    maxfreq = sr / 2 if maxfreq is None else maxfreq
    fftfreqs = np.arange(nfft) / nfft * sr
    minmel, maxmel = _hz2mel(minfreq), _hz2mel(maxfreq)
    binfreqs = _mel2hz(minmel + np.arange(nfilts + 2) / (nfilts + 1) * (maxmel - minmel))
    wts = np.zeros((nfilts, nfft))
    for i in range(nfilts):
        fs = binfreqs[i:i + 3]
        fs = fs[1] + width * (fs - fs[1])
        lo = (fftfreqs - fs[0]) / (fs[1] - fs[0])
        hi = (fs[2] - fftfreqs) / (fs[2] - fs[1])
        wts[i] = np.maximum(0, np.minimum(lo, hi))
    wts = (2 / (binfreqs[2:nfilts + 2] - binfreqs[:nfilts]))[:, None] * wts
    return wts


def _r_round(x):
    return float(np.round(x))  # half to even, as R's round(x, 0)


def powspec(x, sr, wintime, steptime):
    """tuneR powspec() via signal::specgram(): |FFT|^2, nfft / 2 rows x frames."""
    winpts = int(_r_round(wintime * sr))
    steppts = int(_r_round(steptime * sr))
    nfft = int(2 ** math.ceil(math.log(winpts) / math.log(2)))
    window = 0.54 - 0.46 * np.cos(2 * np.pi * np.arange(winpts) / (winpts - 1)) if winpts > 1 else np.ones(1)
    x = np.asarray(x, float)
    if len(x) > winpts:
        nn = int((len(x) - winpts - 1) / steppts + 1e-10)  # seq(1, length(x) - win_size, by = step)
        offs = np.arange(nn + 1) * steppts
    else:
        offs = np.zeros(1, dtype=np.int64)
    S = np.zeros((nfft, len(offs)))
    for i, o in enumerate(offs):
        seg = x[o:o + winpts]
        S[:len(seg), i] = seg * window[:len(seg)]
    F = np.fft.fft(S, axis=0)
    return np.abs(F[:nfft // 2]) ** 2


def get_mel_spec(s, samplingRate, windowLength=40, overlap=50, step=None, throwaway=-120, maxFreq=None):
    """getMelSpec(), R/matchPars.R:510-560 (melfcc(spec_out = TRUE)$aspectrum)."""
    if step is None:
        step = windowLength * (1 - overlap / 100)
    sr = samplingRate
    maxFreq = sr / 2 if maxFreq is None else maxFreq
    x = np.asarray(s, float)
    pre = x.copy()
    pre[1:] = x[1:] - 0.97 * x[:-1]  # filter(x, c(1, -0.97), sides = 1); y[1] = x[1]
    P = powspec(pre, sr, windowLength / 1000, step / 1000)
    nfreqs = P.shape[0]
    nbands = int(100 * windowLength / 20)
    wts = fft2melmx((nfreqs - 1) * 2, sr, nbands, 1.0, 0.0, maxFreq)[:, :nfreqs]
    spec = wts @ P
    spec = spec[:, spec.mean(axis=0) > 2 ** (throwaway / 10)]
    if spec.size == 0:
        return spec
    v = spec - spec.min() + 1  # log01
    v = np.log(v)
    v = v - v.min()
    return v / v.max()


def _match_columns(m, ncol):
    """matchColumns(matrix_short, nCol, padWith = NA), central (matchLengths)."""
    short = np.arange(1, m.shape[1] + 1, dtype=float)
    padded = np.concatenate([np.full(ncol, np.nan), short, np.full(ncol, np.nan)])
    start = math.ceil((1 + len(padded)) / 2 - ncol / 2)
    pos = padded[start - 1:start - 1 + ncol]
    out = np.full((m.shape[0], ncol), np.nan)
    out[:, ~np.isnan(pos)] = m
    return out


def dtw_normalized(x, y):
    """dtw::dtw(x, y, distance.only = TRUE)$normalizedDistance with the package
    defaults (Euclidean local distance, symmetric2 step pattern: distance / (n + m))."""
    x = np.ascontiguousarray(x, float)
    y = np.ascontiguousarray(y, float)
    out = C.c_double()
    dp = C.POINTER(C.c_double)
    native.check(native.lib().sg_dtw_symmetric2(x.ctypes.data_as(dp), len(x), y.ctypes.data_as(dp), len(y),
                                                C.byref(out)))
    return out.value


def compare_sounds(target=None, targetSpec=None, cand=None, samplingRate=None,
                   method=("cor", "cosine", "pixel", "dtw"), windowLength=40, overlap=50, step=None,
                   penalizeLengthDif=True, throwaway=-120, maxFreq=None, summary=True):
    """compareSounds(), R/matchPars.R:313-416 (padWith = NA)."""
    kw = dict(windowLength=windowLength, overlap=overlap, step=step, throwaway=throwaway, maxFreq=maxFreq)
    if targetSpec is None:
        targetSpec = get_mel_spec(target, samplingRate, **kw)
    candSpec = get_mel_spec(cand, samplingRate, **kw)
    if targetSpec.shape[1] < candSpec.shape[1]:
        targetSpec = _match_columns(targetSpec, candSpec.shape[1])
    elif targetSpec.shape[1] > candSpec.shape[1]:
        candSpec = _match_columns(candSpec, targetSpec.shape[1])
    nc = targetSpec.shape[1]
    sim = {m: np.full(nc, np.nan) for m in method}
    for c in range(nc):
        t, d = targetSpec[:, c], candSpec[:, c]
        ok = ~(np.isnan(t) | np.isnan(d))
        if "cor" in method and ok.sum() > 1:
            a, b = t[ok] - t[ok].mean(), d[ok] - d[ok].mean()
            den = math.sqrt(float(a @ a) * float(b @ b))
            sim["cor"][c] = float(a @ b) / den if den > 0 else np.nan
        if "cosine" in method:
            sim["cosine"][c] = float(t @ d) / math.sqrt(float(t @ t) * float(d @ d)) if ok.all() else np.nan
        if "pixel" in method:
            sim["pixel"][c] = 1 - float(np.mean(np.abs(t - d)))
        if "dtw" in method and ok.all():
            sim["dtw"][c] = 1 - dtw_normalized(t, d)
    if penalizeLengthDif:
        out = {m: float(np.nansum(v)) / len(v) for m, v in sim.items()}
    else:
        out = {m: float(np.nanmean(v)) if np.isfinite(v).any() else np.nan for m, v in sim.items()}
    if summary:
        vals = [out[m] for m in method if not math.isnan(out[m])]
        return float(np.mean(vals)) if vals else math.nan
    return out


# ------------------------------------------------------- on the GPU (sg_mel.hip)
_METHOD_BITS = {"cor": 1, "cosine": 2, "pixel": 4, "dtw": 8}
_METHOD_ORDER = ("cor", "cosine", "pixel", "dtw")


def _mel_params(samplingRate, windowLength=40, overlap=50, step=None, throwaway=-120, maxFreq=None,
                penalizeLengthDif=True):
    from . import _abi
    return _abi.sg_mel_params(float(samplingRate), float(windowLength), float(overlap),
                              math.nan if step is None else float(step), float(throwaway),
                              math.nan if maxFreq is None else float(maxFreq), int(bool(penalizeLengthDif)), 0)


def get_mel_spec_gpu(s, samplingRate, windowLength=40, overlap=50, step=None, throwaway=-120, maxFreq=None, device=0):
    """getMelSpec() (R/matchPars.R:510-560) computed on the GPU (sg_mel_spec, fp64):
    the same nb x nc matrix as get_mel_spec."""
    L = native.lib()
    ctx = native.default_context(device)
    x = np.ascontiguousarray(np.asarray(s, dtype=np.float64))
    P = _mel_params(samplingRate, windowLength, overlap, step, throwaway, maxFreq)
    nb, nc = C.c_int32(), C.c_int32()
    dp = C.POINTER(C.c_double)
    native.check(L.sg_mel_spec(ctx.ptr, x.ctypes.data_as(dp), len(x), C.byref(P), None, 0, C.byref(nb), C.byref(nc)),
                 ctx.ptr)
    out = np.zeros(nb.value * nc.value)
    native.check(L.sg_mel_spec(ctx.ptr, x.ctypes.data_as(dp), len(x), C.byref(P), out.ctypes.data_as(dp), len(out),
                               C.byref(nb), C.byref(nc)), ctx.ptr)
    return out.reshape(nc.value, nb.value).T


def compare_sounds_batch(targetSpec, data, offsets, lengths, samplingRate, method=_METHOD_ORDER, windowLength=40,
                         overlap=50, step=None, penalizeLengthDif=True, throwaway=-120, maxFreq=None, device=0):
    """compareSounds(targetSpec = targetSpec, cand = c, ..., summary = FALSE) for a
    batch of candidates already in HBM (`data`: a float32 CUDA tensor, candidate i
    at offsets[i], lengths[i] samples, < 0 for a failed call -- the layout of
    batch.synthesize_packed), in one launch sequence (sg_compare_sounds_batch):
    returns (per method a float array over the candidates, the summary array:
    the mean of the non-NA methods, compareSounds(summary = TRUE))."""
    L = native.lib()
    ctx = native.default_context(device)
    mask = 0
    for m in method:
        mask |= _METHOD_BITS[m]
    T = np.asfortranarray(np.asarray(targetSpec, dtype=np.float64))
    nb, ncT = T.shape if T.ndim == 2 else (0, 0)
    tflat = np.ascontiguousarray(T.T.ravel())  # column-major
    offs = np.ascontiguousarray(np.asarray(offsets, dtype=np.int64))
    lens = np.ascontiguousarray(np.asarray(lengths, dtype=np.int64))
    n = len(offs)
    out = np.full(4 * n, np.nan)
    summ = np.full(n, np.nan)
    P = _mel_params(samplingRate, windowLength, overlap, step, throwaway, maxFreq, penalizeLengthDif)
    dp = C.POINTER(C.c_double)
    i64p = C.POINTER(C.c_int64)
    native.check(L.sg_compare_sounds_batch(ctx.ptr, tflat.ctypes.data_as(dp), int(nb), int(ncT), C.c_void_p(
        data.data_ptr()), offs.ctypes.data_as(i64p), lens.ctypes.data_as(i64p), n, C.byref(P), mask,
        out.ctypes.data_as(dp), summ.ctypes.data_as(dp)), ctx.ptr)
    out = out.reshape(n, 4)
    return {m: out[:, k] for k, m in enumerate(_METHOD_ORDER) if m in method}, summ


# ---------------------------------------------------------------- matchPars
def match_pars(target, samplingRate, pars, init=None, method=("cor", "cosine", "pixel", "dtw"), probMutation=.25,
               stepVariance=0.1, maxIter=50, minExpectedDelta=0.001, windowLength=40, overlap=50, step=None,
               penalizeLengthDif=True, throwaway=-120, maxFreq=None, rng=None, pop=1, device=0, verbose=False):
    """matchPars(), R/matchPars.R:81-311, with each generation's `pop` mutants
    synthesized as one GPU batch. `rng` (rrng.RRng) supplies every draw (the
    mutations and soundgen()'s own) in R's order for pop = 1. Returns
    {"history": [{"pars", "sim"}...], "pars": best, "evaluated": candidates}."""
    from . import batch
    from .rrng import RRng
    rng = rng if rng is not None else RRng(1)
    D = _Draws(rng)
    kw = dict(windowLength=windowLength, overlap=overlap, step=step, penalizeLengthDif=penalizeLengthDif,
              throwaway=throwaway, maxFreq=maxFreq)
    targetSpec = get_mel_spec_gpu(target, samplingRate, windowLength, overlap, step, throwaway, maxFreq, device)
    defaults = MATCHPARS_DEFAULTS
    parDefault = {p: copy.deepcopy(defaults[p]) for p in pars}
    for k, v in (init or {}).items():
        if k not in defaults:
            raise ValueError("init parameter not recognized: %s" % k)
        parDefault[k] = copy.deepcopy(v)
    parDefault["samplingRate"] = samplingRate

    def call(p):
        return {"kind": "soundgen", "args": _soundgen_args(p), "rng": rng}

    def score(calls):
        """One generation on the GPU: the candidates synthesized as one batch into
        HBM, their spectra and similarities in one launch sequence; -inf for a
        call the planner refused."""
        data, offs, lens = batch.synthesize_packed(calls, device)
        _, summ = compare_sounds_batch(targetSpec, data, offs, lens, samplingRate, method, device=device, **kw)
        return [(-math.inf if n < 0 or math.isnan(v) else float(v)) for v, n in zip(summ, lens)], lens

    sims, lens = score([call(parDefault)])
    if lens[0] < 0:
        raise ValueError("Invalid initial pars")
    sim0 = sims[0]
    history = [{"pars": parDefault, "sim": sim0}]
    parLoop, i, evaluated = parDefault, 1, 1
    while i < maxIter:
        muts = [wiggle_pars(D, parLoop, list(pars), probMutation, stepVariance) for _ in range(pop)]
        sims, _ = score([call(m) for m in muts])
        best, best_m = -math.inf, None
        for m, s in zip(muts, sims):
            evaluated += 1
            if s > best:
                best, best_m = s, m
        if best - history[-1]["sim"] > minExpectedDelta:
            history.append({"pars": best_m, "sim": best})
            parLoop = best_m
            i = 1
            if verbose:
                print("Best similarity: ", round(best, 4))
        else:
            i += pop - 1
        i += 1
    return {"history": history, "pars": history[-1]["pars"], "evaluated": evaluated}


def _soundgen_args(p):
    out = {}
    for k, v in p.items():
        if isinstance(v, dict) and k not in ("formants", "formantsNoise", "tempEffects"):
            v = {c: list(np.atleast_1d(x)) for c, x in v.items()}
        out[k] = v
    return out
