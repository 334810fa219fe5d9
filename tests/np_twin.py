"""TEST INFRASTRUCTURE — an independent NumPy restatement of the simple
(temperature = 0, nonlinBalance = 0) generateHarmonics() path and of the R /
seewave numerics it relies on, written from the reference R sources, used to
cross-check the C oracle (oracle/sg_oracle.c) inside this container where R
itself is absent (parity vs R is unpinned).

Reference lines followed:
  getGlottalCycles   R/utilities_soundgen.R:477-486
  upsample           R/utilities_soundgen.R:392-416
  findZeroCrossing   R/utilities_soundgen.R:255-295
  crossFade          R/utilities_soundgen.R:328-375
  fadeInOut          R/utilities_soundgen.R:440-459
  getRolloff         R/sourceSpectrum.R:71-186
  generateHarmonics  R/source.R:173-471 (the deterministic branch)
  seewave stft/istft seewave_2.0.5.tar.gz::seewave/R/seewave.r:7782-7819, :3447-3486
"""
import numpy as np


def seq_len(a, b, n):
    """seq(a, b, length.out = n) — R seq.default."""
    if n <= 0:
        return np.zeros(0)
    if n == 1:
        return np.array([float(a)])
    if a == b:
        return np.full(n, float(a))
    by = (b - a) / (n - 1)
    out = a + np.arange(n) * by
    out[-1] = b
    return out


def seqint_len(a, b, n):
    """seq.int(a, b, length.out = n) — R's C seq.int (symmetric interior)."""
    i = np.arange(n, dtype=np.float64)
    if n == 1:
        return np.array([float(a)])
    by = (b - a) / (n - 1)
    out = np.where(i < n // 2, a + i * by, b - (n - 1 - i) * by)
    out[0], out[-1] = a, b
    return out


def r_round(x):
    return np.rint(x)  # half to even, as R's round(x, 0)


def glottal_cycles(pitch, sr):
    gc, i = [], 1
    while i < len(pitch):
        gc.append(i)
        i = i + max(2, int(np.floor(sr / pitch[i - 1])))
    return np.array(gc, dtype=np.int64)


def fmm_coef(x, y):
    """Forsythe-Malcolm-Moler cubic spline (end conditions from cubics through
    the first / last four points), tridiagonal solve."""
    n = len(x)
    x = np.asarray(x, float)
    y = np.asarray(y, float)
    b, c, d = np.zeros(n), np.zeros(n), np.zeros(n)
    if n < 3:
        t = (y[1] - y[0]) / (x[1] - x[0])
        b[:] = t
        return b, c, d
    h = np.diff(x)
    dy = np.diff(y) / h
    diag = np.zeros(n)
    rhs = np.zeros(n)
    diag[0], diag[-1] = -h[0], -h[-1]
    diag[1:-1] = 2 * (h[:-1] + h[1:])
    rhs[1:-1] = dy[1:] - dy[:-1]
    if n > 3:
        rhs[0] = (dy[2] - dy[1]) / (x[3] - x[1]) - (dy[1] - dy[0]) / (x[2] - x[0])
        rhs[0] = rhs[0] * h[0] ** 2 / (x[3] - x[0])
        rhs[-1] = (dy[-1] - dy[-2]) / (x[-1] - x[-3]) - (dy[-2] - dy[-3]) / (x[-2] - x[-4])
        rhs[-1] = -rhs[-1] * h[-1] ** 2 / (x[-1] - x[-4])
    # forward elimination (sub = super = h)
    dd = diag.copy()
    r = rhs.copy()
    for i in range(1, n):
        t = h[i - 1] / dd[i - 1]
        dd[i] -= t * h[i - 1]
        r[i] -= t * r[i - 1]
    sig = np.zeros(n)
    sig[-1] = r[-1] / dd[-1]
    for i in range(n - 2, -1, -1):
        sig[i] = (r[i] - h[i] * sig[i + 1]) / dd[i]
    b[-1] = dy[-1] + h[-1] * (sig[-2] + 2 * sig[-1])
    b[:-1] = dy - h * (sig[1:] + 2 * sig[:-1])
    d[:-1] = (sig[1:] - sig[:-1]) / h
    c = 3 * sig
    d[-1] = d[-2]
    return b, c, d


def spline(x, y, n):
    """spline(x, y, n = n)$y with method 'fmm'."""
    x = np.asarray(x, float)
    y = np.asarray(y, float)
    b, c, d = fmm_coef(x, y)
    u = seqint_len(x[0], x[-1], n)
    i = np.clip(np.searchsorted(x, u, side="right") - 1, 0, len(x) - 1)
    dx = u - x[i]
    return y[i] + dx * (b[i] + dx * (c[i] + dx * d[i]))


def approx(x, y, n):
    """approx(x, y, n = n)$y, linear, rule = 1."""
    x = np.asarray(x, float)
    y = np.asarray(y, float)
    v = seqint_len(x[0], x[-1], n)
    j = np.clip(np.searchsorted(x, v, side="right"), 1, len(x) - 1)
    i = j - 1
    out = y[i] + (y[j] - y[i]) * ((v - x[i]) / (x[j] - x[i]))
    out = np.where(v == x[j], y[j], out)
    out = np.where(v == x[i], y[i], out)
    return out


def upsample(ppg, sr):
    gcl = r_round(sr / np.asarray(ppg, float))
    c = np.cumsum(gcl)
    gc_up = np.concatenate([[1.0], c])
    l = len(ppg)
    if l == 1:
        pu = np.repeat(ppg, gcl.astype(int))
    elif l == 2:
        pu = seq_len(ppg[0], ppg[1], int(c[-1]))
    else:
        t = np.ones(l)
        t[-1] = c[-1]
        for i in range(2, l):
            t[i - 1] = c[i - 2] + r_round(gcl[i - 1] / 2)
        pu = spline(t, ppg, int(c[-1]))
    return pu, gc_up


def get_rolloff(pitch, nH, rolloff=-12, rolloffOct=-2, rolloffKHz=-6, baseline=200, throwaway=-120, sr=16000,
                rolloffParab=0, rolloffParabHarm=2, rolloffParabCeiling=None):
    pitch = np.atleast_1d(np.asarray(pitch, float))
    h = np.arange(1, nH + 1)[:, None]
    r = (rolloff + rolloffKHz * (pitch[None, :] - baseline) / 1000) * np.log2(h)
    if rolloffOct != 0:
        r = r + np.where(h >= 2, rolloffOct * (pitch[None, :] * h - baseline) / 1000, 0.0)
    r = np.where(h * pitch[None, :] >= sr / 2, -np.inf, r)
    if rolloffParab != 0:
        # R/sourceSpectrum.R:103-132: per-column harmonic counts (a ceiling in Hz, or rolloffParabHarm)
        rphs = [r_round(rolloffParabCeiling / p) if rolloffParabCeiling is not None else r_round(rolloffParabHarm)
                for p in pitch]
        for g, rph in enumerate(rphs):
            if rph == 2:
                rph = 3
            with np.errstate(divide="ignore"):
                a = -4 * rolloffParab / (rph - 1) ** 2
            b = -a * (1 + rph)
            c = a * rph
            if rph < 3:
                if rph < 2:
                    r[0, g] = r[0, g] + rolloffParab
            else:
                k = np.arange(1, int(rph) + 1)
                r[:int(rph), g] = r[:int(rph), g] + a * k ** 2 + b * k + c
    r = np.where(r < throwaway, -np.inf, r)
    r = r - r.max(axis=0, keepdims=True)
    r = 2.0 ** (r / 10)
    keep = r.sum(axis=1) > 0
    return r[keep]


def find_zero_crossing(a, location):
    n = len(a)
    if n < 1 or location < 1 or location > n:
        return None
    if n == 1 and location == 1:
        return location
    zl = zr = None
    i = 0
    if location > 1:
        i = location
        while i > 1:
            if a[i - 1] > 0 and a[i - 2] < 0:
                zl = i - 1
                break
            i -= 1
    if location < n:
        i = location
    while i < n - 1:
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


def cross_fade(a1, a2, sr, crossLen=15):
    a1 = np.asarray(a1, float)
    a2 = np.asarray(a2, float)
    z1 = find_zero_crossing(a1, len(a1))
    if z1 is not None:
        a1 = np.concatenate([a1[:z1], [0.0]])
    z2 = find_zero_crossing(a2, 1)
    if z2 is not None:
        a2 = a2[z2:]
    cl = int(min(np.floor(crossLen * sr / 1000), len(a1) - 1, len(a2) - 1))
    if cl < 2:
        return np.concatenate([a1, a2])
    m = seq_len(0, 1, cl)
    idx1 = len(a1) - cl
    cross = m[::-1] * a1[idx1:] + m * a2[:cl]
    return np.concatenate([a1[:idx1], cross, a2[cl:]])


def fade_in_out(a, length_fade):
    a = np.array(a, float)
    if length_fade < 2:
        return a
    lf = int(min(length_fade, len(a)))
    f = seq_len(0, 1, lf)
    a[:lf] *= f
    a[len(a) - lf:] *= f[::-1]
    return a


def generate_harmonics_simple(pitch, sr=16000, attackLen=50, rolloff=-18, rolloffOct=-2, rolloffKHz=-6,
                              pitchFloor=75, pitchCeiling=3500, psr=3500, throwaway=-120, **_):
    """generateHarmonics() with temperature = 0, nonlinBalance = 0, no vibrato,
    no amplAnchors: one epoch, sine bank, crossFade onto 0, /max, fade."""
    pitch = np.asarray(pitch, float)
    gc = glottal_cycles(pitch, psr)
    ppg = np.clip(pitch[gc - 1], pitchFloor, pitchCeiling)
    nH = int(np.ceil((sr / 2 - ppg.min()) / ppg.min()))
    A = get_rolloff(ppg, nH, rolloff, rolloffOct, rolloffKHz, 200, throwaway, sr)
    pu, gc_up = upsample(ppg, sr)
    acc, s = np.zeros(len(pu)), 0.0
    # cumsum in extended precision, as R's cumsum (long double accumulator)
    acc = np.cumsum(pu.astype(np.longdouble)).astype(np.float64)
    integr = acc / sr
    idx = gc_up  # epoch = all gcs: idx_gc_up = gc_up[1:(nGC+1)]
    lo, hi = int(idx.min()), int(idx.max())
    ie = integr[lo - 1:hi]
    n = len(ie)
    w = np.zeros(n)
    for h in range(A.shape[0]):
        am = approx(idx[:-1], A[h], n)
        w = w + np.sin(2 * np.pi * ie * (h + 1)) * am
    wave = cross_fade(np.array([0.0]), w, sr, 15)
    wave = wave / wave.max()
    if attackLen > 0:
        wave = fade_in_out(wave, np.floor(attackLen * sr / 1000))
    return wave


def hamming(n):
    return 0.54 - 0.46 * np.cos(2 * np.pi * np.arange(n) / (n - 1))


def hanning(n):
    return 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(n) / (n - 1))


def stft(wave, wl, step):
    """seewave::stft(wave, wl, step, wn = 'hamming', complex = TRUE): nr x nc."""
    w = hamming(wl)
    cols = []
    for x0 in step:
        i0 = int(x0) - 1
        cols.append(np.fft.fft(wave[i0:i0 + wl] * w)[: wl // 2] / wl)
    return np.array(cols).T


def istft(z, ovlp, wl):
    """seewave::istft(z, ovlp, wl, wn = 'hanning') incl. the Nyquist quirk."""
    nr, nc = z.shape
    h = wl * (100 - ovlp) / 100
    x = np.zeros(int(wl + (nc - 1) * h))
    win = hanning(wl)
    for f in range(nc):
        X = np.concatenate([z[:, f], [np.real(z[nr - 1, f])], np.conj(z[1:, f][::-1])])
        y = np.real(np.fft.ifft(X))  # R: Re(fft(X, inverse = TRUE) / length(X))
        b = f * h
        i0 = int(b)
        seg = np.resize(y, wl) * win  # xprim * win recycles xprim (length 2 nr = wl - 1 for an odd wl)
        end = min(len(x), i0 + wl)
        x[i0:end] += seg[: end - i0]
    return x * h / np.sum(win ** 2)


# ---------------------------------------------------------------- loess
# loess(y ~ x, span) + predict (R 3.4 stats defaults, 1-D; netlib dloess
# algorithm as R's loessf.f carries it): widened bounding box, median k-d tree
# down to floor(n span 0.2) points per cell, vertex fits (floor(n span) nearest,
# tricube, equilibrated columns, SVD pseudo-inverse), cubic Hermite between
# consecutive vertices. Written independently of oracle/sg_oracle.c.
def _loess_vertices(x, span):
    n = len(x)
    fc = int(np.floor(n * (span * 0.2)))
    lo, hi = x.min(), x.max()
    mu = 0.005 * max(hi - lo, 1e-10 * max(abs(lo), abs(hi)) + 1e-30)
    verts = [lo - mu, hi + mu]
    queue = [(0, n - 1, lo - mu, hi + mu)]  # 0-based point ranges, breadth first
    while queue:
        l, u, v0, v1 = queue.pop(0)
        if u - l + 1 <= fc or v1 - v0 <= 0:
            continue
        m = (l + u + 2) // 2 - 1  # R: floor((l + u) / 2) on 1-based positions
        if x[m] == v0 or x[m] == v1:
            continue
        verts.append(x[m])
        queue.append((l, m, v0, x[m]))
        queue.append((m + 1, u, x[m], v1))
    return np.array(sorted(verts))


def _loess_vertex_fit(x, y, span, v):
    n = len(x)
    nf = int(min(n, np.floor(n * span)))
    d2 = (x - v) ** 2
    order = np.argsort(d2, kind="stable")[:nf]
    rho = d2[order[-1]] * max(1.0, span)
    if not rho > 0:  # zero-width neighbourhood: R's weights are 0/0
        return np.nan, np.nan
    r = np.sqrt(d2[order] / rho)
    w = np.sqrt((1 - r ** 3) ** 3)
    dx = x[order] - v
    B = np.stack([w, w * dx, w * dx * dx], axis=1)
    eta = w * y[order]
    if B.shape[0] < 3:
        B = np.vstack([B, np.zeros((3 - B.shape[0], 3))])
        eta = np.concatenate([eta, np.zeros(3 - len(eta))])
    cn = np.linalg.norm(B, axis=0)
    cn[cn == 0] = 1
    B = B / cn
    U, s, Vt = np.linalg.svd(B, full_matrices=False)
    tol = s.max() * 100 * np.finfo(float).eps
    g = np.where(s > tol, (U.T @ eta) / np.where(s > 0, s, 1), 0.0)
    coef = Vt.T @ g / cn
    return coef[0], coef[1]


def loess(x, y, span, z):
    x = np.asarray(x, float)
    y = np.asarray(y, float)
    vx = _loess_vertices(x, span)
    fits = np.array([_loess_vertex_fit(x, y, span, v) for v in vx])
    if np.isnan(fits).any():  # predict(): .C refuses the NaN vertex values
        raise FloatingPointError("NA/NaN/Inf in foreign function call")
    z = np.asarray(z, float)
    i = np.clip(np.searchsorted(vx, z, side="left") - 1, 0, len(vx) - 2)
    v0, v1 = vx[i], vx[i + 1]
    h = (z - v0) / (v1 - v0)
    phi0, phi1 = (1 - h) ** 2 * (1 + 2 * h), h ** 2 * (3 - 2 * h)
    psi0, psi1 = h * (1 - h) ** 2, -h ** 2 * (1 - h)
    out = phi0 * fits[i, 0] + phi1 * fits[i + 1, 0] + (psi0 * fits[i, 1] + psi1 * fits[i + 1, 1]) * (v1 - v0)
    out[(z < x.min()) | (z > x.max())] = np.nan
    return out


def smooth_contour_loess(time, value, len_, sr, floor=None, ceiling=None, pitch=False):
    """getSmoothContour(anchors, len, method = 'loess') for 3-10 anchors."""
    t = np.asarray(time, float)
    v = np.asarray(value, float)
    if floor is not None:
        v = np.maximum(v, floor)
    if ceiling is not None:
        v = np.minimum(v, ceiling)
    if pitch:
        v = 12 * np.log2(v / 16.3516)
        floor = 12 * np.log2(floor / 16.3516) if floor is not None else None
        ceiling = 12 * np.log2(ceiling / 16.3516) if ceiling is not None else None
    t = (t - t.min()) / (t - t.min()).max()
    pos = {}
    for tp, val in zip(t * len_, v):
        tp = 1.0 if tp == 0 else tp
        if int(tp) >= 1:
            pos[int(tp)] = val
    xs = np.array(sorted(pos))
    ys = np.array([pos[k] for k in xs])
    span = (1 / (1 + np.exp(len_ / sr * 1000 / 500)) + 0.5) / 1.1 ** (len(t) - 3)
    z = np.arange(1, len_ + 1, dtype=float)
    while True:  # try(predict(...)); while (try-error) span = span + 0.1
        try:
            out = loess(xs, ys, span, z)
            break
        except FloatingPointError:
            span = span + 0.1
    while True:
        out = loess(xs, ys, span, z)
        if floor is None or not np.any(out < floor - 1e-6):
            break
        span /= 1.1
    if floor is not None:
        out = np.maximum(out, floor)
    if ceiling is not None:
        out = np.minimum(out, ceiling)
    if pitch:
        out = 16.3516 * 2 ** (out / 12)
    return out
