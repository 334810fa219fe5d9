"""morph(): a batch driver over soundgen() (R/morph.R:30-209 with its helpers
morphDF / morphFormants / morphList, R/utilities_morph.R:37-285).

The formula arithmetic (which parameters differ from soundgen()'s defaults,
log-frequency interpolation, per-anchor matching of contours) is host work on a
few dozen numbers and is restated here in Python with R's semantics, quirks
included (noted inline). The nMorphs soundgen() calls it produces are then
planned as ONE batch and synthesized on the GPU in one pass (R calls soundgen()
nMorphs times in a loop, R/morph.R:200-207); savePath writes each morph with
the GPU 16-bit converter (seewave::savewav, R/morph.R:203-206).

Parity: restated from the R sources; no R in this container, so the formula
values are checked against hand-derived cases (tests/test_morph.py), "parity
unpinned" against R itself.
"""
import copy
import math

import numpy as np

from . import rargs, rcall


class DataFrame(dict):
    """An R data.frame (columns by name). identical(list, data.frame) is FALSE in R."""


# soundgen()'s formals (R/soundgen.R:208-277) as morph() evaluates them: anchors
# given as data.frame(...) in the formals are data frames, the rest as written
def _defaults():
    d = copy.deepcopy(rargs.SOUNDGEN_DEFAULTS)
    for k in ("pitchAnchors", "noiseAnchors", "mouthAnchors"):
        d[k] = DataFrame(d[k])
    d["tempEffects"] = dict(rargs.TEMP_EFFECTS_DEFAULT)
    # plot / play / savePath / invalidArgAction are excluded by morph() itself (R/morph.R:66)
    d.pop("invalidArgAction", None)
    return d


def _norm(v):
    """R values as comparable Python: length-1 numeric vectors are scalars."""
    if isinstance(v, DataFrame):
        return ("df", tuple((k, _norm(x)) for k, x in v.items()))
    if isinstance(v, dict):
        return ("list", tuple((k, _norm(x)) for k, x in v.items()))
    if isinstance(v, (list, tuple, np.ndarray)):
        vals = [float(x) if isinstance(x, (int, float, np.floating)) and not isinstance(x, bool) else x for x in v]
        return vals[0] if len(vals) == 1 else ("vec", tuple(vals))
    if isinstance(v, (int, np.integer)) and not isinstance(v, bool):
        return float(v)
    return v


def _identical(a, b):
    return _norm(a) == _norm(b)


def _dollar(lst, name):
    """R's `$` on a list: exact name, else the unique partial match (a quirk that
    matters here: f1$formants finds formantsNoise when formants is absent)."""
    if name in lst:
        return lst[name]
    hits = [k for k in lst if k.startswith(name)]
    return lst[hits[0]] if len(hits) == 1 else None


def _is_list(v):
    return isinstance(v, dict)


def _vec(v):
    return [float(x) for x in (v if isinstance(v, (list, tuple, np.ndarray)) else [v])]


def _as_df(x):
    """as.data.frame() of a list of columns: recycle to the longest."""
    cols = {k: _vec(v) for k, v in x.items()}
    n = max(len(c) for c in cols.values())
    return DataFrame({k: [c[i % len(c)] for i in range(n)] for k, c in cols.items()})


def _has_na(df):
    return any(math.isnan(v) for c in df.values() for v in c)


def _div(a, b):
    """IEEE division as R does it (x / 0 is +-Inf or NaN)."""
    if b == 0:
        return math.nan if a == 0 or math.isnan(a) else math.copysign(math.inf, a)
    return a / b


def _r_seq_len(a, b, n):
    if n == 1:
        return [float(a)]
    by = (b - a) / (n - 1)
    v = [a + i * by for i in range(n)]
    v[-1] = b
    return v


def morphDF(a, b, nMorphs=5):
    """morphDF(a, b, nMorphs), method 'perAnchor' (the default), R/utilities_morph.R:37-197."""
    if _identical(a, b):
        return [copy.deepcopy(a) for _ in range(nMorphs)]
    a = a if a is None or isinstance(a, float) else _as_df(a)
    b = b if b is None or isinstance(b, float) else _as_df(b)

    def bad(d):
        return d is None or isinstance(d, float) or len(d) < 2 or _has_na(d)
    if bad(a) and not bad(b) and len(b) == 2:
        a = DataFrame((k, [0.0] * len(v) if i == 1 else list(v)) for i, (k, v) in enumerate(b.items()))
    elif bad(b) and not bad(a) and len(a) == 2:
        b = DataFrame((k, [0.0] * len(v) if i == 1 else list(v)) for i, (k, v) in enumerate(a.items()))
    elif bad(a) and bad(b):
        return [None] * nMorphs
    ka, kb = list(a), list(b)
    ax, ay, bx, by = a[ka[0]], a[ka[1]], b[kb[0]], b[kb[1]]
    mx_x, mn_x = max(max(ax), max(bx)), min(min(ax), min(bx))
    mx_y, mn_y = max(max(ay), max(by)), min(min(ay), min(by))
    swap = False
    if len(ax) < len(bx):  # the longer data frame first
        a, b, ka, kb, ax, ay, bx, by = b, a, kb, ka, bx, by, ax, ay
        swap = True
    na, nb = len(ax), len(bx)
    an = [(_div(ax[i] - mn_x, mx_x - mn_x), _div(ay[i] - mn_y, mx_y - mn_y)) for i in range(na)]
    bn = [(_div(bx[i] - mn_x, mx_x - mn_x), _div(by[i] - mn_y, mx_y - mn_y)) for i in range(nb)]

    def dist(p, q):
        return math.sqrt((p[0] - q[0]) ** 2 + (p[1] - q[1]) ** 2)

    def which_min(v):  # first minimum, NaN ignored
        best, bi = math.inf, None
        for i, x in enumerate(v):
            if not math.isnan(x) and (x < best or bi is None):
                best, bi = x, i
        if bi is None:  # which.min(all NaN) is integer(0): R stops at the assignment
            raise ValueError("morphDF: anchors cannot be matched (a constant coordinate: R errors here)")
        return bi
    match = [None] * na
    if na > 2:
        for i in range(1, na - 1):  # middle anchors of a: the closest anchor of b
            d = [dist(bn[x], an[i]) for x in range(nb)]
            if nb > 2:
                match[i] = which_min(d[1:-1]) + 2  # middle anchors to middle anchors (1-based)
            else:
                match[i] = which_min(d) + 1
    match[0], match[na - 1] = 1, nb
    used = set(match)
    not_matched = [i + 1 for i in range(nb) if (i + 1) not in used]
    for i in not_matched:
        j = which_min([dist(an[x], bn[i - 1]) for x in range(na)])
        match[j] = not_matched[0]  # R assigns the whole vector; the first element is kept
    for i in range(na):  # non-decreasing
        m = max(match[:i + 1])
        if match[i] < m:
            match[i] = m
    idx = _r_seq_len(0.0, 1.0, nMorphs)
    out = [None] * nMorphs
    for d in range(nMorphs):
        rows, seen = [], set()
        for i in range(na):
            t = ax[i] + idx[d] * (bx[match[i] - 1] - ax[i])
            v = ay[i] + idx[d] * (by[match[i] - 1] - ay[i])
            if (t, v) not in seen:  # hybrid[!duplicated(hybrid[, 1:2]), ]
                seen.add((t, v))
                rows.append((t, v))
        df = DataFrame({ka[0]: [r[0] for r in rows], ka[1]: [r[1] for r in rows]})
        out[nMorphs - d - 1 if swap else d] = df
    return out


_FORMANT_COLS = ("time", "freq", "amp", "width")


def _formant_df(f):
    """A formant as R's data.frame with its columns in R's order (time, freq, amp,
    width; presets.json stores them sorted): morphFormants indexes columns by position."""
    d = _as_df(f)
    return DataFrame([(k, d[k]) for k in _FORMANT_COLS if k in d] + [(k, v) for k, v in d.items()
                                                                     if k not in _FORMANT_COLS])


def morphFormants(f1, f2, nMorphs=5):
    """R/utilities_morph.R:204-225: morph freq, amp and width against time."""
    f1, f2 = _formant_df(f1), _formant_df(f2)
    for f in (f1, f2):
        if len(next(iter(f.values()))) == 1:  # rbind(f, f); time[2] = 1
            for k in f:
                f[k] = f[k] * 2
            f["time"][1] = 1.0
    k1, k2 = list(f1), list(f2)
    sub = lambda f, ks, j: DataFrame({ks[0]: f[ks[0]], ks[j]: f[ks[j]]})  # noqa: E731
    h = morphDF(sub(f1, k1, 1), sub(f2, k2, 1), nMorphs)
    h_amp = morphDF(sub(f1, k1, 2), sub(f2, k2, 2), nMorphs)
    h_width = morphDF(sub(f1, k1, 3), sub(f2, k2, 3), nMorphs)
    for i in range(len(h)):
        h[i]["amp"] = h_amp[i]["amp"]
        h[i]["width"] = h_width[i]["width"]
    return h


def morphList(l1, l2, nMorphs=5):
    """R/utilities_morph.R:254-285: equal formant counts (a silent copy of the other
    list's next formant), then morph formant by formant, by position. Naming
    follows R's two loops: padding l2 takes l1's LAST name (names can repeat,
    :256-260); padding l1 takes l2's name at the new position (names(l1) is
    indexed after l1 grew, :261-265)."""
    a = [(k, copy.deepcopy(v)) for k, v in l1.items()]
    b = [(k, copy.deepcopy(v)) for k, v in l2.items()]
    while len(a) > len(b):
        f = copy.deepcopy(a[len(b)][1])
        f["amp"] = 0.0
        b.append((a[-1][0], f))
    while len(b) > len(a):
        f = copy.deepcopy(b[len(a)][1])
        f["amp"] = 0.0
        a.append((b[len(a)][0], f))
    out = [[(k, copy.deepcopy(v)) for k, v in a] for _ in range(nMorphs)]
    for fi in range(len(a)):
        temp = morphFormants(a[fi][1], b[fi][1], nMorphs)
        for i in range(nMorphs):
            out[i][fi] = (a[fi][0], temp[i])
    return [_unique_names(o) for o in out]


def _unique_names(pairs):
    """A named R list as a dict; a repeated name gets a suffix (the formant list is
    used by position, only the name "f1" carries meaning, R/sourceSpectrum.R:469)."""
    d = {}
    for k, v in pairs:
        key, j = k, 1
        while key in d:
            key, j = "%s.dup%d" % (k, j), j + 1
        d[key] = v
    return d


def _as_formula(x, which):
    if isinstance(x, str):  # paste0('list', substr(formula, 9, nchar(formula)))
        return rcall.parse_call(x)
    if not isinstance(x, dict):
        raise TypeError('%s must be either a list of pars like "list(sylLen = 500)" or a character string like '
                        '"soundgen(sylLen = 500"' % which)
    return copy.deepcopy(x)


def morph_formulas(formula1, formula2, nMorphs):
    """The nMorphs soundgen() argument lists of morph() (R/morph.R:37-197)."""
    formula1, formula2 = _as_formula(formula1, "Formula1"), _as_formula(formula2, "Formula2")
    defaults = _defaults()
    nd1 = [k for k, v in formula1.items() if not _identical(v, defaults.get(k))]
    nd2 = [k for k, v in formula2.items() if not _identical(v, defaults.get(k))]
    names = list(dict.fromkeys(nd1 + nd2))
    f1 = {k: copy.deepcopy(defaults.get(k)) for k in names}
    f2 = {k: copy.deepcopy(defaults.get(k)) for k in names}
    for k in formula1:
        if k in f1:
            f1[k] = copy.deepcopy(formula1[k])
    for k in formula2:
        if k in f2:
            f2[k] = copy.deepcopy(formula2[k])
    # a formant list missing on one side becomes the other side's, silenced (R/morph.R:95-114)
    for fa, fb in ((f1, f2), (f2, f1)):
        for key in ("formants", "formantsNoise"):
            if not _is_list(_dollar(fa, key)) and _is_list(_dollar(fb, key)):
                fa[key] = copy.deepcopy(_dollar(fb, key))
                for f in fa[key].values():
                    f["amp"] = 0.0
    # log pitch and formant frequencies (R/morph.R:117-148)
    def log_freqs(f):
        if "pitchAnchors" in f and isinstance(f["pitchAnchors"], dict) and _numeric(f["pitchAnchors"].get("value")):
            f["pitchAnchors"]["value"] = _map(math.log, f["pitchAnchors"]["value"])
        for key in ("formants", "formantsNoise"):
            if key in f and isinstance(f[key], dict):
                for fm in f[key].values():
                    if _numeric(fm.get("freq")):
                        fm["freq"] = _map(math.log, fm["freq"])
    log_freqs(f1)
    log_freqs(f2)
    formulas = [copy.deepcopy(f1) for _ in range(nMorphs)]
    for p, name in enumerate(f1):
        a, b = f1[name], list(f2.values())[p]
        if _numeric(a) and not isinstance(a, dict):
            m = _r_seq_len(float(_vec(a)[0]), float(_vec(b)[0]), nMorphs)
        elif name in ("formants", "formantsNoise"):
            m = morphList(a, b, nMorphs)
        else:
            m = morphDF(a, b, nMorphs)
        for h in range(nMorphs):
            formulas[h][name] = m[h]
    for h in range(nMorphs):  # back to Hz (R/morph.R:170-197)
        f = formulas[h]
        if "pitchAnchors" in f1 and isinstance(f.get("pitchAnchors"), dict) and _numeric(f["pitchAnchors"].get("value")):
            f["pitchAnchors"]["value"] = _map(math.exp, f["pitchAnchors"]["value"])
        for key in ("formants", "formantsNoise"):
            if key in f1 and isinstance(f.get(key), dict):
                for fm in f[key].values():
                    if _numeric(fm.get("freq")):
                        fm["freq"] = _map(math.exp, fm["freq"])
    return formulas


def _numeric(v):
    """class(v) == 'numeric' for a parsed R value (doubles; NA/NULL are not)."""
    if isinstance(v, bool) or v is None:
        return False
    if isinstance(v, (int, float)):
        return True
    return isinstance(v, (list, tuple)) and len(v) > 0 and all(
        isinstance(x, (int, float)) and not isinstance(x, bool) for x in v)


def _map(fn, v):
    return [fn(x) for x in v] if isinstance(v, (list, tuple)) else fn(v)


def _soundgen_args(formula):
    """A morphed formula as soundgen() keyword arguments (data frames -> column dicts)."""
    out = {}
    for k, v in formula.items():
        if isinstance(v, dict) and k not in ("formants", "formantsNoise", "tempEffects"):
            v = {c: list(x) if isinstance(x, (list, tuple)) else x for c, x in v.items()}
        out[k] = v
    return out


def morph(formula1, formula2, nMorphs, playMorphs=False, savePath=None, samplingRate=16000, normals=None,
          uniforms=None, device=0):
    """morph(formula1, formula2, nMorphs, playMorphs, savePath, samplingRate),
    R/morph.R:30-209. Returns {"formulas": [...], "sounds": [...]}; the nMorphs
    soundgen() calls run as one GPU batch.
    Random draws: R's loop (R/morph.R:200-201) runs the morphs on ONE continuous
    RNG stream, morph h using the draws left by morph h-1. Pass normals/uniforms
    as a list of nMorphs arrays (each morph's own draws, e.g. R's stream split at
    the morph boundaries) to reproduce that; a single array is read from its start
    by every morph (all morphs share one perturbation; parity with R's sequence
    unpinned then)."""
    if playMorphs:
        raise NotImplementedError("playMorphs: audio playback is outside the synthesis path")
    formulas = morph_formulas(formula1, formula2, nMorphs)

    def per(v, h):
        return v[h] if isinstance(v, (list, tuple)) else v
    for v in (normals, uniforms):
        if isinstance(v, (list, tuple)) and len(v) != nMorphs:
            raise ValueError("per-morph draws: %d arrays for %d morphs" % (len(v), nMorphs))
    calls = [{"kind": "soundgen", "args": _soundgen_args(f), "normals": per(normals, h), "uniforms": per(uniforms, h)}
             for h, f in enumerate(formulas)]
    from . import batch
    if savePath is not None:  # one plan and one execute: the 16-bit files and the fp32 sounds
        paths = ["%smorph_%d.wav" % (savePath, h + 1) for h in range(nMorphs)]  # paste0(savePath, 'morph_', h, '.wav')
        _, sounds = batch.synthesize_to_wav(calls, paths, samplingRate, device, return_float=True)
    else:
        sounds = batch.synthesize(calls, device)
    for s in sounds:
        if isinstance(s, Exception):
            raise s
    return {"formulas": formulas, "sounds": [np.asarray(s, np.float64) for s in sounds]}
