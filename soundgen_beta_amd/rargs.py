"""R-level argument semantics of soundgen()/generateHarmonics(), marshalled
into the plain C structs of include/soundgen_hip.h.

Mirrors the reference's formals and defaults:
  soundgen()          R/soundgen.R:208-277
  generateHarmonics() R/source.R:173-205
  permittedValues     R/presets.R:22-79
and the argument coercions done at the top of soundgen():
  numeric anchors -> data.frame(time = seq(0, 1, ...), value)   R/soundgen.R:305-315
  list formants   -> lapply(formants, as.data.frame)            R/soundgen.R:384-389
  vowel strings   -> convertStringToFormants()                  R/utilities_soundgen.R:135-222
"""
import math

import numpy as np

from . import _abi

NA = None  # R's NA / NULL for anchors and formants

# permittedValues rows used by soundgen(): name -> (default, low, high, step)
PERMITTED_VALUES = {
    "repeatBout": (1, 1, 20, 1), "nSyl": (1, 1, 10, 1), "sylLen": (300, 20, 5000, 10),
    "pauseLen": (200, 20, 1000, 10), "temperature": (.025, 0, 1, .025),
    "maleFemale": (0, -1, 1, .1), "creakyBreathy": (0, -1, 1, .1),
    "nonlinBalance": (0, 0, 100, 1), "nonlinDep": (50, 0, 100, 1), "jitterDep": (3, 0, 24, .1),
    "jitterLen": (1, 1, 100, 1), "vibratoFreq": (5, 3, 10, .5), "vibratoDep": (0, 0, 3, .125),
    "shimmerDep": (0, 0, 100, 1), "attackLen": (50, 0, 200, 10), "rolloff": (-12, -60, 0, 1),
    "rolloffOct": (-12, -30, 10, 1), "rolloffParab": (0, -50, 50, 5),
    "rolloffParabHarm": (3, 1, 20, 1), "rolloffKHz": (-6, -20, 0, 1), "rolloffLip": (6, 0, 20, 1),
    "formantDep": (1, 0, 5, .1), "formantDepStoch": (30, 0, 60, 10), "vocalTract": (15.5, 2, 100, .5),
    "subFreq": (100, 10, 1000, 10), "subDep": (100, 0, 500, 10), "shortestEpoch": (300, 50, 500, 25),
    "amDep": (0, 0, 100, 5), "amFreq": (30, 10, 100, 5), "amShape": (0, -1, 1, .025),
    "samplingRate": (16000, 8000, 44100, 100), "windowLength": (40, 5, 100, 2.5),
    "rolloffNoise": (-14, -20, 20, 1), "overlap": (50, 0, 99, 1), "addSilence": (100, 0, 1000, 50),
    "pitchFloor": (50, 1, 1000, 1), "pitchCeiling": (3500, 10, 100000, 10),
    "pitchSamplingRate": (3500, 10, 100000, 10), "throwaway": (-120, -200, -10, 10),
    "mouthOpening": (.5, 0, 1, .05), "pitch": (100, 25, 3500, 1), "noiseAmpl": (0, -120, 40, 1),
}

TEMP_EFFECTS_ORDER = ["sylLenDep", "formDrift", "formDisp", "pitchDriftDep", "pitchDriftFreq",
                      "pitchAnchorsDep", "noiseAnchorsDep", "amplAnchorsDep"]
TEMP_EFFECTS_DEFAULT = {"sylLenDep": .02, "formDrift": .3, "formDisp": .2, "pitchDriftDep": .5,
                        "pitchDriftFreq": .125, "pitchAnchorsDep": .05, "noiseAnchorsDep": .1,
                        "amplAnchorsDep": .1}

# soundgen() formals, R/soundgen.R:208-277
SOUNDGEN_DEFAULTS = dict(
    repeatBout=1, nSyl=1, sylLen=300, pauseLen=200,
    pitchAnchors={"time": [0, .1, .9, 1], "value": [100, 150, 135, 100]},
    pitchAnchorsGlobal=NA, temperature=0.025, tempEffects=None,
    maleFemale=0, creakyBreathy=0, nonlinBalance=0, nonlinDep=50, jitterLen=1, jitterDep=3,
    vibratoFreq=5, vibratoDep=0, shimmerDep=0, attackLen=50, rolloff=-12, rolloffOct=-12,
    rolloffKHz=-6, rolloffParab=0, rolloffParabHarm=3, rolloffLip=6,
    formants={"f1": {"time": 0, "freq": 860, "amp": 30, "width": 120},
              "f2": {"time": 0, "freq": 1280, "amp": 40, "width": 120},
              "f3": {"time": 0, "freq": 2900, "amp": 25, "width": 200}},
    formantDep=1, formantDepStoch=30, vocalTract=15.5, subFreq=100, subDep=100,
    shortestEpoch=300, amDep=0, amFreq=30, amShape=0,
    noiseAnchors={"time": [0, 300], "value": [-120, -120]}, formantsNoise=NA,
    rolloffNoise=-14, mouthAnchors={"time": [0, 1], "value": [.5, .5]}, amplAnchors=NA,
    amplAnchorsGlobal=NA, samplingRate=16000, windowLength=50, overlap=75, addSilence=100,
    pitchFloor=50, pitchCeiling=3500, pitchSamplingRate=3500, throwaway=-120,
    invalidArgAction="adjust",
)

# generateHarmonics() formals, R/source.R:173-205
HARM_DEFAULTS = dict(
    attackLen=50, nonlinBalance=0, nonlinDep=0, jitterDep=0, jitterLen=1, vibratoFreq=100,
    vibratoDep=0, shimmerDep=0, creakyBreathy=0, rolloff=-18, rolloffOct=-2, rolloffKHz=-6,
    rolloffParab=0, rolloffParabHarm=3, rolloffLip=6, rolloff_perAmpl=12, temperature=0,
    pitchDriftDep=.5, pitchDriftFreq=.125, randomWalk_trendStrength=.5, shortestEpoch=300,
    subFreq=100, subDep=0, amDep=0, amFreq=30, overlap=75, samplingRate=16000,
    pitchFloor=75, pitchCeiling=3500, pitchSamplingRate=3500, throwaway=-120,
)

# Vowel dictionaries of presets$<speaker>$Formants$vowels (R/presets.R:176-212,
# :268-305) as {vowel: [(name, freq, amp, width), ...]} (time is always 0).
VOWELS = {
    "M1": {
        "a": [("f1", 860, 30, 120), ("f2", 1280, 40, 120), ("f3", 2900, 25, 200)],
        "o": [("f1", 630, 35, 100), ("f2", 900, 35, 100), ("f3", 3000, 30, 200), ("f4", 3960, 30, 200)],
        "i": [("f1", 300, 25, 80), ("f2", 2700, 30, 100), ("f3", 3400, 40, 350), ("f4", 4200, 40, 350)],
        "e": [("f1", 530, 30, 50), ("f1.4", 1100, -20, 100), ("f1.6", 1400, 20, 100),
              ("f2", 2400, 40, 300), ("f3", 4000, 30, 300)],
        "u": [("f1", 375, 25, 80), ("f2", 550, 35, 120), ("f3", 2100, 25, 300), ("f4", 4200, 45, 250)],
        "0": [("f1", 640, 30, 100), ("f2", 1670, 30, 100), ("f3", 2700, 30, 100), ("f4", 3880, 30, 100)],
    },
    "F1": {
        "a": [("f1", 900, 30, 80), ("f2", 1300, 30, 160), ("f3", 3300, 25, 130), ("f4", 4340, 20, 370)],
        "o": [("f1", 800, 30, 80), ("f2", 1100, 30, 80), ("f3", 3560, 40, 200), ("f4", 5830, 50, 200)],
        "i": [("f1", 330, 30, 120), ("f2", 2700, 40, 120), ("f3", 3580, 30, 200), ("f4", 4710, 30, 200),
              ("f5", 5800, 30, 200)],
        "e": [("f1", 930, 30, 100), ("f2", 2470, 30, 100), ("f3", 3300, 25, 120), ("f4", 4200, 30, 200)],
        "u": [("f1", 450, 30, 80), ("f2", 850, 40, 120), ("f3", 2900, 30, 200), ("f4", 4100, 30, 275)],
        "0": [("f1", 790, 30, 100), ("f2", 1600, 30, 100), ("f3", 3100, 30, 100), ("f4", 3900, 30, 100)],
    },
}


def convertStringToFormants(phonemeString, speaker="M1"):
    """R/utilities_soundgen.R:135-222. Returns an ordered dict name -> columns."""
    if speaker not in VOWELS:
        speaker = "M1"
    dic = VOWELS[speaker]
    valid = [p for p in phonemeString if p in dic]
    if not valid:
        return NA
    uniq = list(dict.fromkeys(valid))
    vowels = {v: {n: (fr, a, w) for (n, fr, a, w) in dic[v]} for v in uniq}
    names = sorted({n for v in uniq for n in vowels[v]})
    for v in uniq:  # fill absent formants with amp 0, width 100, freq of the first vowel having it
        for f in names:
            if f not in vowels[v]:
                fr = next(vowels[u][f][0] for u in uniq if f in vowels[u])
                vowels[v][f] = (fr, 0, 100)
    stamps = _seq_len(0.0, 1.0, len(valid))
    out = {}
    for f in names:
        rows = [vowels[v][f] for v in valid]
        out[f] = {"time": list(stamps), "freq": [r[0] for r in rows],
                  "amp": [r[1] for r in rows], "width": [r[2] for r in rows]}
    # R removes a formant when sum(f$amp == 0) == length(f); length() of a
    # data.frame is its column count (4), so only formants with exactly four
    # zero-amplitude rows are dropped (reference quirk, kept).
    out = {f: out[f] for f in names if sum(a == 0 for a in out[f]["amp"]) != 4}
    return out


def _seq_len(a, b, n):
    """R seq(a, b, length.out = n)."""
    if n == 1:
        return np.array([a], dtype=np.float64)
    by = (b - a) / (n - 1)
    v = a + np.arange(n, dtype=np.float64) * by
    v[-1] = b
    return v


def _is_na(x):
    if x is None:
        return True
    if isinstance(x, float) and math.isnan(x):
        return True
    if isinstance(x, str) and x == "NA":
        return True
    return False


def as_anchors(x, time_to=1.0):
    """Anchors -> (time, value) float64 arrays, or None for NA.
    Numeric vectors become data.frame(time = seq(0, time_to, len), value)."""
    if _is_na(x):
        return None
    if isinstance(x, dict):
        t = np.atleast_1d(np.asarray(x["time"], dtype=np.float64))
        v = np.atleast_1d(np.asarray(x["value"], dtype=np.float64))
        n = max(len(t), len(v))
        if len(t) < n:
            t = np.resize(t, n)
        if len(v) < n:
            v = np.resize(v, n)
        return np.ascontiguousarray(t), np.ascontiguousarray(v)
    v = np.atleast_1d(np.asarray(x, dtype=np.float64))
    if len(v) == 0:
        return None
    return _seq_len(0.0, float(time_to), len(v)), np.ascontiguousarray(v)


def r_max_lengths(x):
    """max(unlist(lapply(x, length))) as R evaluates it on formantsNoise
    (R/soundgen.R:662): 1 per string, the field count of each formant list; 0 for NA."""
    if _is_na(x):
        return 0
    if isinstance(x, str):
        return 1
    if isinstance(x, dict):
        return max((len(v) if isinstance(v, dict) else np.atleast_1d(v).size) for v in x.values())
    return max((np.atleast_1d(v).size for v in x), default=0)


def as_formants(x, speaker="M1"):
    """formants -> ordered list of (name, time, freq, amp, width) or None."""
    if _is_na(x):
        return None
    if isinstance(x, str):
        x = convertStringToFormants(x, speaker)
        if x is None:
            return None
    out = []
    for name, f in x.items():
        cols = [np.atleast_1d(np.asarray(f[k], dtype=np.float64)) for k in ("time", "freq", "amp", "width")]
        n = max(len(c) for c in cols)
        cols = [np.resize(c, n) for c in cols]  # as.data.frame recycling
        out.append((name,) + tuple(cols))
    return out


class Holder:
    """Keeps the numpy buffers behind a filled C struct alive."""

    def __init__(self):
        self.keep = []
        self._fmemo = {}  # formants converted once per object (a batch shares preset formant lists)
        self._amemo = {}  # anchors by value: one pair of buffers per distinct anchor set
        self._rmemo = {}  # injected draw arrays by identity (a batch often shares one stream)
        self._ramemo = {}  # the same for random_addrs: (array, address, count)

    def max_lengths_of(self, x):
        """r_max_lengths(x), once per string or (live) object."""
        key = ("L", x) if isinstance(x, str) or x is None else ("Lo", id(x))
        hit = self._fmemo.get(key)
        if hit is None:
            hit = self._fmemo[key] = (r_max_lengths(x), x)
        return hit[0]

    def formants_of(self, x):
        """sg_formants of an R formants argument (vowel string, formant lists or NA);
        the same string or the same (live) object is converted once per Holder."""
        key = ("s", x) if isinstance(x, str) else ("o", id(x))
        hit = self._fmemo.get(key)
        if hit is None:
            hit = self._fmemo[key] = (self.formants(as_formants(x)), x)  # x kept alive: its id stays unique
        return hit[0]

    def arr(self, a, dtype=np.float64):
        a = np.ascontiguousarray(np.asarray(a, dtype=dtype))
        self.keep.append(a)
        return a

    def anchors_of(self, x, time_to=1.0):
        """sg_anchors of an R anchors argument, converted once per distinct value
        (a batch repeats a few anchor sets: presets, defaults, NA)."""
        if isinstance(x, dict):
            t, v = x["time"], x["value"]
            key = ("d", tuple(t) if isinstance(t, (list, tuple, np.ndarray)) else (t,),
                   tuple(v) if isinstance(v, (list, tuple, np.ndarray)) else (v,))
        elif isinstance(x, (list, tuple, np.ndarray)):
            key = ("v", tuple(x), time_to)
        else:
            key = ("s", x if not (isinstance(x, float) and math.isnan(x)) else "NA", time_to)
        hit = self._amemo.get(key)
        if hit is None:  # one sg_anchors per distinct value; assigning it into a struct copies it
            hit = _abi.sg_anchors()
            if key[0] == "d" and len(key[1]) == len(key[2]) and key[1]:
                # time and value in one buffer; the pointers keep it alive
                a = np.array(key[1] + key[2], dtype=np.float64)
                n = len(key[1])
                hit.n = n
                hit.time = _abi.C.pointer(_abi.C.c_double.from_buffer(a))
                hit.value = _abi.C.pointer(_abi.C.c_double.from_buffer(a, 8 * n))
            else:
                an = as_anchors(x, time_to=time_to)
                if an is not None:
                    t, v = self.arr(an[0]), self.arr(an[1])
                    hit.n, hit.time, hit.value = len(t), _abi.dptr(t), _abi.dptr(v)
            self._amemo[key] = hit
        return hit

    def anchors(self, an):
        if an is None:
            s = _abi.sg_anchors()
            s.n = 0
            return s
        key = (tuple(an[0]), tuple(an[1]))
        hit = self._amemo.get(key)
        if hit is None:
            t, v = self.arr(an[0]), self.arr(an[1])
            hit = self._amemo[key] = (len(t), _abi.dptr(t), _abi.dptr(v))
        s = _abi.sg_anchors()
        s.n, s.time, s.value = hit
        return s

    def formants(self, fl):
        s = _abi.sg_formants()
        if not fl:
            s.n_formants = 0
            s.f1_index = -1
            return s
        s.n_formants = len(fl)
        names = [f[0] for f in fl]
        s.f1_index = names.index("f1") if "f1" in names else -1
        npnt = self.arr([len(f[1]) for f in fl], np.int32)
        cat = [self.arr(np.concatenate([f[k] for f in fl])) for k in (1, 2, 3, 4)]
        s.n_points = _abi.iptr(npnt)
        s.time, s.freq, s.amp, s.width = (_abi.dptr(c) for c in cat)
        return s

    def random_addrs(self, normals=None, uniforms=None):
        """(normals address, count, uniforms address, count) of injected draw arrays
        for the bulk descriptor writer (0, 0 for an absent array); the arrays are
        kept alive, float64 C-contiguous ones without a copy."""
        out = []
        for x in (normals, uniforms):
            if x is None:
                out += (0, 0)
                continue
            hit = self._ramemo.get(id(x))
            if hit is None or hit[0] is not x:
                if type(x) is np.ndarray and x.dtype == np.float64 and x.flags.c_contiguous and x.flags.writeable:
                    p = _abi.C.addressof(_abi.C.c_double.from_buffer(x)) if x.shape[0] else 0
                    n = x.shape[0]
                else:
                    a = self.arr(x)
                    p, n = (a.ctypes.data if len(a) else 0), len(a)
                hit = self._ramemo[id(x)] = (x, p, n)
            out += (hit[1], hit[2])
        return out

    def random(self, normals=None, uniforms=None, rng=None):
        """sg_random from injected arrays and/or a draw source `rng` (an object
        with standard_normal(), random() and gamma(shape, scale), e.g. a
        numpy Generator) bound to the norm/unif/gamma callbacks."""
        r = _abi.sg_random()

        def buf(x):
            hit = self._rmemo.get(id(x))
            if hit is None or hit[0] is not x:
                if type(x) is np.ndarray and x.dtype == np.float64 and x.flags.c_contiguous and x.flags.writeable:
                    # a window of one stream (kept alive by the memo): pointer without a copy or a cast
                    p, n = _abi.C.pointer(_abi.C.c_double.from_buffer(x)), x.shape[0]
                else:
                    a = self.arr(x)
                    p, n = _abi.dptr(a), len(a)
                hit = self._rmemo[id(x)] = (x, p, n)
            return hit[1], hit[2]
        if normals is not None:
            r.normals, r.n_normals = buf(normals)
        if uniforms is not None:
            r.uniforms, r.n_uniforms = buf(uniforms)
        if rng is not None and hasattr(rng, "bind"):  # RRng: native callbacks into the library
            rng.bind(r)
            self.keep.append(rng)
        elif rng is not None:
            def unif_n(_u, out, n):  # runif(n) in one call (ABI 5 bulk callback)
                np.ctypeslib.as_array(out, (n,))[:] = rng.random(n)
            cbs = (_abi.NORM_CB(lambda _u: float(rng.standard_normal())),
                   _abi.UNIF_CB(lambda _u: float(rng.random())),
                   _abi.GAMMA_CB(lambda _u, shape, rate: float(rng.gamma(shape, 1.0 / rate))),
                   _abi.UNIF_N_CB(unif_n))
            self.keep.extend(cbs)
            r.norm_cb, r.unif_cb, r.gamma_cb, r.unif_n_cb = cbs
        return r


def resolve_soundgen_kwargs(kw):
    """Fill soundgen() defaults for missing args; returns a plain dict."""
    unknown = kw.keys() - SOUNDGEN_DEFAULTS.keys()
    if unknown:
        raise TypeError("soundgen(): unused argument(s) %s" % sorted(unknown))
    a = dict(SOUNDGEN_DEFAULTS)
    a.update(kw)
    te = dict(TEMP_EFFECTS_DEFAULT)
    if a.get("tempEffects"):
        te.update(a["tempEffects"])
    a["tempEffects"] = te
    return a


# the scalar (double) fields of sg_soundgen_args, written in one structured-array
# store per call instead of one ctypes setattr each
_SG_SCALARS = [f for f, t in _abi.sg_soundgen_args._fields_ if t is _abi.C.c_double]
_SG_SCALAR_DT = np.dtype({"names": _SG_SCALARS, "formats": ["<f8"] * len(_SG_SCALARS),
                          "offsets": [getattr(_abi.sg_soundgen_args, f).offset for f in _SG_SCALARS],
                          "itemsize": _abi.C.sizeof(_abi.sg_soundgen_args)})
_NAN = float("nan")
_ACTIONS = {"adjust": 0, "abort": 1, "ignore": 2}


def _scalar(v):
    if v is None or (isinstance(v, str) and v == "NA"):
        return _NAN
    return float(v)


def scalar_view(args_array, n):
    """Structured numpy view of the scalar fields of a ctypes sg_soundgen_args array
    (fill_soundgen_args writes a call's scalars with one store into it)."""
    return np.frombuffer(args_array, dtype=_SG_SCALAR_DT, count=n)


def fill_soundgen_args(h, kw, out=None, scalars=None, i=0):
    """kwargs (R names) -> sg_soundgen_args (buffers kept alive by h); fills `out`
    in place when given (scalars: scalar_view of the array `out` belongs to, i:
    its index there)."""
    a = resolve_soundgen_kwargs(kw)
    s = _abi.sg_soundgen_args() if out is None else out
    vals = tuple(map(a.__getitem__, _SG_SCALARS))
    if None in vals or "NA" in vals:
        vals = tuple(map(_scalar, vals))
    if scalars is None:
        scalars, i = np.frombuffer(s, dtype=_SG_SCALAR_DT, count=1), 0
    scalars[i] = vals
    te = a["tempEffects"]
    s.tempEffects = (C_double8())(*[float(te[k]) for k in TEMP_EFFECTS_ORDER])
    s.pitchAnchors = h.anchors_of(a["pitchAnchors"])
    s.pitchAnchorsGlobal = h.anchors_of(a["pitchAnchorsGlobal"])
    s.amplAnchors = h.anchors_of(a["amplAnchors"])
    s.amplAnchorsGlobal = h.anchors_of(a["amplAnchorsGlobal"])
    s.mouthAnchors = h.anchors_of(a["mouthAnchors"])
    s.noiseAnchors = h.anchors_of(a["noiseAnchors"], time_to=a["sylLen"])
    s.formants = h.formants_of(a["formants"])
    s.formantsNoise = h.formants_of(a["formantsNoise"])
    s.formantsNoise_rlen = h.max_lengths_of(a["formantsNoise"])
    s.invalidArgAction = _ACTIONS[a["invalidArgAction"]]
    return s


_D8 = _abi.C.c_double * 8


def C_double8():
    return _D8


# ---------------------------------------------------------------- bulk writer
# Marshalling a batch one ctypes field at a time cost ~90 us per call (a 16k-call
# C5 chunk took longer to marshal than to plan natively). ArgsWriter keeps, per
# call, one Python tuple of plain numbers (scalars, tempEffects, and the
# (n, address, address) of every anchor and formant struct) and writes all calls
# at the end through a structured numpy view of the sg_soundgen_args array, field
# by field. Anchor and formant buffers are converted once per object (identity)
# or value and kept alive by the Holder. The bytes written equal those of
# fill_soundgen_args (tests/test_planner.py compares them).
_ANCHOR_FIELDS = ("pitchAnchors", "pitchAnchorsGlobal", "amplAnchors", "amplAnchorsGlobal", "mouthAnchors",
                  "noiseAnchors")
_FORMANT_FIELDS = ("formants", "formantsNoise")
_FORMANT_SUB = ("n_formants", "f1_index", "n_points", "time", "freq", "amp", "width")


def _addr(p):
    """Address held by a ctypes pointer (0 for NULL)."""
    return _abi.C.cast(p, _abi.C.c_void_p).value or 0


def _wide_dtypes():
    S = _abi.sg_soundgen_args
    names, formats, offsets = [], [], []

    def add(name, fmt, off):
        names.append(name)
        formats.append(fmt)
        offsets.append(off)
    for f in _SG_SCALARS:
        add(f, "<f8", getattr(S, f).offset)
    add("tempEffects", ("<f8", (8,)), S.tempEffects.offset)
    for f in _ANCHOR_FIELDS:
        o = getattr(S, f).offset
        add(f + ".n", "<i4", o + _abi.sg_anchors.n.offset)
        add(f + ".time", "<u8", o + _abi.sg_anchors.time.offset)
        add(f + ".value", "<u8", o + _abi.sg_anchors.value.offset)
    for f in _FORMANT_FIELDS:
        o = getattr(S, f).offset
        for sub in _FORMANT_SUB:
            add(f + "." + sub, "<i4" if sub in ("n_formants", "f1_index") else "<u8",
                o + getattr(_abi.sg_formants, sub).offset)
    add("invalidArgAction", "<i4", S.invalidArgAction.offset)
    add("formantsNoise_rlen", "<i4", S.formantsNoise_rlen.offset)
    view = np.dtype({"names": names, "formats": formats, "offsets": offsets, "itemsize": _abi.C.sizeof(S)})
    packed = np.dtype({"names": names, "formats": formats})
    return view, packed


_WIDE_VIEW, _WIDE_PACKED = _wide_dtypes()
_TE_DEFAULT = tuple(float(TEMP_EFFECTS_DEFAULT[k]) for k in TEMP_EFFECTS_ORDER)
_DEFAULT_KEYS = SOUNDGEN_DEFAULTS.keys()


class ArgsWriter:
    """Collects soundgen() calls for one sg_soundgen_args array and writes them
    all in finish() (fields equal to fill_soundgen_args')."""

    def __init__(self, h, args_array, n):
        self.h, self.args, self.n = h, args_array, n
        self.rows, self.idx = [], []
        self._tmemo = {}   # anchors by (identity, time_to): (object, (n, time, value))
        self._ftmemo = {}  # formants by identity / string: (object, 7-tuple)

    def _anchor(self, x, time_to):
        if type(x) is dict:  # a well-formed data frame does not depend on time_to
            hit = self._tmemo.get(id(x))
            if hit is not None and hit[0] is x:
                return hit[1]
            t, v = x["time"], x["value"]
            tt = t if isinstance(t, (list, tuple, np.ndarray)) else (t,)
            vv = v if isinstance(v, (list, tuple, np.ndarray)) else (v,)
            n = len(tt)
            if n and n == len(vv):  # anchors_of' time-and-value buffer, built directly
                a = np.fromiter((*tt, *vv), dtype=np.float64, count=2 * n)
                self.h.keep.append(a)
                p = _abi.C.addressof(_abi.C.c_double.from_buffer(a))
                trip = (n, p, p + 8 * n)
                self._tmemo[id(x)] = (x, trip)
                return trip
        key = (id(x), time_to)
        hit = self._tmemo.get(key)
        if hit is not None and hit[0] is x:
            return hit[1]
        trip = None
        if trip is None:
            s = self.h.anchors_of(x, time_to=time_to)
            trip = (s.n, _addr(s.time), _addr(s.value))
        self._tmemo[key] = (x, trip)
        return trip

    def _formants(self, x):
        key = ("s", x) if isinstance(x, str) else ("o", id(x))
        hit = self._ftmemo.get(key)
        if hit is None or (key[0] == "o" and hit[0] is not x):
            s = self.h.formants_of(x)
            hit = self._ftmemo[key] = (x, (s.n_formants, s.f1_index, _addr(s.n_points), _addr(s.time),
                                           _addr(s.freq), _addr(s.amp), _addr(s.width)))
        return hit[1]

    def add(self, i, kw):
        unknown = kw.keys() - _DEFAULT_KEYS
        if unknown:
            raise TypeError("soundgen(): unused argument(s) %s" % sorted(unknown))
        a = dict(SOUNDGEN_DEFAULTS)
        a.update(kw)
        vals = tuple(map(a.__getitem__, _SG_SCALARS))
        if None in vals or "NA" in vals:
            vals = tuple(map(_scalar, vals))
        te_in = kw.get("tempEffects")
        if te_in:
            te = dict(TEMP_EFFECTS_DEFAULT)
            te.update(te_in)
            te = tuple(float(te[k]) for k in TEMP_EFFECTS_ORDER)
        else:
            te = _TE_DEFAULT
        an = self._anchor
        row = (vals + (te,) + an(a["pitchAnchors"], 1.0) + an(a["pitchAnchorsGlobal"], 1.0)
               + an(a["amplAnchors"], 1.0) + an(a["amplAnchorsGlobal"], 1.0) + an(a["mouthAnchors"], 1.0)
               + an(a["noiseAnchors"], a["sylLen"]) + self._formants(a["formants"])
               + self._formants(a["formantsNoise"])
               + (_ACTIONS[a["invalidArgAction"]], self.h.max_lengths_of(a["formantsNoise"])))
        self.rows.append(row)
        self.idx.append(i)

    def finish(self):
        if not self.rows:
            return
        packed = np.array(self.rows, dtype=_WIDE_PACKED)
        view = np.frombuffer(self.args, dtype=_WIDE_VIEW, count=self.n)
        idx = np.asarray(self.idx, dtype=np.int64)
        whole = len(idx) == self.n
        for name in _WIDE_PACKED.names:
            if whole:
                view[name] = packed[name]
            else:
                view[name][idx] = packed[name]
        self.rows, self.idx = [], []


def fill_harm_params(kw):
    unknown = set(kw) - set(HARM_DEFAULTS)
    if unknown:
        raise TypeError("generateHarmonics(): unused argument(s) %s" % sorted(unknown))
    p = dict(HARM_DEFAULTS)
    p.update(kw)
    s = _abi.sg_harm_params()
    for f in _abi.HARM_FIELDS:
        setattr(s, f, float(p[f]))
    return s
