"""The R drop-in boundary, driven the way R drives it.

r/src/sg_r_shim.c (the .Call shim a maintainer adds to the reference package)
is compiled against tests/rmock (a test double of the R C API it calls: SEXP
vectors, lists with names, matrices, Rf_error unwinding, R_registerRoutines,
R's RNG as the library's restatement) and linked to libsoundgen_hip.so as
r/src/Makevars links the package. Each test builds the exact argument objects
the R wrappers of r/R/soundgen_hip.R hand to .Call -- the wrapper bodies are
restated below, line for line -- and calls the routine by its registered name.

CPU: the registration table, and the shim's argument checks and error path
(R's stop() semantics, protect stack reset). GPU: every entry against the
oracle on R's RNG stream (set.seed), including how far the stream advanced.
"""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from soundgen_beta_amd import native, rargs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MOCK = os.path.join(ROOT, "tests", "rmock")
TOL = 1e-5

ROUTINES = {"C_sg_generate_harmonics": 3, "C_sg_soundgen": 1, "C_sg_generate_noise": 4,
            "C_sg_spectral_envelope": 5, "C_sg_formant_filter": 4, "C_sg_soundgen_batch": 2}
REALSXP, INTSXP, VECSXP = 14, 13, 19


class RShim:
    """The shim library plus the R-object builders of the test double."""

    def __init__(self):
        native.lib()  # libsoundgen_hip.so first (the shim links it)
        subprocess.run(["make", "-s", "-C", MOCK], check=True, timeout=120)
        L = C.CDLL(os.path.join(MOCK, "_build", "librshim_test.so"))
        vp = C.c_void_p
        for f, res, args in (("rm_null", vp, []), ("rm_real", vp, [C.c_ssize_t, C.POINTER(C.c_double)]),
                             ("rm_int", vp, [C.c_ssize_t, C.POINTER(C.c_int)]), ("rm_lgl_na", vp, []),
                             ("rm_matrix", vp, [C.c_int, C.c_int, C.POINTER(C.c_double)]),
                             ("rm_list", vp, [C.c_int, C.POINTER(vp), C.POINTER(C.c_char_p)]),
                             ("rm_type", C.c_int, [vp]), ("rm_length", C.c_ssize_t, [vp]),
                             ("rm_real_ptr", C.POINTER(C.c_double), [vp]), ("rm_nrow", C.c_int, [vp]),
                             ("rm_ncol", C.c_int, [vp]), ("rm_elt", vp, [vp, C.c_ssize_t]),
                             ("rm_call", C.c_int, [C.c_char_p, C.c_int, C.POINTER(vp), C.POINTER(vp)]),
                             ("rm_error", C.c_char_p, []), ("rm_protect_depth", C.c_int, []),
                             ("rm_init", C.c_int, []), ("rm_n_routines", C.c_int, []),
                             ("rm_routine", C.c_char_p, [C.c_int, C.POINTER(C.c_int)]),
                             ("rm_set_seed", None, [C.c_int]), ("rm_unif", C.c_double, []),
                             ("rm_unload", None, [])):
            getattr(L, f).restype = res
            getattr(L, f).argtypes = args
        self.L = L
        assert L.rm_init() == 0  # R_useDynamicSymbols(dll, FALSE)

    # ---- R objects
    def null(self):
        return self.L.rm_null()

    def na(self):
        return self.L.rm_lgl_na()

    def real(self, x):
        a = np.ascontiguousarray(np.atleast_1d(np.asarray(x, dtype=np.float64)))
        return self.L.rm_real(len(a), a.ctypes.data_as(C.POINTER(C.c_double)))

    def int_(self, x):
        a = np.ascontiguousarray(np.atleast_1d(np.asarray(x, dtype=np.int32)))
        return self.L.rm_int(len(a), a.ctypes.data_as(C.POINTER(C.c_int)))

    def matrix(self, m):  # R stores column-major
        m = np.asarray(m, dtype=np.float64)
        a = np.ascontiguousarray(m.T.ravel())
        return self.L.rm_matrix(m.shape[0], m.shape[1], a.ctypes.data_as(C.POINTER(C.c_double)))

    def list(self, items, named=True):
        """list(k = v, ...) from (name, SEXP) pairs, or unnamed from SEXPs."""
        if named:
            names = (C.c_char_p * max(1, len(items)))(*[k.encode() for k, _ in items])
            vals = [v for _, v in items]
        else:
            names, vals = None, list(items)
        arr = (C.c_void_p * max(1, len(vals)))(*vals)
        return self.L.rm_list(len(vals), arr, names)

    def data_frame(self, time, value):
        return self.list([("time", self.real(time)), ("value", self.real(value))])

    # ---- .Call
    def call(self, name, *args):
        out = C.c_void_p()
        argv = (C.c_void_p * max(1, len(args)))(*args)
        rc = self.L.rm_call(name.encode(), len(args), argv, C.byref(out))
        if rc == -1:
            raise RError(self.L.rm_error().decode())
        assert rc == 0, (name, rc)
        assert self.L.rm_protect_depth() == 0  # PROTECT / UNPROTECT balanced
        return out.value

    def as_array(self, x):
        assert self.L.rm_type(x) == REALSXP
        n = self.L.rm_length(x)
        return np.ctypeslib.as_array(self.L.rm_real_ptr(x), (n,)).copy() if n else np.zeros(0)

    def as_matrix(self, x):
        nr, nc = self.L.rm_nrow(x), self.L.rm_ncol(x)
        return self.as_array(x).reshape(nc, nr).T


class RError(Exception):
    pass


@pytest.fixture(scope="module")
def shim():
    return RShim()


# ---- the R wrappers of r/R/soundgen_hip.R, restated --------------------------

def sg_anchors(R, v):
    """.sg_anchors(v): numeric vector -> data.frame(time = seq(0, 1, ...)); a
    list / data.frame -> data.frame of doubles; NA / NULL -> NULL."""
    if v is None or (isinstance(v, float) and np.isnan(v)):
        return R.null()
    if isinstance(v, dict):
        return R.data_frame(v["time"], v["value"])
    v = np.atleast_1d(np.asarray(v, dtype=np.float64))
    return R.data_frame(np.linspace(0, 1, len(v)) if len(v) > 1 else [0.0], v)


def sg_flatten_formants(R, formants):
    """.sg_flatten_formants(formants): list(n_points, f1_index, time, freq, amp, width)."""
    fs = rargs.as_formants(formants)
    if not fs:
        return R.null()
    names = [f[0] for f in fs]
    return R.list([("n_points", R.int_([len(f[1]) for f in fs])),
                   ("f1_index", R.int_([names.index("f1") if "f1" in names else -1])),
                   ("time", R.real(np.concatenate([f[1] for f in fs]))),
                   ("freq", R.real(np.concatenate([f[2] for f in fs]))),
                   ("amp", R.real(np.concatenate([f[3] for f in fs]))),
                   ("width", R.real(np.concatenate([f[4] for f in fs])))])


def r_generateNoise(R, len, noiseAnchors=None, rolloffNoise=-6, attackLen=10, windowLength_points=1024,
                    samplingRate=16000, overlap=75, throwaway=-120, filterNoise=None):
    """generateNoise() of r/R/soundgen_hip.R (R/source.R:57-68 formals)."""
    if noiseAnchors is None:
        noiseAnchors = {"time": [0, 300], "value": [-120, -120]}
    pars = R.list([("rolloffNoise", R.real(rolloffNoise)), ("attackLen", R.real(attackLen)),
                   ("windowLength_points", R.real(windowLength_points)), ("samplingRate", R.real(samplingRate)),
                   ("overlap", R.real(overlap)), ("throwaway", R.real(throwaway))])
    fn = R.null()
    if filterNoise is not None:
        m = np.asarray(filterNoise, dtype=np.float64)
        fn = R.matrix(m if m.ndim == 2 else m[:, None])
    return R.as_array(R.call("C_sg_generate_noise", R.real(len), sg_anchors(R, noiseAnchors), pars, fn))


def r_getSpectralEnvelope(R, nr, nc, formants=None, formantDep=1, rolloffLip=6, mouthAnchors=None,
                          mouthOpenThres=0, openMouthBoost=0, vocalTract=None, temperature=0, formDrift=.3,
                          formDisp=.2, formantDepStoch=30, smoothLinearFactor=1, samplingRate=16000,
                          speedSound=35400):
    """getSpectralEnvelope() of r/R/soundgen_hip.R (R/sourceSpectrum.R:261-283 formals)."""
    pars = R.list([("formantDep", R.real(formantDep)), ("rolloffLip", R.real(rolloffLip)),
                   ("mouthOpenThres", R.real(mouthOpenThres)), ("openMouthBoost", R.real(openMouthBoost)),
                   ("vocalTract", R.real(np.nan if vocalTract is None else vocalTract)),
                   ("temperature", R.real(temperature)), ("formDrift", R.real(formDrift)),
                   ("formDisp", R.real(formDisp)), ("formantDepStoch", R.real(formantDepStoch)),
                   ("smoothLinearFactor", R.real(smoothLinearFactor)), ("samplingRate", R.real(samplingRate)),
                   ("speedSound", R.real(speedSound))])
    return R.as_matrix(R.call("C_sg_spectral_envelope", R.int_(nr), R.int_(nc), sg_flatten_formants(R, formants),
                              pars, sg_anchors(R, mouthAnchors)))


# formals(soundgen_hip) (R/soundgen.R:208-277), NA as None
SOUNDGEN_FORMALS = dict(
    repeatBout=1, nSyl=1, sylLen=300, pauseLen=200,
    pitchAnchors={"time": [0, .1, .9, 1], "value": [100, 150, 135, 100]}, pitchAnchorsGlobal=None,
    temperature=0.025, tempEffects={}, maleFemale=0, creakyBreathy=0, nonlinBalance=0, nonlinDep=50,
    jitterLen=1, jitterDep=3, vibratoFreq=5, vibratoDep=0, shimmerDep=0, attackLen=50, rolloff=-12,
    rolloffOct=-12, rolloffKHz=-6, rolloffParab=0, rolloffParabHarm=3, rolloffLip=6,
    formants={"f1": dict(time=0, freq=860, amp=30, width=120), "f2": dict(time=0, freq=1280, amp=40, width=120),
              "f3": dict(time=0, freq=2900, amp=25, width=200)},
    formantDep=1, formantDepStoch=30, vocalTract=15.5, subFreq=100, subDep=100, shortestEpoch=300, amDep=0,
    amFreq=30, amShape=0, noiseAnchors={"time": [0, 300], "value": [-120, -120]}, formantsNoise=None,
    rolloffNoise=-14, mouthAnchors={"time": [0, 1], "value": [.5, .5]}, amplAnchors=None, amplAnchorsGlobal=None,
    samplingRate=16000, windowLength=50, overlap=75, addSilence=100, pitchFloor=50, pitchCeiling=3500,
    pitchSamplingRate=3500, throwaway=-120, invalidArgAction="adjust")
TE = ("sylLenDep", .02), ("formDrift", .3), ("formDisp", .2), ("pitchDriftDep", .5), ("pitchDriftFreq", .125), \
     ("pitchAnchorsDep", .05), ("noiseAnchorsDep", .1), ("amplAnchorsDep", .1)
ANCHORS = ("pitchAnchors", "pitchAnchorsGlobal", "noiseAnchors", "mouthAnchors", "amplAnchors", "amplAnchorsGlobal")


def sg_soundgen_args(R, call):
    """.sg_soundgen_args(a) on formals(soundgen_hip) overridden by `call`: the
    named list soundgen_hip / soundgen_batch hand to .Call, in formals order."""
    a = dict(SOUNDGEN_FORMALS)
    a.update(call)
    items = []
    for k, v in a.items():
        if k == "tempEffects":
            te = dict(TE)
            te.update(v or {})
            items.append((k, R.real([te[n] for n, _ in TE])))
        elif k == "invalidArgAction":
            items.append((k, R.int_(["adjust", "abort", "ignore"].index(v))))
        elif k in ANCHORS:
            items.append((k, sg_anchors(R, v)))
        elif k in ("formants", "formantsNoise"):
            continue
        else:
            items.append((k, R.real(v)))
    items.append(("formantsNoise_rlen", R.int_(rargs.r_max_lengths(a["formantsNoise"]))))
    for k in ("formants", "formantsNoise"):  # a$x_flat = NULL drops the entry (R's `$<-`)
        if rargs.as_formants(a[k]):
            items.append((k + "_flat", sg_flatten_formants(R, a[k])))
    return R.list(items)


def r_soundgen_batch(R, calls, devices=None):
    """soundgen_batch(calls, devices): the node of `devices` (NULL: device 0; [-1]: every visible device)."""
    dev = R.null() if devices is None else R.int_(devices)
    out = R.call("C_sg_soundgen_batch", R.list([sg_soundgen_args(R, c) for c in calls], named=False), dev)
    assert R.L.rm_type(out) == VECSXP and R.L.rm_length(out) == len(calls)
    return [R.as_array(R.L.rm_elt(out, i)) for i in range(len(calls))]


# ---- CPU ---------------------------------------------------------------------

def test_shim_registers_every_entry(shim):
    got = {}
    for i in range(shim.L.rm_n_routines()):
        n = C.c_int()
        name = shim.L.rm_routine(i, C.byref(n)).decode()
        got[name] = n.value
    assert got == ROUTINES
    # every .Call of the R wrappers names a registered routine with its arity
    src = open(os.path.join(ROOT, "r", "R", "soundgen_hip.R")).read()
    called = re.findall(r"\.Call\((C_\w+)", src)
    assert set(called) >= {"C_sg_generate_harmonics", "C_sg_soundgen", "C_sg_generate_noise",
                           "C_sg_spectral_envelope", "C_sg_soundgen_batch"}
    assert set(called) <= set(ROUTINES)
    for name in ("generateHarmonics", "soundgen_hip", "generateNoise", "getSpectralEnvelope", "soundgen_batch"):
        assert re.search(r"^%s = function\(" % name, src, re.M), name


def test_shim_argument_errors_unwind_like_stop(shim):
    R = shim
    with pytest.raises(RError, match="nr and nc must be positive"):
        R.call("C_sg_spectral_envelope", R.int_(0), R.int_(5), R.null(), R.list([]), R.null())
    with pytest.raises(RError, match="formants must be flattened"):
        R.call("C_sg_spectral_envelope", R.int_(10), R.int_(5), R.list([("x", R.real(1))]), R.list([]), R.null())
    with pytest.raises(RError, match="windowLength_points / 2 rows"):
        R.call("C_sg_generate_noise", R.real(1000), R.null(), R.list([("windowLength_points", R.real(64))]),
               R.matrix(np.ones((31, 2))))
    with pytest.raises(RError, match="len must be"):
        R.call("C_sg_generate_noise", R.real(-1), R.null(), R.list([]), R.null())
    with pytest.raises(RError, match="list of argument lists"):
        R.call("C_sg_soundgen_batch", R.real(1), R.null())
    with pytest.raises(RError, match="integer vector of 1 to 64"):
        R.call("C_sg_soundgen_batch", R.list([sg_soundgen_args(R, dict(sylLen=100))], named=False), R.real(0))
    with pytest.raises(RError, match="anchors must be numeric"):
        R.call("C_sg_soundgen", R.list([("pitchAnchors", R.list([("time", R.int_([0, 1])),
                                                                  ("value", R.int_([1, 2]))]))]))
    assert R.L.rm_protect_depth() == 0
    # an empty batch returns list() without touching the device
    out = R.call("C_sg_soundgen_batch", R.list([], named=False), R.null())
    assert R.L.rm_type(out) == VECSXP and R.L.rm_length(out) == 0


def test_shim_without_gpu_stops_with_the_device_message(shim):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    R = shim
    with pytest.raises(RError, match="no usable MI355X"):
        r_getSpectralEnvelope(R, 64, 3, formants="a")
    with pytest.raises(RError, match="no usable MI355X"):
        r_soundgen_batch(R, [dict(sylLen=100, temperature=0)])


# ---- GPU: every entry vs the oracle on R's RNG ------------------------------

def _rms(a, b):
    return float(np.sqrt(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2)))


def _same_stream_position(R, rr):
    """The shim's R stream and the oracle's generator drew the same number of values."""
    assert R.L.rm_unif() == rr.random()


@pytest.mark.gpu
@pytest.mark.parametrize("case", [
    dict(formants="a", samplingRate=44100),
    dict(formants="aui", samplingRate=16000, mouthAnchors={"time": [0, 1], "value": [0, .8]}, mouthOpenThres=.2,
         openMouthBoost=5),
    dict(formants=None, vocalTract=17),
    dict(formants="a", temperature=0.1, vocalTract=15, formantDepStoch=20),
    dict(formants={"f1": dict(time=[0, 1], freq=[700, 400], amp=[30, 25], width=[100, 150]),
                   "f2": dict(time=[0, 1], freq=[1200, 2100], amp=30, width=120)},
         temperature=0.2, samplingRate=44100),
])
def test_shim_spectral_envelope_vs_oracle(shim, oracle, case):
    from soundgen_beta_amd.rrng import RRng
    nr, nc = (1102, 23) if case.get("samplingRate") == 44100 else (400, 17)
    shim.L.rm_set_seed(7)
    got = r_getSpectralEnvelope(shim, nr, nc, **case)
    rr = RRng(7)
    want = oracle.spectral_envelope(nr, nc, rng=rr, **case)
    assert got.shape == (nr, nc)
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=0)
    _same_stream_position(shim, rr)


@pytest.mark.gpu
def test_shim_generate_noise_vs_oracle(shim, oracle):
    from soundgen_beta_amd.rrng import RRng
    filt = np.abs(np.random.default_rng(3).normal(1, .5, size=(400, 4)))
    for seed, kw in ((1, dict(len=16000, noiseAnchors={"time": [0, 1000], "value": [-30, -10]})),
                     (2, dict(len=9000, noiseAnchors={"time": [0, 500], "value": [-20, -20]}, rolloffNoise=-12,
                              windowLength_points=800, filterNoise=filt)),
                     (3, dict(len=5000))):
        shim.L.rm_set_seed(seed)
        got = r_generateNoise(shim, **kw)
        rr = RRng(seed)
        k = dict(kw)
        want = oracle.generate_noise(k.pop("len"), k.pop("noiseAnchors", {"time": [0, 300], "value": [-120, -120]}),
                                     rng=rr, **k)
        assert len(got) == len(want) == kw["len"]
        assert _rms(got, want) <= TOL
        _same_stream_position(shim, rr)


SHIM_CALLS = [
    dict(sylLen=400, temperature=0, addSilence=0, pitchAnchors=[120, 180]),
    dict(sylLen=300, temperature=0.1, addSilence=20, formants="ae", noiseAnchors={"time": [0, 300],
                                                                                  "value": [-30, -20]}),
    dict(sylLen=250, nSyl=2, pauseLen=80, temperature=0.05, samplingRate=22050, jitterDep=1, shimmerDep=5),
    dict(sylLen=350, temperature=0.05, nonlinBalance=60, subFreq=90, subDep=60, pitchAnchors=[300, 400, 250],
         tempEffects={"formDrift": 0.5}),
    dict(sylLen=200, pitchAnchors=None, noiseAnchors={"time": [0, 200], "value": [-10, -10]},
         formantsNoise="i", temperature=0.1),
]


@pytest.mark.gpu
def test_shim_soundgen_and_batch_vs_oracle(shim, oracle):
    """soundgen_hip (C_sg_soundgen) call by call and soundgen_batch
    (C_sg_soundgen_batch) over the same calls after the same set.seed(): both
    equal the oracle drawing one R stream in call order."""
    from soundgen_beta_amd.rrng import RRng
    rr = RRng(11)
    want = []
    for c in SHIM_CALLS:
        a = dict(SOUNDGEN_FORMALS)
        a.update(c)
        a.pop("invalidArgAction")
        want.append(oracle.soundgen(rng=rr, **a))
    shim.L.rm_set_seed(11)
    single = [shim.as_array(shim.call("C_sg_soundgen", sg_soundgen_args(shim, c))) for c in SHIM_CALLS]
    _same_stream_position(shim, rr)
    rr = RRng(11)
    for c in SHIM_CALLS:
        a = dict(SOUNDGEN_FORMALS)
        a.update(c)
        a.pop("invalidArgAction")
        oracle.soundgen(rng=rr, **a)
    shim.L.rm_set_seed(11)
    batched = r_soundgen_batch(shim, SHIM_CALLS)
    _same_stream_position(shim, rr)
    # the same batch over a 2-way node on device 0 (two shards, two streams): R's
    # stream recorded in call order, the shards planned from it
    shim.L.rm_set_seed(11)
    node2 = r_soundgen_batch(shim, SHIM_CALLS, devices=[0, 0])
    u_node = shim.L.rm_unif()
    shim.L.rm_set_seed(11)
    r_soundgen_batch(shim, SHIM_CALLS)
    assert shim.L.rm_unif() == u_node  # both leave R's stream at one position
    for i, (s, b, b2, w) in enumerate(zip(single, batched, node2, want)):
        assert len(s) == len(b) == len(b2) == len(w), i
        assert _rms(s, w) <= TOL, i
        np.testing.assert_array_equal(s, b)
        np.testing.assert_array_equal(b, b2)


@pytest.mark.gpu
def test_shim_generate_harmonics_and_batch_error(shim, oracle):
    R = shim
    pitch = np.full(1750, 140.0)
    pars = R.list([("samplingRate", R.real(16000)), ("rolloff", R.real(-12)), ("attackLen", R.real(20)),
                   ("jitterDep", R.real(0.5)), ("temperature", R.real(0.05))])
    from soundgen_beta_amd.rrng import RRng
    R.L.rm_set_seed(5)
    got = R.as_array(R.call("C_sg_generate_harmonics", R.real(pitch), pars, R.null()))
    rr = RRng(5)
    want = oracle.generate_harmonics(pitch, rng=rr, samplingRate=16000, rolloff=-12, attackLen=20, jitterDep=0.5,
                                     temperature=0.05)
    assert len(got) == len(want) and _rms(got, want) <= TOL
    _same_stream_position(R, rr)
    # a call R would stop() on stops the batch, naming it
    with pytest.raises(RError, match="call 2"):
        r_soundgen_batch(R, [dict(sylLen=100, temperature=0), dict(sylLen=100, samplingRate=-5, temperature=0,
                                                                   invalidArgAction="abort")])
