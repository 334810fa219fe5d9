"""ctypes mirror of include/soundgen_hip.h (data layout only, no logic).

The same plain structs are filled for the product library (libsoundgen_hip.so)
and, in tests, for the CPU oracle (oracle/_build/libsg_oracle.so).
"""
import ctypes as C

import numpy as np

SG_OK = 0
SG_E_ARG = -1
SG_E_DOMAIN = -2
SG_E_RANDOM = -3
SG_E_UNSUPPORTED = -4
SG_E_DEVICE = -5
SG_E_CAPACITY = -6
SG_E_NOMEM = -7
SG_ERR_NAMES = {0: "SG_OK", -1: "SG_E_ARG", -2: "SG_E_DOMAIN", -3: "SG_E_RANDOM",
                -4: "SG_E_UNSUPPORTED", -5: "SG_E_DEVICE", -6: "SG_E_CAPACITY",
                -7: "SG_E_NOMEM"}

SG_CALL_SOUNDGEN = 0
SG_CALL_HARMONICS = 1

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)


class sg_anchors(C.Structure):
    _fields_ = [("n", C.c_int32), ("time", _dp), ("value", _dp)]


class sg_formants(C.Structure):
    _fields_ = [("n_formants", C.c_int32), ("f1_index", C.c_int32),
                ("n_points", _ip), ("time", _dp), ("freq", _dp),
                ("amp", _dp), ("width", _dp)]


class sg_mel_params(C.Structure):
    _fields_ = [("samplingRate", C.c_double), ("windowLength", C.c_double), ("overlap", C.c_double),
                ("step", C.c_double), ("throwaway", C.c_double), ("maxFreq", C.c_double),
                ("penalizeLengthDif", C.c_int32), ("pad", C.c_int32)]


NORM_CB = C.CFUNCTYPE(C.c_double, C.c_void_p)
UNIF_CB = C.CFUNCTYPE(C.c_double, C.c_void_p)
GAMMA_CB = C.CFUNCTYPE(C.c_double, C.c_void_p, C.c_double, C.c_double)
UNIF_N_CB = C.CFUNCTYPE(None, C.c_void_p, _dp, C.c_int64)  # ABI 5: runif(n) into out


class sg_random(C.Structure):
    _fields_ = [("normals", _dp), ("n_normals", C.c_int64),
                ("uniforms", _dp), ("n_uniforms", C.c_int64),
                ("norm_cb", NORM_CB), ("unif_cb", UNIF_CB), ("gamma_cb", GAMMA_CB),
                ("user", C.c_void_p), ("unif_n_cb", UNIF_N_CB)]


HARM_FIELDS = ["attackLen", "nonlinBalance", "nonlinDep", "jitterDep", "jitterLen",
               "vibratoFreq", "vibratoDep", "shimmerDep", "creakyBreathy",
               "rolloff", "rolloffOct", "rolloffKHz", "rolloffParab", "rolloffParabHarm",
               "rolloffLip", "rolloff_perAmpl", "temperature", "pitchDriftDep",
               "pitchDriftFreq", "randomWalk_trendStrength", "shortestEpoch", "subFreq",
               "subDep", "amDep", "amFreq", "overlap", "samplingRate", "pitchFloor",
               "pitchCeiling", "pitchSamplingRate", "throwaway"]


class sg_harm_params(C.Structure):
    _fields_ = [(f, C.c_double) for f in HARM_FIELDS]


class sg_soundgen_args(C.Structure):
    _fields_ = [
        ("repeatBout", C.c_double), ("nSyl", C.c_double), ("sylLen", C.c_double),
        ("pauseLen", C.c_double),
        ("pitchAnchors", sg_anchors), ("pitchAnchorsGlobal", sg_anchors),
        ("temperature", C.c_double), ("tempEffects", C.c_double * 8),
        ("maleFemale", C.c_double), ("creakyBreathy", C.c_double),
        ("nonlinBalance", C.c_double), ("nonlinDep", C.c_double),
        ("jitterLen", C.c_double), ("jitterDep", C.c_double), ("vibratoFreq", C.c_double),
        ("vibratoDep", C.c_double), ("shimmerDep", C.c_double),
        ("attackLen", C.c_double), ("rolloff", C.c_double), ("rolloffOct", C.c_double),
        ("rolloffKHz", C.c_double), ("rolloffParab", C.c_double),
        ("rolloffParabHarm", C.c_double), ("rolloffLip", C.c_double),
        ("formants", sg_formants),
        ("formantDep", C.c_double), ("formantDepStoch", C.c_double), ("vocalTract", C.c_double),
        ("subFreq", C.c_double), ("subDep", C.c_double), ("shortestEpoch", C.c_double),
        ("amDep", C.c_double), ("amFreq", C.c_double), ("amShape", C.c_double),
        ("noiseAnchors", sg_anchors), ("formantsNoise", sg_formants),
        ("rolloffNoise", C.c_double),
        ("mouthAnchors", sg_anchors), ("amplAnchors", sg_anchors),
        ("amplAnchorsGlobal", sg_anchors),
        ("samplingRate", C.c_double), ("windowLength", C.c_double), ("overlap", C.c_double),
        ("addSilence", C.c_double), ("pitchFloor", C.c_double), ("pitchCeiling", C.c_double),
        ("pitchSamplingRate", C.c_double), ("throwaway", C.c_double),
        ("invalidArgAction", C.c_int32), ("formantsNoise_rlen", C.c_int32),
    ]


class sg_call_desc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("args", C.POINTER(sg_soundgen_args)),
                ("pitch", _dp), ("pitch_len", C.c_int64),
                ("harm", C.POINTER(sg_harm_params)), ("amplAnchors", sg_anchors),
                ("random", sg_random)]


def dptr(a):
    """double* of a C-contiguous float64 numpy array (None -> NULL)."""
    if a is None:
        return _dp()
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_dp)


def iptr(a):
    if a is None:
        return _ip()
    assert a.dtype == np.int32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_ip)
