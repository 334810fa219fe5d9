"""Loader of the in-tree HIP library soundgen_beta_amd/lib/libsoundgen_hip.so.

There is no CPU fallback: if the library is missing or the GPU is not
usable, calls raise. (The planner entry points work without a GPU so host
bookkeeping can be tested on CPU; every synthesis call needs the device.)
"""
import ctypes as C
import os
import re

from . import _abi

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SG_HIP_LIB") or os.path.join(_HERE, "lib", "libsoundgen_hip.so")  # override: experiments
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "soundgen_hip.h")

_lib = None
# the planner's default threshold on its fp32 conditioning estimate of a formant
# filter (sg_set_fp64_policy; DESIGN.md §5 "fp64 path")
HP_RHO_DEFAULT = 100.0


class SoundgenError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s: %s" % (_abi.SG_ERR_NAMES.get(code, code), msg))
        self.code = code


def declared_symbols():
    """Function names declared in include/soundgen_hip.h."""
    txt = open(HEADER_PATH).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(sg_[a-z_0-9]+)\s*\(", txt)))


def lib():
    global _lib
    if _lib is not None:
        return _lib
    # Share torch's HIP runtime when torch is present: torch/lib/libamdhip64.so
    # has the same SONAME as /opt/rocm's, so importing torch first makes our
    # NEEDED entry resolve to that copy (one runtime, valid device pointers).
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError("libsoundgen_hip.so not built (run __graft_entry__.build()): %s" % LIB_PATH)
    L = C.CDLL(LIB_PATH)
    vp = C.c_void_p
    dp = C.POINTER(C.c_double)
    i64 = C.c_int64
    i64p = C.POINTER(C.c_int64)
    L.sg_ctx_create.argtypes = [C.c_int, C.POINTER(vp)]
    L.sg_ctx_destroy.argtypes = [vp]
    L.sg_last_error.argtypes = [vp]
    L.sg_last_error.restype = C.c_char_p
    L.sg_plan_batch.argtypes = [vp, C.POINTER(_abi.sg_call_desc), i64, C.POINTER(vp)]
    L.sg_plan_destroy.argtypes = [vp]
    L.sg_plan_n_calls.argtypes = [vp]
    L.sg_plan_n_calls.restype = i64
    L.sg_plan_total_samples.argtypes = [vp]
    L.sg_plan_total_samples.restype = i64
    L.sg_plan_lengths.argtypes = [vp, i64p, i64p]
    L.sg_plan_status.argtypes = [vp, C.POINTER(C.c_int32)]
    L.sg_plan_call_message.argtypes = [vp, i64]
    L.sg_plan_call_message.restype = C.c_char_p
    L.sg_plan_device_bytes.argtypes = [vp]
    L.sg_plan_device_bytes.restype = i64
    L.sg_plan_upload.argtypes = [vp, vp]
    L.sg_plan_release_host.argtypes = [vp]
    L.sg_execute.argtypes = [vp, vp, vp, vp]
    L.sg_execute_plans.argtypes = [vp, C.POINTER(vp), C.POINTER(vp), C.c_int, vp]
    L.sg_set_profiling.argtypes = [vp, C.c_int]
    L.sg_profile_read.argtypes = [vp, dp, i64p]
    L.sg_profile_read_kernel.argtypes = [vp, C.c_int, dp, i64p]
    L.sg_plan_stft_stats.argtypes = [vp, i64p, i64p, dp]
    L.sg_plan_conditioning.argtypes = [vp, dp]
    L.sg_plan_noise_conditioning.argtypes = [vp, dp]
    L.sg_plan_precision.argtypes = [vp, C.POINTER(C.c_int32), i64p, i64p]
    L.sg_set_fp64_policy.argtypes = [C.c_int32, C.c_double]
    L.sg_set_amp_policy.argtypes = [C.c_int32]
    L.sg_set_uniform_gather.argtypes = [C.c_int32]
    if hasattr(L, "sg_plan_sine_tasks"):  # ABI 4 (an older library still loads for A/B runs)
        L.sg_plan_sine_tasks.argtypes = [vp, i64p]
    L.sg_set_sine_table.argtypes = [C.c_int32]
    L.sg_plan_table_stats.argtypes = [C.c_void_p, C.POINTER(i64), C.POINTER(i64), C.POINTER(i64)]
    L.sg_host_cache_trim.argtypes = []
    L.sg_host_cache_trim.restype = i64
    L.sg_get_smooth_contour.argtypes = [_abi.sg_anchors, C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_double,
                                        C.c_int32, C.c_double, C.c_double, C.POINTER(C.c_double),
                                        C.POINTER(C.c_int64)]
    L.sg_plan_amp_count.restype = C.c_int64
    L.sg_plan_amp_count.argtypes = [C.c_void_p]
    L.sg_plan_debug_amps.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.c_int64]
    L.sg_plan_call_work.argtypes = [vp, dp, dp]
    L.sg_dtw_symmetric2.argtypes = [dp, i64, dp, i64, dp]
    L.sg_mel_spec.argtypes = [vp, dp, i64, C.POINTER(_abi.sg_mel_params), dp, i64, C.POINTER(C.c_int32),
                              C.POINTER(C.c_int32)]
    L.sg_compare_sounds_batch.argtypes = [vp, dp, C.c_int32, C.c_int32, vp, i64p, i64p, i64,
                                          C.POINTER(_abi.sg_mel_params), C.c_int32, dp, dp]
    L.sg_rrng_create.argtypes = [C.c_int32, C.POINTER(vp)]
    L.sg_rrng_destroy.argtypes = [vp]
    L.sg_rrng_set_seed.argtypes = [vp, C.c_int32]
    for f in ("unif", "norm", "exp"):
        getattr(L, "sg_rrng_" + f).argtypes = [vp]
        getattr(L, "sg_rrng_" + f).restype = C.c_double
    L.sg_rrng_gamma.argtypes = [vp, C.c_double, C.c_double]
    L.sg_rrng_gamma.restype = C.c_double
    L.sg_random_bind_rrng.argtypes = [C.POINTER(_abi.sg_random), vp]
    L.sg_plan_kernel_stats.argtypes = [vp, i64p, i64p, i64p, i64p]
    L.sg_synchronize.argtypes = [vp]
    L.sg_execute_to_host.argtypes = [vp, vp, dp]
    L.sg_generate_harmonics.argtypes = [vp, dp, i64, C.POINTER(_abi.sg_harm_params), _abi.sg_anchors,
                                        C.POINTER(_abi.sg_random), dp, i64, i64p]
    L.sg_soundgen.argtypes = [vp, C.POINTER(_abi.sg_soundgen_args), C.POINTER(_abi.sg_random), dp, i64, i64p]
    L.sg_formant_filter.argtypes = [vp, dp, i64, dp, C.c_int32, C.c_int32, C.c_double, dp, i64, i64p]
    L.sg_generate_noise.argtypes = [vp, i64, _abi.sg_anchors, C.c_double, C.c_double, C.c_int32, C.c_double,
                                    C.c_double, C.c_double, dp, C.c_int32, C.POINTER(_abi.sg_random), dp]
    L.sg_spectral_envelope.argtypes = [vp, C.c_int32, C.c_int32, C.POINTER(_abi.sg_formants), C.c_double,
                                       C.c_double, _abi.sg_anchors, C.c_double, C.c_double, C.c_double,
                                       C.c_double, C.c_double, C.c_double, C.c_double, C.c_double, C.c_double,
                                       C.c_double, C.POINTER(_abi.sg_random), dp]
    L.sg_get_rolloff.argtypes = [dp, C.c_int32, C.c_int32] + [C.c_double] * 9 + [dp, C.POINTER(C.c_int32)]
    fp = C.POINTER(C.c_float)
    L.sg_debug_wave_fft.argtypes = [vp, C.c_int32, C.c_int32, C.c_int32, fp, fp]
    i16p = C.POINTER(C.c_int16)
    L.sg_pcm16.argtypes = [vp, vp, vp, vp, vp]
    L.sg_savewav_pcm.argtypes = [vp, dp, i64, dp, i16p]
    L.sg_wav_write.argtypes = [C.c_char_p, i16p, i64, C.c_int32]
    L.sg_permitted_value.argtypes = [C.c_int32, C.POINTER(C.c_char_p), dp]
    L.sg_noise_threshold.argtypes = [C.c_int32, C.c_double]
    L.sg_noise_threshold.restype = C.c_double
    L.sg_abi_version.restype = C.c_int
    # whole-node batch path (sg_node.cpp; ABI 3, chunks and divergence ABI 5). Guarded
    # like sg_plan_sine_tasks: an older library still loads for A/B runs
    if not hasattr(L, "sg_node_create"):
        _lib = L
        return L
    L.sg_device_count.restype = C.c_int
    L.sg_node_create.argtypes = [C.POINTER(C.c_int32), C.c_int32, C.POINTER(vp)]
    L.sg_node_destroy.argtypes = [vp]
    L.sg_node_size.argtypes = [vp]
    L.sg_node_size.restype = C.c_int32
    L.sg_node_last_error.argtypes = [vp]
    L.sg_node_last_error.restype = C.c_char_p
    L.sg_node_plan_batch.argtypes = [vp, vp, i64, C.POINTER(vp)]
    L.sg_node_plan_destroy.argtypes = [vp]
    L.sg_node_plan_n_calls.argtypes = [vp]
    L.sg_node_plan_n_calls.restype = i64
    L.sg_node_plan_total_samples.argtypes = [vp]
    L.sg_node_plan_total_samples.restype = i64
    L.sg_node_plan_lengths.argtypes = [vp, i64p, i64p]
    L.sg_node_plan_status.argtypes = [vp, C.POINTER(C.c_int32)]
    L.sg_node_plan_call_message.argtypes = [vp, i64]
    L.sg_node_plan_call_message.restype = C.c_char_p
    L.sg_node_plan_owner.argtypes = [vp, C.POINTER(C.c_int32)]
    L.sg_node_plan_costs.argtypes = [vp, dp]
    L.sg_node_plan_shard_samples.argtypes = [vp, C.c_int32]
    L.sg_node_plan_shard_samples.restype = i64
    L.sg_node_execute_to_host.argtypes = [vp, vp, dp]
    L.sg_node_execute_to_host_f32.argtypes = [vp, vp, C.POINTER(C.c_float)]
    if hasattr(L, "sg_node_plan_chunks"):
        L.sg_node_plan_chunks.argtypes = [vp, C.c_int32]
        L.sg_node_plan_chunks.restype = C.c_int32
        L.sg_node_plan_diverged.argtypes = [vp]
        L.sg_node_plan_diverged.restype = C.c_int32
        L.sg_node_plan_call_work.argtypes = [vp, dp, dp]
    if hasattr(L, "sg_rrng_unif_n"):
        L.sg_rrng_unif_n.argtypes = [vp, dp, i64]
    _lib = L
    return L


def check(rc, ctx=None):
    if rc < 0:
        msg = lib().sg_last_error(ctx).decode() if ctx is not None else ""
        raise SoundgenError(rc, msg)
    return rc


class Context:
    """A device context (one HIP stream on one GPU)."""

    def __init__(self, device=0):
        self.device = device
        self.ptr = C.c_void_p()
        rc = lib().sg_ctx_create(device, C.byref(self.ptr))
        if rc < 0:
            raise SoundgenError(rc, "sg_ctx_create(%d) failed (no usable GPU?)" % device)

    def close(self):
        if self.ptr:
            lib().sg_ctx_destroy(self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Node:
    """Several devices driven from this process (sg_node_*): a batch is sharded
    over them by calls (LPT), each device synthesizes its shard and copies it over
    its own link. devices: ordinals (repeats allowed: a 2-way node on one GPU), or
    None for every visible device. Planning works without a GPU."""

    def __init__(self, devices=None):
        L = lib()
        self.ptr = C.c_void_p()
        if devices is None:
            rc = L.sg_node_create(None, 0, C.byref(self.ptr))
        else:
            d = (C.c_int32 * len(devices))(*devices)
            rc = L.sg_node_create(d, len(devices), C.byref(self.ptr))
        if rc < 0:
            raise SoundgenError(rc, "sg_node_create failed (no usable GPU?)")
        self.size = int(L.sg_node_size(self.ptr))

    def check(self, rc):
        if rc < 0:
            raise SoundgenError(rc, lib().sg_node_last_error(self.ptr).decode())
        return rc

    def close(self):
        if self.ptr:
            lib().sg_node_destroy(self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_ctx = {}


def default_context(device=0):
    if device not in _default_ctx:
        _default_ctx[device] = Context(device)
    return _default_ctx[device]
