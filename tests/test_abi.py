"""The C-ABI library loads and exports every symbol include/soundgen_hip.h
declares (no compute calls: runs on CPU)."""
import ctypes

from soundgen_beta_amd import native


def test_library_loads():
    L = native.lib()
    assert L.sg_abi_version() == 5


def test_exports_every_declared_symbol():
    L = native.lib()
    names = native.declared_symbols()
    assert len(names) > 15
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_no_context_without_gpu_or_ok():
    # sg_ctx_create either succeeds (GPU box) or fails cleanly (CPU box)
    p = ctypes.c_void_p()
    rc = native.lib().sg_ctx_create(0, ctypes.byref(p))
    if rc == 0:
        native.lib().sg_ctx_destroy(p)
    else:
        assert rc == -5
