"""Run by tests/test_sanitizers.py inside the sanitized process only: the
libraries under test are the ASan/UBSan builds and the runtime is live."""
import ctypes as C
import os

import pytest


def test_sanitized_libraries_are_loaded():
    if not os.environ.get("SG_HIP_LIB", "").endswith("_san.so"):
        pytest.skip("not under tests/sanitize/run.sh")
    from soundgen_beta_amd import native
    from oracle import oracle as O
    L = native.lib()
    assert native.LIB_PATH.endswith("libsoundgen_hip_san.so") and O._LIB_PATH.endswith("libsg_oracle_san.so")
    O.lib()
    maps = open("/proc/self/maps").read()
    assert "libsoundgen_hip_san.so" in maps and "libsg_oracle_san.so" in maps and "libasan" in maps
    assert hasattr(C.CDLL(None), "__asan_report_load8")  # the ASan runtime is in the process
    assert L.sg_abi_version() == 5
