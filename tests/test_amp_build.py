"""Harmonic amplitude matrices built on the device (sg_amp_build)
against the host-built restatement of getRolloff / shimmer / getVocalFry_per_epoch
(R/sourceSpectrum.R:71-186, R/source.R:316-323, R/subharmonics.R:25-86).

CPU: the planner's host evaluation of the device formula (sg_plan_debug_amps,
the kernel's code compiled for the host) equals the host-built blocks bit for
bit, and the plans' lengths and offsets are unchanged. GPU: a batch synthesized
with device-built amplitudes matches the host-built one (the two differ only by
the platforms' pow / exp)."""
import ctypes as C

import numpy as np
import pytest

import bench
from soundgen_beta_amd import batch, native


def _plan_amps(calls, host_built):
    L = native.lib()
    assert L.sg_set_amp_policy(host_built) == 0
    try:
        p = batch.Plan(calls, None)
        n = L.sg_plan_amp_count(p.ptr)
        a = np.zeros(n, np.float32)
        assert L.sg_plan_debug_amps(p.ptr, a.ctypes.data_as(C.POINTER(C.c_float)), n) == 0
        return p, a
    finally:
        L.sg_set_amp_policy(0)


@pytest.mark.parametrize("config,n", [("c2", 64), ("c3", 64), ("c4", 64), ("c5", 512)])
def test_device_formula_equals_host_built(config, n):
    calls = bench.CONFIGS[config][0](n)
    ph, ah = _plan_amps(calls, 1)
    pd, ad = _plan_amps(calls, 0)
    assert np.array_equal(ph.lengths, pd.lengths) and np.array_equal(ph.offsets, pd.offsets)
    assert np.array_equal(ph.status, pd.status)
    assert ah.size == ad.size and ah.size > 0
    assert np.array_equal(ah, ad)


@pytest.mark.gpu
def test_device_built_amplitudes_synthesize_like_host_built():
    calls = bench.c5_calls(256)
    L = native.lib()
    outs = []
    for host_built in (1, 0):
        assert L.sg_set_amp_policy(host_built) == 0
        try:
            outs.append(batch.synthesize(calls))
        finally:
            L.sg_set_amp_policy(0)
    worst = 0.0
    for a, b in zip(*outs):
        assert len(a) == len(b)
        if len(a):
            worst = max(worst, float(np.sqrt(np.mean((a.astype(np.float64) - b) ** 2))))
    assert worst <= 1e-7, worst
