"""The whole-node path on the GPU (sg_node_*): a 2-way node mapped onto device
0 (two contexts, two streams, two shards) gives byte-equal samples to the
single-device plan of the whole batch, for injected draws and for one R stream
of draws (RRng callbacks, as the R shim binds R's RNG). N > 1 physical devices
are not reachable on the 1-GPU test box."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

pytestmark = pytest.mark.gpu


def _single(calls):
    import torch
    from soundgen_beta_amd import batch, native
    p = batch.Plan(calls, native.default_context(0))
    p.upload()
    out = torch.full((max(p.total, 1),), float("nan"), dtype=torch.float32, device="cuda")
    p.execute(out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return p, out.cpu().numpy()


def test_node_two_way_on_one_device_equals_single_plan():
    from soundgen_beta_amd import batch, native
    calls = bench.CONFIGS["c5"][0](64)
    p1, y1 = _single(calls)
    node = native.Node([0, 0])
    p2 = batch.NodePlan(calls, node)
    assert np.array_equal(p2.lengths, p1.lengths) and np.array_equal(p2.offsets, p1.offsets)
    assert len(set(p2.owner.tolist())) == 2
    y2 = p2.execute_to_host(np.float32)
    for o, n, st in zip(p1.offsets, p1.lengths, p1.status):
        if st == 0:
            assert np.array_equal(y1[o:o + n], y2[o:o + n]), o
    # the double entry point (the R shim's) carries the same values
    y3 = p2.execute_to_host()
    assert np.array_equal(y3, y2.astype(np.float64))
    p2.close()
    node.close()


def test_node_r_stream_equals_single_plan():
    from soundgen_beta_amd import batch, native
    from soundgen_beta_amd.rrng import RRng
    args = [dict(sylLen=150 + 40 * i, temperature=0.15, samplingRate=22050, addSilence=0, formants="i",
                 noiseAnchors={"time": [0, 150], "value": [-30, -20]},
                 pitchAnchors={"time": [0, 1], "value": [140 + 15 * i, 110]}) for i in range(8)]
    g1 = RRng(21)  # one stream for the whole batch, as R's
    p1, y1 = _single([{"kind": "soundgen", "args": a, "rng": g1} for a in args])
    node = native.Node([0, 0])
    g = RRng(21)
    p2 = batch.NodePlan([{"kind": "soundgen", "args": a, "rng": g} for a in args], node)
    y2 = p2.execute_to_host(np.float32)
    assert np.array_equal(p2.lengths, p1.lengths)
    for o, n in zip(p1.offsets, p1.lengths):
        assert np.array_equal(y1[o:o + n], y2[o:o + n]), o
    p2.close()
    node.close()


def test_synthesize_node_default_devices(oracle):
    """batch.synthesize_node over every visible device (the R shim's default)
    against the oracle."""
    from test_spectral_cpu import N, U
    from soundgen_beta_amd import batch
    cases = [dict(sylLen=300, samplingRate=16000, temperature=0, addSilence=0, formants="a",
                  pitchAnchors={"time": [0, 1], "value": [180, 120]}),
             dict(sylLen=200, samplingRate=16000, temperature=0, addSilence=0, formants="o", nSyl=2, pauseLen=50)]
    ys = batch.synthesize_node([{"kind": "soundgen", "args": a, "normals": N, "uniforms": U} for a in cases])
    for a, y in zip(cases, ys):
        ref = oracle.soundgen(normals=N, uniforms=U, **a)
        assert len(y) == len(ref)
        assert float(np.sqrt(np.mean((y - ref) ** 2))) <= 1e-5
