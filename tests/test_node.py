"""The whole-node batch path (sg_node_*, include/soundgen_hip.h ABI 3): one
process shards a batch over several devices by calls (LPT over the analytic
cost) -- SURVEY.md §8e for the callers the R API keeps (soundgen_batch,
morph(), matchPars()). CPU: planning needs no device (contexts are created at
execution), so the in-library sharding is checked here against whole-batch
planning; the GPU tests (test_gpu_node.py) run it."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from soundgen_beta_amd import batch, dist, native  # noqa: E402
from soundgen_beta_amd.rrng import RRng  # noqa: E402


def _c5(n):
    return bench.CONFIGS["c5"][0](n)


def test_node_plan_equals_whole_batch_plan():
    calls = _c5(96)
    whole = batch.Plan(calls, None)
    for devs in ([0, 0], [0, 1, 2], [3]):
        node = native.Node(devs)
        p = batch.NodePlan(calls, node)
        assert np.array_equal(p.lengths, whole.lengths)
        assert np.array_equal(p.offsets, whole.offsets)
        assert np.array_equal(p.status, whole.status)
        assert p.total == whole.total
        assert set(p.owner.tolist()) <= set(range(len(devs)))
        # each shard holds exactly its calls' 64-sample slots
        for k in range(len(devs)):
            want = int(sum((whole.lengths[i] + 63) // 64 * 64 for i in np.nonzero(p.owner == k)[0]))
            assert p.shard_samples(k) == want
        p.close()
        node.close()


def test_node_assignment_is_lpt_over_the_dist_cost_model():
    """The C++ cost model restates dist.call_cost: the same assignment, and the
    load balance of bench's C5 mix (max / mean predicted load per device)."""
    calls = _c5(512)
    for k in (2, 4, 8):
        node = native.Node(list(range(k)))
        p = batch.NodePlan(calls, node)
        want = dist.lpt_assign([dist.call_cost(c) for c in calls], k)
        assert np.array_equal(p.owner, want), k
        cost = np.array([dist.call_cost(c) for c in calls])
        load = np.array([cost[p.owner == r].sum() for r in range(k)])
        assert load.max() / load.mean() < 1.02, (k, load)
        p.close()
        node.close()


def test_node_callback_stream_matches_serial_planning():
    """Draws from ONE R stream (RRng callbacks, as the R shim binds R's RNG): the
    node records every call's draws in call order, then plans the shards from
    them. Lengths, statuses and the stream position afterwards equal serial
    whole-batch planning on the same seed."""
    args = [dict(sylLen=120 + 30 * i, temperature=0.2, samplingRate=16000, addSilence=0, formants="a",
                 pitchAnchors={"time": [0, 1], "value": [150 + 10 * i, 120]}) for i in range(10)]
    g1, g2 = RRng(11), RRng(11)
    whole = batch.Plan([{"kind": "soundgen", "args": a, "rng": g1} for a in args], None)
    node = native.Node([0, 0, 0])
    p = batch.NodePlan([{"kind": "soundgen", "args": a, "rng": g2} for a in args], node)
    assert np.array_equal(p.lengths, whole.lengths)
    assert np.array_equal(p.status, whole.status) and not p.status.any()
    assert len(set(p.owner.tolist())) == 3
    assert g1.random() == g2.random()
    p.close()
    node.close()


def test_node_callback_stream_stops_at_failing_call():
    a = dict(sylLen=200, temperature=0.2, samplingRate=16000, addSilence=0)
    bad = dict(a, samplingRate=-5, invalidArgAction="abort")
    g1, g2 = RRng(5), RRng(5)
    node = native.Node([0, 0])
    p = batch.NodePlan([{"kind": "soundgen", "args": x, "rng": g1} for x in (a, a, bad, a)], node)
    assert list(p.status[:2]) == [0, 0] and p.status[2] != 0 and p.status[3] != 0
    assert "not planned" in p.message(3)
    batch.Plan([{"kind": "soundgen", "args": x, "rng": g2} for x in (a, a)], None)
    assert g1.random() == g2.random()
    p.close()
    node.close()


def test_node_draws_only_recording_equals_serial_plan_c5():
    """C5 presets (noise, stochastic formants, vocal fry, several bouts) drawing from
    ONE RRng stream: the node's draws-only recording pass (Batch::draws_only, no device
    work planned) plus the parallel replay gives every call the plan serial planning
    gives it -- lengths, statuses, the sine-bank terms and FFT flops each call emits
    (both depend on every draw) -- and leaves the stream where serial planning does."""
    args = [c["args"] for c in _c5(192)]
    g1, g2 = RRng(2026), RRng(2026)
    whole = batch.Plan([{"kind": "soundgen", "args": a, "rng": g1} for a in args], None)
    node = native.Node([0, 0, 0, 0])
    p = batch.NodePlan([{"kind": "soundgen", "args": a, "rng": g2} for a in args], node)
    assert np.array_equal(p.lengths, whole.lengths)
    assert np.array_equal(p.status, whole.status) and not p.diverged
    rows_w, flops_w = whole.call_work()
    rows_n, flops_n = p.call_work()
    # rows are integer counts; a call's flops are a difference of the batch's running
    # fp64 total, so they carry its rounding (the batch around the call differs)
    assert np.array_equal(rows_n, rows_w)
    np.testing.assert_allclose(flops_n, flops_w, rtol=1e-9)
    assert g1.random() == g2.random()
    p.close()
    node.close()


def test_node_chunks_and_bulk_uniform_callback():
    """Shards are planned in chunks of consecutive calls (SG_NODE_CHUNK calls, default
    4096): a small batch is one chunk per shard. The Python draw callbacks (numpy
    Generator) pass runs of uniforms through the bulk callback (ABI 5): the same plan
    as one uniform per callback."""
    calls = _c5(24)
    node = native.Node([0, 0])
    p = batch.NodePlan(calls, node)
    assert [p.chunks(k) for k in range(2)] == [1, 1]
    p.close()
    node.close()
    args = [dict(c["args"]) for c in calls[:6]]
    plans = []
    for bulk in (True, False):
        rng = np.random.default_rng(5)
        pl = batch.Plan([{"kind": "soundgen", "args": a, "rng": rng} for a in args], None)
        plans.append((pl.lengths.copy(), pl.call_work(), rng.random()))
        pl.close()
        if bulk:
            from soundgen_beta_amd import _abi
            orig = _abi.UNIF_N_CB
            _abi.UNIF_N_CB = lambda f: orig()  # a NULL bulk callback: one draw per callback
    _abi.UNIF_N_CB = orig
    (l1, (r1, f1), x1), (l2, (r2, f2), x2) = plans
    assert np.array_equal(l1, l2) and np.array_equal(r1, r2) and np.array_equal(f1, f2) and x1 == x2
