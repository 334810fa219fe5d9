"""Sharded batch path (soundgen_beta_amd/dist.py) on CPU, torch.distributed gloo
at world size 2: LPT assignment, the packed exchange step (all_gather of the
packed lengths, then one point-to-point send per peer of its packed buffer and
(offset, length) table), and every rank running the REAL host planner on its
shard. The per-rank synthesizer is the oracle here (test infrastructure); on
the GPU box it is batch.synthesize_packed and the packed HBM buffer goes over
RCCL."""
import os
import socket

import numpy as np
import pytest

from soundgen_beta_amd import dist as sgd


def _calls():
    calls = []
    for f0 in (90.0, 130.0, 170.0, 210.0, 260.0):
        calls.append({"kind": "harmonics", "pitch": np.full(700, f0),
                      "params": dict(samplingRate=16000, rolloff=-12, attackLen=20)})
    calls.append({"kind": "soundgen", "args": dict(sylLen=200, samplingRate=16000, temperature=0, addSilence=0,
                                                   pitchAnchors=[120, 180])})
    calls.append({"kind": "soundgen", "args": dict(sylLen=150, samplingRate=16000, temperature=0, addSilence=0,
                                                   pitchAnchors=None,
                                                   noiseAnchors={"time": [0, 150], "value": [-20, -20]}),
                  "uniforms": np.random.default_rng(5).uniform(size=400 * 40)})
    calls.append({"kind": "harmonics", "pitch": np.full(1, 150.0), "params": dict(samplingRate=16000)})  # refused
    return calls


def _oracle_synth(calls):
    from oracle import oracle as O
    out = []
    for c in calls:
        try:
            if c["kind"] == "harmonics":
                out.append(O.generate_harmonics(c["pitch"], **c["params"]))
            else:
                out.append(O.soundgen(uniforms=c.get("uniforms"), **c["args"]))
        except Exception as e:  # noqa: BLE001 -- a refused call travels as a failed slot
            out.append(e)
    return out


def _bench():
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    return bench


def test_lpt_assignment_balanced_and_deterministic():
    costs = [10, 9, 8, 7, 6, 5, 4, 3, 2, 1]
    a = sgd.lpt_assign(costs, 3)
    assert list(a) == list(sgd.lpt_assign(costs, 3))
    loads = [sum(c for c, r in zip(costs, a) if r == k) for k in range(3)]
    assert max(loads) - min(loads) <= max(costs)
    assert set(a) == {0, 1, 2}
    assert sgd.call_cost(_calls()[0]) > 0 and sgd.call_cost(_calls()[-2]) > 0


def test_cost_na_pitch():
    """R's NA (NaN, None, "NA", all-NA anchors or pitch) means no voiced part:
    the call costs its per-sample work only, and never raises (shard() runs it on
    every rank)."""
    base = dict(sylLen=300, samplingRate=16000, temperature=0, addSilence=0)
    voiced = sgd.call_cost({"kind": "soundgen", "args": dict(base, pitchAnchors=[120, 180])})
    unvoiced = sgd.call_cost({"kind": "soundgen", "args": dict(base, pitchAnchors=None)})
    assert voiced > unvoiced > 0
    for pa in (float("nan"), "NA", [float("nan"), float("nan")], {"time": [0, 1], "value": [float("nan")] * 2},
               {"time": [0, 1], "value": [None, None]}):
        assert sgd.call_cost({"kind": "soundgen", "args": dict(base, pitchAnchors=pa)}) == unvoiced, pa
    # NA values among finite ones are dropped, not propagated
    part = sgd.call_cost({"kind": "soundgen", "args": dict(base, pitchAnchors=[120, float("nan"), 180])})
    assert np.isfinite(part) and part > unvoiced
    h = {"kind": "harmonics", "params": dict(samplingRate=16000)}
    assert sgd.call_cost(dict(h, pitch=np.full(700, np.nan))) > 0
    assert sgd.call_cost(dict(h, pitch=np.full(700, np.nan))) < sgd.call_cost(dict(h, pitch=np.full(700, 150.0)))
    mixed = np.full(700, 150.0)
    mixed[:300] = np.nan
    assert np.isfinite(sgd.call_cost(dict(h, pitch=mixed)))
    sgd.shard([dict(h, pitch=np.full(700, np.nan)), {"kind": "soundgen", "args": dict(base, pitchAnchors="NA")}], 0, 2)


def test_cost_rows_follow_get_rolloff(oracle):
    """harmonic_rows() counts the rows getRolloff keeps (the oracle's, no cap)."""
    for f0, kw in ((100.0, dict(rolloff=-12, rolloffOct=-12, rolloffKHz=-6)),
                   (71.0, dict(rolloff=-24, rolloffOct=0, rolloffKHz=-10)),
                   (400.0, dict(rolloff=-6, rolloffOct=-2, rolloffKHz=-6))):
        nH = int(np.ceil((44100 / 2 - f0) / f0))
        A = oracle.get_rolloff([f0], nHarmonics=nH, samplingRate=44100, rolloffParab=0, **kw)
        assert sgd.harmonic_rows(f0, 44100, **kw) == A.shape[0], (f0, kw)


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = sgd.synthesize_sharded(_calls(), rank, world, synth=_oracle_synth, comm_device="cpu")
        # a peer whose shard packs to 0 samples (its only call is refused) sends no
        # buffer; the root still returns every call, as host arrays with to_host
        two = [_calls()[0], _calls()[-1]]
        res0 = sgd.synthesize_sharded(two, rank, world, synth=_oracle_synth, comm_device="cpu", to_host=True)
        # bench.py's default exchange at N > 1 (dist.gather_timed): the shard's outputs in
        # several plan regions of one packed buffer (plan k at base b_k, its calls at
        # b_k + offsets), gathered to rank 0 in call order
        calls = _calls()
        idx, mine, _ = sgd.shard(calls, rank, world)
        outs = _oracle_synth(mine)
        half = len(outs) // 2
        parts = [sgd.pack_outputs(outs[:half]), sgd.pack_outputs(outs[half:])]
        base = [0, int(parts[0][0].numel()) + 64]
        import torch
        data = torch.zeros(base[1] + int(parts[1][0].numel()), dtype=torch.float32)
        offs, lens = [], []
        for (d, o, n), b in zip(parts, base):
            data[b:b + d.numel()] = d
            offs.append(b + o)
            lens.append(n)
        gt, ms = sgd.gather_timed(data, np.concatenate(offs), np.concatenate(lens), calls, rank, world)
        assert ms >= 0
        if rank == 0:
            assert len(gt) == len(calls)
            for g, r in zip(gt, res):
                assert isinstance(g, Exception) == isinstance(r, Exception)
                if not isinstance(g, Exception):
                    assert np.array_equal(g.numpy(), np.asarray(r))
        else:
            assert gt is None
        # the real host planner on this rank's shard of 96 C5 calls (CPU planning)
        from soundgen_beta_amd import batch
        calls = _bench().c5_calls(96)
        idx, mine, owner = sgd.shard(calls, rank, world)
        p = batch.Plan(mine, None)
        mine_plan = (idx.tolist(), p.lengths.tolist(), p.offsets.tolist(), p.status.tolist(), int(p.total))
        plans = [None] * world
        dist.all_gather_object(plans, mine_plan)
        if rank == 0:
            assert sgd.lpt_assign([sgd.call_cost(c) for c in two], world).tolist() == [0, 1]
            assert isinstance(res0[0], np.ndarray) and res0[0].dtype == np.float32 and len(res0[0]) > 0
            assert isinstance(res0[1], Exception)
            q.put(([np.asarray(y, np.float64) if not isinstance(y, Exception) else None for y in res], plans))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
def test_gloo_world2_gather_and_sharded_planning():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, plans = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    # the gathered batch equals the single-process one, the refused call stays refused
    want = _oracle_synth(_calls())
    assert len(got) == len(want)
    owner = sgd.lpt_assign([sgd.call_cost(c) for c in _calls()], 2)
    assert set(owner) == {0, 1}  # both ranks did work
    for g, w in zip(got, want):
        if isinstance(w, Exception):
            assert g is None
            continue
        assert len(g) == len(w)
        np.testing.assert_allclose(g, np.asarray(w, np.float32), rtol=0, atol=1e-6)
    # per-rank planning: the union of the shards is the whole-batch plan (lengths, status),
    # each shard's offsets are its own 256-B aligned packing
    from soundgen_beta_amd import batch
    whole = batch.Plan(_bench().c5_calls(96), None)
    seen = np.zeros(whole.n, dtype=bool)
    for idx, lens, offs, status, total in plans:
        idx = np.asarray(idx)
        assert not seen[idx].any()
        seen[idx] = True
        assert np.array_equal(np.asarray(lens), whole.lengths[idx])
        assert np.array_equal(np.asarray(status), whole.status[idx])
        slot = (np.asarray(lens) + 63) // 64 * 64
        assert np.array_equal(np.asarray(offs), np.concatenate([[0], np.cumsum(slot)[:-1]]))
        assert total == int(slot.sum())
    assert seen.all()
