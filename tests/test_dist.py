"""Sharded batch path (soundgen_beta_amd/dist.py) on CPU: LPT assignment and
the gather to rank 0 over torch.distributed gloo, world size 2. The per-rank
synthesizer is the oracle here (test infrastructure); on the GPU box it is
batch.synthesize, exchanged over RCCL."""
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
    return calls


def _oracle_synth(calls):
    from oracle import oracle as O
    out = []
    for c in calls:
        if c["kind"] == "harmonics":
            out.append(O.generate_harmonics(c["pitch"], **c["params"]))
        else:
            out.append(O.soundgen(uniforms=c.get("uniforms"), **c["args"]))
    return out


def test_lpt_assignment_balanced_and_deterministic():
    costs = [10, 9, 8, 7, 6, 5, 4, 3, 2, 1]
    a = sgd.lpt_assign(costs, 3)
    assert list(a) == list(sgd.lpt_assign(costs, 3))
    loads = [sum(c for c, r in zip(costs, a) if r == k) for k in range(3)]
    assert max(loads) - min(loads) <= max(costs)
    assert set(a) == {0, 1, 2}
    assert sgd.call_cost(_calls()[0]) > 0 and sgd.call_cost(_calls()[-1]) > 0


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = sgd.synthesize_sharded(_calls(), rank, world, synth=_oracle_synth, comm_device="cpu")
        if rank == 0:
            q.put([np.asarray(y, np.float64) for y in res])
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
def test_gloo_world2_gather_matches_single_process():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    want = _oracle_synth(_calls())
    assert len(got) == len(want)
    owner = sgd.lpt_assign([sgd.call_cost(c) for c in _calls()], 2)
    assert set(owner) == {0, 1}  # both ranks did work
    for g, w in zip(got, want):
        assert len(g) == len(w)
        np.testing.assert_allclose(g, np.asarray(w, np.float32), rtol=0, atol=1e-6)
