"""Multi-GPU sharding of a batch of calls.

Calls are independent and every normalisation is per call (R/source.R:449,
R/soundgen.R:807), so a batch shards by calls with no data-path collective:
each rank plans and synthesizes its own calls. The only exchange is the
optional gather of the packed outputs to one rank (a consumer that needs the
whole batch in one process): per peer, one int64 length vector and one packed
fp32 buffer, point-to-point to the root (on MI355X every peer has its own xGMI
link to rank 0, so the transfers do not serialise on a ring).

Assignment is LPT (longest processing time first) over an analytic cost per
call, identical on every rank (no communication needed to agree on it).
"""
import os
import math

import numpy as np

# cost model: one unit = one synthesized sample-row of the sine bank; an FFT
# frame of wl points costs ~5 wl log2(wl) flops against ~4 per sample-row
_FFT_UNIT = 5.0 / 4.0


def _anchors_len(a):
    if a is None:
        return 0
    if isinstance(a, dict):
        return len(np.atleast_1d(a.get("value", a.get("time", []))))
    return len(np.atleast_1d(a))


def call_cost(call):
    """Analytic cost of one call (relative units, used only for balancing)."""
    kind = call.get("kind", "soundgen")
    if kind == "harmonics":
        p = call.get("params", {})
        sr = float(p.get("samplingRate", 16000))
        psr = float(p.get("pitchSamplingRate", 3500))
        pitch = np.asarray(call["pitch"], dtype=np.float64)
        n = len(pitch) / psr * sr
        f0 = max(float(np.nanmin(pitch)) if len(pitch) else 100.0, 1.0)
        rows = min(sr / 2 / f0, 64.0)
        return n * max(rows, 1.0)
    a = call.get("args", {})
    sr = float(a.get("samplingRate", 16000))
    dur = float(a.get("sylLen", 300)) * max(1, int(a.get("nSyl", 1))) * max(1, int(a.get("repeatBout", 1)))
    dur += float(a.get("pauseLen", 0)) * max(0, int(a.get("nSyl", 1)) - 1)
    n = dur / 1000.0 * sr
    pa = a.get("pitchAnchors", "default")
    f0 = 150.0
    if pa is None:
        rows = 0.0
    else:
        if isinstance(pa, dict):
            vals = np.atleast_1d(pa.get("value", [150.0]))
        elif isinstance(pa, str):
            vals = [150.0]
        else:
            vals = np.atleast_1d(pa)
        f0 = max(float(np.min(vals)), 1.0)
        rows = min(sr / 2 / f0, 64.0)
    wl = max(4.0, 2 * round(float(a.get("windowLength", 50)) * sr / 1000 / 2))
    hop = wl * (1 - float(a.get("overlap", 75)) / 100)
    frames = n / max(hop, 1.0)
    noise = 1.0 + (_anchors_len(a.get("noiseAnchors")) > 0)
    return n * max(rows, 1.0) + _FFT_UNIT * frames * noise * 2 * wl * math.log2(wl)


def lpt_assign(costs, world):
    """Rank of each call: largest cost first onto the least-loaded rank
    (ties: lowest rank, then original order) -- deterministic everywhere."""
    costs = np.asarray(costs, dtype=np.float64)
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    load = np.zeros(world)
    rank = np.zeros(len(costs), dtype=np.int64)
    for i in order:
        r = int(np.argmin(load))
        rank[i] = r
        load[r] += costs[i]
    return rank


def shard(calls, rank, world):
    """Indices (ascending) and calls this rank synthesizes."""
    owner = lpt_assign([call_cost(c) for c in calls], world)
    idx = np.nonzero(owner == rank)[0]
    return idx, [calls[i] for i in idx], owner


def gather_to_root(outputs, owner, rank, world, device="cpu", root=0):
    """Send this rank's outputs (list of 1-D arrays or exceptions, in shard
    order) to `root`; the root returns the whole batch in call order, the
    others None. Uses torch.distributed point-to-point (gloo or RCCL)."""
    import torch
    import torch.distributed as dist

    def pack(outs):
        lens = np.array([len(o) if not isinstance(o, Exception) else -1 for o in outs], dtype=np.int64)
        parts = [np.asarray(o, np.float32) for o in outs if not isinstance(o, Exception)]
        data = np.concatenate(parts) if parts else np.zeros(0, np.float32)
        return lens, data

    if rank != root:
        lens, data = pack(outputs)
        dist.send(torch.from_numpy(lens).to(device), dst=root)
        if data.size:
            dist.send(torch.from_numpy(data).to(device), dst=root)
        return None
    result = [None] * len(owner)
    for r in range(world):
        idx = np.nonzero(owner == r)[0]
        if r == root:
            outs = list(outputs)
        else:
            lt = torch.empty(len(idx), dtype=torch.int64, device=device)
            dist.recv(lt, src=r)
            lens = lt.cpu().numpy()
            total = int(lens[lens > 0].sum())
            buf = np.zeros(0, np.float32)
            if total:
                bt = torch.empty(total, dtype=torch.float32, device=device)
                dist.recv(bt, src=r)
                buf = bt.cpu().numpy()
            outs, o = [], 0
            for n in lens:
                if n < 0:
                    outs.append(RuntimeError("call failed on rank %d" % r))
                else:
                    outs.append(buf[o:o + n])
                    o += int(n)
        for i, y in zip(idx, outs):
            result[i] = y
    return result


def synthesize_sharded(calls, rank, world, device=None, synth=None, root=0, comm_device=None):
    """Every rank synthesizes its LPT shard (on its GPU) and the root gathers
    the batch in call order. `synth` (default batch.synthesize) maps a list of
    calls to a list of outputs; `device` defaults to the rank's LOCAL_RANK GPU;
    `comm_device` is where the exchange tensors live ("cpu" for gloo,
    "cuda:<local>" for RCCL)."""
    if device is None:
        device = int(os.environ.get("LOCAL_RANK", "0"))
    if synth is None:
        from . import batch

        def synth(cs):
            return batch.synthesize(cs, device)
    idx, mine, owner = shard(calls, rank, world)
    outs = synth(mine) if mine else []
    if world == 1:
        return outs
    return gather_to_root(outs, owner, rank, world, comm_device or "cpu", root)
