"""Multi-GPU sharding of a batch of calls.

Calls are independent and every normalisation is per call (R/source.R:449,
R/soundgen.R:807), so a batch shards by calls with no data-path collective:
each rank plans and synthesizes its own calls into one packed fp32 buffer in
its HBM (call i of the shard at offset[i], 256-B aligned slots). The single
exchange step is the gather of those packed buffers to the root (a consumer
that needs the whole batch in one process):
  1. all_gather of every rank's packed length (int64), then
  2. one send per peer of its packed DEVICE buffer plus its (offset, length)
     table, received by the root into one device buffer per peer, all peers in
     one batch_isend_irecv group. On MI355X every peer has its own xGMI link to
     rank 0, so the transfers run concurrently and do not serialise on a ring.

Assignment is LPT (longest processing time first) over an analytic cost per
call, identical on every rank (no communication to agree on it). The cost is
the work the planner will emit, estimated from the arguments alone:
  sine bank:  samples x harmonic rows above `throwaway` (getRolloff's slope,
              R/sourceSpectrum.R:71-186), x (nSub + 1) with subharmonics
              (R/subharmonics.R:25-86: sideband rows between harmonics)
  STFT/OLA:   filter + noise frames x 5 wl log2 wl (sg_stft_ola)
  per sample: assembly and mixes (finalize, sg_mix)
with weights measured on the C5 workload (kernel time per unit
from the rocprofv3 kernel stats). Host planning (~4.6 ns per sample on 16
threads) is also about proportional to samples, so the same assignment
balances it.
tools/dist_balance.py checks the assignment against the planner's actual
per-call work (sg_plan_call_work).
"""
import math
import os

import numpy as np

# weights: ns of one MI355X per unit (calibrated by tools/dist_balance.py)
W_ROW = 0.0035     # per (sample, row) of the sine bank
W_FLOP = 0.00004   # per nominal FFT flop of sg_stft_ola
W_SAMPLE = 0.05    # per output sample: finalize, mixes


def _is_na(v):
    return v is None or (isinstance(v, str) and v.upper() == "NA")


def _finite(v):
    """Finite values of an anchor list or pitch vector; NaN / None / "NA" are
    R's NA (unvoiced), the planner treats them as absent."""
    if _is_na(v):
        return np.zeros(0)
    v = np.atleast_1d(np.asarray([np.nan if _is_na(x) else x for x in np.atleast_1d(v).tolist()],
                                 dtype=np.float64))
    return v[np.isfinite(v)]


def _anchor_values(pa, default):
    """Pitch anchor values of a call, or None when it has no voiced part
    (pitchAnchors NULL / NA / all NA: R/soundgen.R:465 builds a pitch contour only
    from a list)."""
    if _is_na(pa):
        return None
    if isinstance(pa, dict):
        v = _finite(pa.get("value", default))
    elif isinstance(pa, str):
        v = _finite(default)
    else:
        v = _finite(pa)
    return v if len(v) else None


def harmonic_rows(f0, sr, rolloff=-12.0, rolloffOct=-12.0, rolloffKHz=-6.0, throwaway=-120.0):
    """Rows getRolloff keeps at pitch f0: harmonics below Nyquist whose dB level
    (rolloff + rolloffKHz (f0 - 200) / 1000) log2 h + rolloffOct (f0 h - 200) / 1000
    (h >= 2, R/sourceSpectrum.R:86-101) stays above throwaway."""
    f0 = max(float(f0), 1.0)
    nH = int(math.ceil((sr / 2 - f0) / f0))
    slope = rolloff + rolloffKHz * (f0 - 200) / 1000
    n = 1
    for h in range(2, max(nH, 1) + 1):
        db = slope * math.log2(h) + rolloffOct * (f0 * h - 200) / 1000
        if db < throwaway:
            break
        n = h
    return n


def call_cost(call):
    """Analytic cost of one call in ns of one MI355X (used only for balancing)."""
    kind = call.get("kind", "soundgen")
    if kind == "harmonics":
        p = call.get("params", {})
        sr = float(p.get("samplingRate", 16000))
        psr = float(p.get("pitchSamplingRate", 3500))
        pitch = np.atleast_1d(call["pitch"])
        n = len(pitch) / psr * sr
        voiced = _finite(pitch)
        rows = 0
        if len(voiced):  # all-NA pitch: nothing voiced, no sine-bank rows
            rows = harmonic_rows(float(np.median(voiced)), sr, p.get("rolloff", -18), p.get("rolloffOct", -2),
                                 p.get("rolloffKHz", -6), p.get("throwaway", -120))
        return n * (rows * W_ROW + W_SAMPLE)
    a = call.get("args", {})
    sr = float(a.get("samplingRate", 16000))
    nSyl = max(1, int(a.get("nSyl", 1)))
    rep = max(1, int(a.get("repeatBout", 1)))
    dur = float(a.get("sylLen", 300)) * nSyl * rep + float(a.get("pauseLen", 200)) * (nSyl - 1) * rep
    n = dur / 1000.0 * sr
    vals = _anchor_values(a.get("pitchAnchors", "default"), [100.0, 150.0, 135.0, 100.0])
    rows = 0.0
    if vals is not None:
        f0 = float(np.exp(np.mean(np.log(np.maximum(vals, 1.0)))))
        rows = harmonic_rows(f0, sr, a.get("rolloff", -12), a.get("rolloffOct", -12), a.get("rolloffKHz", -6),
                             a.get("throwaway", -120))
        if float(a.get("subDep", 100)) > 0 and float(a.get("nonlinBalance", 0)) > 0:
            nsub = max(0, round(f0 / max(float(a.get("subFreq", 100)), 1.0)) - 1)
            share = min(1.0, float(a.get("nonlinBalance", 0)) / 100)
            rows *= 1 + nsub * share
    wl = max(4.0, 2 * math.floor(float(a.get("windowLength", 50)) * sr / 1000 / 2))
    hop = wl * (1 - float(a.get("overlap", 75)) / 100)
    frames = n / max(hop, 1.0)
    # a noise phase exists when some noise anchor is above throwaway (R's default
    # noiseAnchors are -120 dB: no breathing)
    na = a.get("noiseAnchors")
    nv = _finite(na.get("value", []) if isinstance(na, dict) else na)
    noise = 1.0 + bool((nv > float(a.get("throwaway", -120))).any())
    fft = 2 * 5 * wl * math.log2(wl) * frames * noise
    return n * (rows * W_ROW + W_SAMPLE) + fft * W_FLOP


def lpt_assign(costs, world):
    """Rank of each call: largest cost first onto the least-loaded rank
    (ties: lowest rank, then original order) -- deterministic everywhere."""
    import heapq
    costs = np.asarray(costs, dtype=np.float64)
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    heap = [(0.0, r) for r in range(world)]
    rank = np.zeros(len(costs), dtype=np.int64)
    for i in order:
        load, r = heapq.heappop(heap)
        rank[i] = r
        heapq.heappush(heap, (load + costs[i], r))
    return rank


def shard(calls, rank, world):
    """Indices (ascending) and calls this rank synthesizes, and every call's owner."""
    owner = lpt_assign([call_cost(c) for c in calls], world)
    idx = np.nonzero(owner == rank)[0]
    return idx, [calls[i] for i in idx], owner


def gather_packed(data, offsets, lengths, owner, rank, world, root=0, to_host=False):
    """The exchange step: every rank holds its shard's outputs packed in `data`
    (a 1-D float32 tensor on the communication device: the rank's GPU under
    RCCL, the CPU under gloo), call i of the shard at offsets[i] with lengths[i]
    samples (-1: the call failed). Returns, on the root, one entry per call of
    the batch in call order: a 1-D float32 tensor view of the received buffer
    (on the communication device: a GPU tensor under RCCL) or, with to_host, a
    float32 numpy array; an exception for a failed call. None elsewhere."""
    import torch
    import torch.distributed as dist
    dev = data.device
    n_loc = torch.tensor([int(data.numel())], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n_loc) for _ in range(world)]
    dist.all_gather(sizes, n_loc)
    sizes = [int(s.item()) for s in sizes]
    counts = [int(np.count_nonzero(owner == r)) for r in range(world)]
    table = torch.as_tensor(np.stack([np.asarray(offsets, np.int64), np.asarray(lengths, np.int64)]).reshape(-1),
                            device=dev)
    if rank != root:
        ops = []
        if counts[rank]:
            ops.append(dist.P2POp(dist.isend, table, root))
        if sizes[rank]:
            ops.append(dist.P2POp(dist.isend, data, root))
        for w in (dist.batch_isend_irecv(ops) if ops else []):
            w.wait()
        return None
    tables, bufs, ops = {}, {}, []
    for r in range(world):
        if r == root:
            continue
        tables[r] = torch.empty(2 * counts[r], dtype=torch.int64, device=dev)
        if counts[r]:
            ops.append(dist.P2POp(dist.irecv, tables[r], r))
        if sizes[r]:
            bufs[r] = torch.empty(sizes[r], dtype=torch.float32, device=dev)
            ops.append(dist.P2POp(dist.irecv, bufs[r], r))
    for w in (dist.batch_isend_irecv(ops) if ops else []):
        w.wait()
    result = [None] * len(owner)
    for r in range(world):
        idx = np.nonzero(owner == r)[0]
        if r == root:
            buf, off, ln = data, np.asarray(offsets, np.int64), np.asarray(lengths, np.int64)
        else:
            t = tables[r].cpu().numpy().reshape(2, -1)
            # a peer whose packed size is 0 (only empty or failed calls) sent no buffer
            buf, off, ln = bufs.get(r, torch.empty(0, dtype=torch.float32, device=dev)), t[0], t[1]
        if to_host:
            buf = buf.cpu().numpy()
        for i, o, n in zip(idx, off, ln):
            result[i] = RuntimeError("call %d failed on rank %d" % (i, r)) if n < 0 else buf[int(o):int(o) + int(n)]
    return result


def pack_outputs(outs, device="cpu"):
    """Host outputs (arrays or exceptions, shard order) -> packed float32 tensor,
    offsets, lengths (-1 for a failed call): the layout batch.synthesize_packed
    produces on the GPU, for synthesizers that return host arrays (tests)."""
    import torch
    lens = np.array([len(o) if not isinstance(o, Exception) else -1 for o in outs], dtype=np.int64)
    slot = np.where(lens > 0, (lens + 63) // 64 * 64, 0)
    offs = np.concatenate([[0], np.cumsum(slot)[:-1]]).astype(np.int64) if len(outs) else np.zeros(0, np.int64)
    data = np.zeros(int(slot.sum()), np.float32)
    for o, n, y in zip(offs, lens, outs):
        if n > 0:
            data[o:o + n] = np.asarray(y, np.float32)
    return torch.from_numpy(data).to(device), offs, lens


def synthesize_sharded(calls, rank, world, device=None, synth=None, root=0, comm_device=None, to_host=False):
    """Every rank synthesizes its LPT shard and the root gathers the batch in call
    order (gather_packed). Default: batch.synthesize_packed on the rank's GPU
    (LOCAL_RANK), the packed device buffer sent as is (RCCL). `synth` maps a list
    of calls to host outputs instead (packed on `comm_device`, e.g. "cpu" for gloo).
    The root's entries are float32 tensor views on the communication device, on
    every path (world 1 included); to_host=True returns float32 numpy arrays."""
    if device is None:
        device = int(os.environ.get("LOCAL_RANK", "0"))
    idx, mine, owner = shard(calls, rank, world)
    if synth is None:
        from . import batch
        data, offs, lens = batch.synthesize_packed(mine, device)
    else:
        outs = synth(mine) if mine else []
        data, offs, lens = pack_outputs(outs, comm_device or "cpu")
    if world == 1:
        buf = data.cpu().numpy() if to_host else data
        return [RuntimeError("call failed") if n < 0 else buf[int(o):int(o) + int(n)] for o, n in zip(offs, lens)]
    return gather_packed(data, offs, lens, owner, rank, world, root, to_host)


def gather_timed(data, offsets, lengths, calls, rank, world, root=0):
    """The bench's exchange step at N > 1 (bench.py, default): every rank's packed
    shard outputs (`data`, shard call i at offsets[i], lengths[i] samples, -1
    failed; shard order as shard() lists it) gathered to the root in call order
    by gather_packed, bracketed by barriers. Returns (root: the per-call list,
    else None; wall ms of the exchange, the same on every rank's clock span).
    A rank whose part of the exchange raises still reaches the closing
    agreement: every rank all-reduces a failure flag before the barrier, and all
    of them raise if any rank failed (the caller's 'reported, not fatal' holds
    on every rank, not only on the one that raised)."""
    import time

    import torch
    import torch.distributed as dist
    owner = lpt_assign([call_cost(c) for c in calls], world)
    sync = (lambda: torch.cuda.synchronize(data.device)) if data.is_cuda else (lambda: None)
    dist.barrier()
    sync()
    t = time.perf_counter()
    got, err = None, None
    try:
        got = gather_packed(data, offsets, lengths, owner, rank, world, root)
        sync()
    except Exception as e:  # noqa: BLE001 -- agreed on below, then re-raised on every rank
        err = e
    flag = torch.tensor([1 if err is not None else 0], dtype=torch.int32,
                        device=data.device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(flag, op=dist.ReduceOp.MAX)
    dist.barrier()
    if int(flag.item()):
        raise RuntimeError("gather_timed: the exchange failed on %s" %
                           ("this rank: %r" % (err,) if err is not None else "another rank"))
    return got, (time.perf_counter() - t) * 1e3

