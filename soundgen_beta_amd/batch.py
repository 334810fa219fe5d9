"""Batch path: plan (host, bit-exact bookkeeping) -> upload (HBM) ->
execute (HIP kernels, no host sync) for a list of independent calls.

A call is a dict:
  {"kind": "harmonics", "pitch": array, "params": {...}, "amplAnchors": ...,
   "normals": array|None, "uniforms": array|None}
  {"kind": "soundgen", "args": {...R soundgen() args...}, "normals":..., "uniforms":...}
"""
import ctypes as C

import numpy as np

from . import _abi, native, rargs


class Marshalled:
    """The C descriptors of a list of calls (sg_call_desc array) and the buffers
    behind them: the Python half of planning, separable from the native half so
    that the two overlap across chunks (plan_uploaded)."""

    def __init__(self, calls):
        self.holder = h = rargs.Holder()
        n = self.n = len(calls)
        N = max(n, 1)
        descs = (_abi.sg_call_desc * N)()
        args = (_abi.sg_soundgen_args * N)()
        self._structs = [args]
        # soundgen() calls with injected draws go through the bulk writers: their
        # argument structs (ArgsWriter) and descriptor fields are written for all
        # calls at once; harmonics calls and draw callbacks take the per-call path
        aw = rargs.ArgsWriter(h, args, N)
        fast, rand = [], []
        for i, c in enumerate(calls):
            kind = c.get("kind", "soundgen")
            if kind != "harmonics" and c.get("rng") is None:
                aw.add(i, c.get("args", {}))
                fast.append(i)
                rand.append(h.random_addrs(c.get("normals"), c.get("uniforms")))
                continue
            d = descs[i]
            d.random = h.random(c.get("normals"), c.get("uniforms"), c.get("rng"))
            if kind == "harmonics":
                d.kind = _abi.SG_CALL_HARMONICS
                p = self.holder.arr(c["pitch"])
                d.pitch, d.pitch_len = _abi.dptr(p), len(p)
                hp = rargs.fill_harm_params(c.get("params", {}))
                self._structs.append(hp)
                d.harm = C.pointer(hp)
                d.amplAnchors = self.holder.anchors(rargs.as_anchors(c.get("amplAnchors")))
            else:
                d.kind = _abi.SG_CALL_SOUNDGEN
                aw.add(i, c.get("args", {}))
                d.args = C.pointer(args[i])
        aw.finish()
        if fast:
            dv = np.frombuffer(descs, dtype=_DESC_VIEW, count=N)
            idx = np.asarray(fast, dtype=np.int64)
            r = np.array(rand, dtype=np.uint64).reshape(-1, 4)
            dv["kind"][idx] = _abi.SG_CALL_SOUNDGEN
            dv["args"][idx] = C.addressof(args) + idx.astype(np.uint64) * C.sizeof(_abi.sg_soundgen_args)
            dv["normals"][idx], dv["n_normals"][idx] = r[:, 0], r[:, 1]
            dv["uniforms"][idx], dv["n_uniforms"][idx] = r[:, 2], r[:, 3]
        self.descs = descs


def _desc_view():
    D, R = _abi.sg_call_desc, _abi.sg_random
    o = D.random.offset
    f = [("kind", "<i4", D.kind.offset), ("args", "<u8", D.args.offset),
         ("normals", "<u8", o + R.normals.offset), ("n_normals", "<i8", o + R.n_normals.offset),
         ("uniforms", "<u8", o + R.uniforms.offset), ("n_uniforms", "<i8", o + R.n_uniforms.offset)]
    return np.dtype({"names": [x[0] for x in f], "formats": [x[1] for x in f], "offsets": [x[2] for x in f],
                     "itemsize": C.sizeof(D)})


_DESC_VIEW = _desc_view()


class NodePlan:
    """A batch planned over a native.Node (sg_node_plan_batch): whole-batch
    lengths, offsets and statuses in call order (sg_plan_batch's layout), the
    device each call went to, and synchronous execution into host memory."""

    def __init__(self, calls, node):
        self.node = node
        m = Marshalled(calls)
        self._m = m
        n = self.n = m.n
        L = native.lib()
        self.ptr = C.c_void_p()
        node.check(L.sg_node_plan_batch(node.ptr, m.descs, n, C.byref(self.ptr)))
        i64p = C.POINTER(C.c_int64)
        self.lengths = np.zeros(n, dtype=np.int64)
        self.offsets = np.zeros(n, dtype=np.int64)
        L.sg_node_plan_lengths(self.ptr, self.lengths.ctypes.data_as(i64p), self.offsets.ctypes.data_as(i64p))
        self.status = np.zeros(n, dtype=np.int32)
        L.sg_node_plan_status(self.ptr, self.status.ctypes.data_as(C.POINTER(C.c_int32)))
        self.owner = np.zeros(n, dtype=np.int32)
        L.sg_node_plan_owner(self.ptr, self.owner.ctypes.data_as(C.POINTER(C.c_int32)))
        self.cost = np.zeros(n, dtype=np.float64)
        L.sg_node_plan_costs(self.ptr, self.cost.ctypes.data_as(C.POINTER(C.c_double)))
        self.total = int(L.sg_node_plan_total_samples(self.ptr))

    def message(self, i):
        return native.lib().sg_node_plan_call_message(self.ptr, i).decode()

    def shard_samples(self, k):
        return int(native.lib().sg_node_plan_shard_samples(self.ptr, k))

    def chunks(self, k):
        return int(native.lib().sg_node_plan_chunks(self.ptr, k))

    @property
    def diverged(self):
        return bool(native.lib().sg_node_plan_diverged(self.ptr))

    def call_work(self):
        """Per call: sine-bank (sample, row) terms and FFT flops the shard plans emit."""
        rows, flops = np.zeros(self.n), np.zeros(self.n)
        dp = C.POINTER(C.c_double)
        native.lib().sg_node_plan_call_work(self.ptr, rows.ctypes.data_as(dp), flops.ctypes.data_as(dp))
        return rows, flops

    def execute_to_host(self, dtype=np.float64):
        """The packed batch (sg_node_plan_total_samples values, call i at offsets[i])."""
        out = np.zeros(max(self.total, 1), dtype=dtype)
        L = native.lib()
        if dtype == np.float32:
            self.node.check(L.sg_node_execute_to_host_f32(self.node.ptr, self.ptr,
                                                          out.ctypes.data_as(C.POINTER(C.c_float))))
        else:
            self.node.check(L.sg_node_execute_to_host(self.node.ptr, self.ptr,
                                                      out.ctypes.data_as(C.POINTER(C.c_double))))
        return out[:self.total]

    def close(self):
        if self.ptr:
            native.lib().sg_node_plan_destroy(self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def synthesize_node(calls, devices=None, node=None):
    """soundgen_batch over several devices of this process (sg_node): the list of
    per-call float64 waveforms (an exception object for a call that failed)."""
    from . import native as _n
    own = node is None
    node = node or _n.Node(devices)
    try:
        p = NodePlan(calls, node)
        y = p.execute_to_host()
        out = []
        for i in range(p.n):
            if p.status[i]:
                out.append(_n.SoundgenError(int(p.status[i]), p.message(i)))
            else:
                out.append(y[p.offsets[i]:p.offsets[i] + p.lengths[i]].copy())
        p.close()
        return out
    finally:
        if own:
            node.close()


class Plan:
    def __init__(self, calls, ctx=None, marshalled=None):
        """Plan `calls` (or the already marshalled ones). ctx may be None: planning
        is host-only."""
        self.ctx = ctx
        m = marshalled if marshalled is not None else Marshalled(calls)
        self._m = m  # keeps the descriptors' buffers alive
        self.holder = m.holder
        n = m.n
        descs = m.descs
        self._descs = descs
        self.ptr = C.c_void_p()
        L = native.lib()
        native.check(L.sg_plan_batch(ctx.ptr if ctx else None, descs, n, C.byref(self.ptr)), ctx.ptr if ctx else None)
        self.n = n
        self.lengths = np.zeros(n, dtype=np.int64)
        self.offsets = np.zeros(n, dtype=np.int64)
        i64p = C.POINTER(C.c_int64)
        L.sg_plan_lengths(self.ptr, self.lengths.ctypes.data_as(i64p), self.offsets.ctypes.data_as(i64p))
        self.status = np.zeros(n, dtype=np.int32)
        L.sg_plan_status(self.ptr, self.status.ctypes.data_as(C.POINTER(C.c_int32)))
        self.total = int(L.sg_plan_total_samples(self.ptr))
        self.uploaded = False

    def message(self, i):
        return native.lib().sg_plan_call_message(self.ptr, i).decode()

    def stats(self):
        v = [C.c_int64() for _ in range(4)]
        native.lib().sg_plan_kernel_stats(self.ptr, *[C.byref(x) for x in v])
        w = [C.c_int64(), C.c_int64(), C.c_double()]
        native.lib().sg_plan_stft_stats(self.ptr, *[C.byref(x) for x in w])
        return dict(harm_samples=v[0].value, harm_terms=v[1].value, harm_amp_bytes=v[2].value,
                    fft_frames=v[3].value, stft_samples=w[0].value, stft_bytes=w[1].value, stft_flops=w[2].value)

    def sine_tasks(self):
        """Sine-bank tasks of the uploaded plan by class: (sg_sine_bank, _pairs, _tall,
        _tall_pairs, _hp)."""
        v = (C.c_int64 * 5)()
        native.check(native.lib().sg_plan_sine_tasks(self.ptr, v))
        return tuple(int(x) for x in v)

    def table_stats(self):
        """Wavetable spans of the uploaded plan: (tables, samples, terms)."""
        v = [C.c_int64() for _ in range(3)]
        native.check(native.lib().sg_plan_table_stats(self.ptr, *[C.byref(x) for x in v]))
        return tuple(x.value for x in v)

    def noise_conditioning(self):
        """Per call: the planner's fp32 conditioning estimate of its pre-filter noise
        (the largest over its filtered bouts; above the threshold the noise frames
        take the fp64 kernel)."""
        v = np.zeros(self.n, dtype=np.float64)
        native.check(native.lib().sg_plan_noise_conditioning(self.ptr, v.ctypes.data_as(C.POINTER(C.c_double))))
        return v

    def conditioning(self):
        """Per call: the planner's fp32 conditioning estimate of its formant filter
        (the largest over its filtered bouts; bouts above the threshold go fp64)."""
        v = np.zeros(self.n, dtype=np.float64)
        native.check(native.lib().sg_plan_conditioning(self.ptr, v.ctypes.data_as(C.POINTER(C.c_double))))
        return v

    def precision(self):
        """Per call: bouts on the fp64 filter path; totals of fp64 frames and tasks."""
        v = np.zeros(self.n, dtype=np.int32)
        fr, tk = C.c_int64(), C.c_int64()
        native.lib().sg_plan_precision(self.ptr, v.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(fr), C.byref(tk))
        return v, fr.value, tk.value

    def call_work(self):
        """Per call: sine-bank (sample, row) terms and nominal FFT flops."""
        rows, flops = np.zeros(self.n), np.zeros(self.n)
        dp = C.POINTER(C.c_double)
        native.lib().sg_plan_call_work(self.ptr, rows.ctypes.data_as(dp), flops.ctypes.data_as(dp))
        return rows, flops

    def device_bytes(self):
        return int(native.lib().sg_plan_device_bytes(self.ptr))

    def upload(self, ctx=None):
        ctx = ctx or self.ctx
        native.check(native.lib().sg_plan_upload(ctx.ptr, self.ptr), ctx.ptr)
        self.ctx = ctx
        self.uploaded = True

    def release_host(self):
        """Free the plan's host copies after upload (execution keeps working)."""
        native.check(native.lib().sg_plan_release_host(self.ptr), None)

    def execute(self, d_out_ptr, stream_ptr=None):
        """Run the kernels writing fp32 samples to device pointer d_out_ptr."""
        native.check(native.lib().sg_execute(self.ctx.ptr, self.ptr, C.c_void_p(d_out_ptr),
                                             C.c_void_p(stream_ptr) if stream_ptr else None), self.ctx.ptr)

    def pcm16(self, d_in_ptr, d_out_ptr, stream_ptr=None):
        """16-bit PCM of every call (seewave::savewav's conversion) from the packed fp32
        output at d_in_ptr into int16 at the same offsets of d_out_ptr (device)."""
        native.check(native.lib().sg_pcm16(self.ctx.ptr, self.ptr, C.c_void_p(d_in_ptr), C.c_void_p(d_out_ptr),
                                           C.c_void_p(stream_ptr) if stream_ptr else None), self.ctx.ptr)

    def close(self):
        if self.ptr:
            native.lib().sg_plan_destroy(self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def execute_plans(ctx, plans, d_out_ptrs, stream_ptr=None):
    """Run several uploaded plans as one batch (sg_execute_plans): plan i writes
    its calls to device pointer d_out_ptrs[i]; the harmonic chains of later plans
    overlap the spectral phases of earlier ones on the context's second stream."""
    n = len(plans)
    if n == 0:
        return
    P = (C.c_void_p * n)(*[p.ptr for p in plans])
    O = (C.c_void_p * n)(*[C.c_void_p(o) for o in d_out_ptrs])
    native.check(native.lib().sg_execute_plans(ctx.ptr, P, O, n, C.c_void_p(stream_ptr) if stream_ptr else None),
                 ctx.ptr)


def chunk_sizes(n, chunk, ramp=True):
    """Chunk sizes for plan_uploaded: `chunk` calls each; with ramp, a first and a
    last chunk of chunk / 4 calls, so that the pipeline's fill (marshal + plan of
    the first chunk, nothing to overlap with) and drain (the last upload) are short."""
    sizes = []
    q = max(1, chunk // 4)
    if ramp and n > chunk:
        sizes.append(q)
    while sum(sizes) < n:
        left = n - sum(sizes)
        if ramp and len(sizes) > 0 and chunk >= left > q:  # the tail: [left - q, q]
            sizes += [left - q, q]
            break
        sizes.append(min(chunk, left))
    return sizes


def plan_uploaded(calls, ctx, chunk, timings=None):
    """Plan `calls` in chunks of `chunk` calls (an int, or a list of chunk sizes)
    and upload each plan, yielding (plan, first call index) in order. A
    three-stage pipeline: while chunk k
    uploads (main thread), chunk k + 1 is planned natively and chunk k + 2 is
    marshalled (two workers). The native calls run without the GIL (ctypes), so
    only marshalling holds it. Each yielded plan is uploaded and its host arrays
    released. `timings` (a list) receives per chunk the seconds of each stage and
    the main thread's wait for the planner."""
    import time
    from concurrent.futures import ThreadPoolExecutor
    sizes = list(chunk) if isinstance(chunk, (list, tuple)) else chunk_sizes(len(calls), chunk, ramp=False)
    starts = [sum(sizes[:i]) for i in range(len(sizes))]
    if not starts or not len(calls):
        return
    stage = {}

    def piece(i):
        return calls[starts[i]:starts[i] + sizes[i]]

    def marshal(i):
        t = time.perf_counter()
        m = Marshalled(piece(i))
        stage[("marshal", i)] = time.perf_counter() - t
        return m

    def plan(i, m):
        t = time.perf_counter()
        p = Plan(None, ctx, m)
        stage[("plan", i)] = time.perf_counter() - t
        return p
    with ThreadPoolExecutor(2) as ex:
        pfut = ex.submit(plan, 0, marshal(0))
        mfut = ex.submit(marshal, 1) if len(starts) > 1 else None
        for i, a in enumerate(starts):
            t0 = time.perf_counter()
            p = pfut.result()
            if mfut is not None:
                pfut = ex.submit(plan, i + 1, mfut.result())
                mfut = ex.submit(marshal, i + 2) if i + 2 < len(starts) else None
            t1 = time.perf_counter()
            p.upload()
            p.release_host()
            t2 = time.perf_counter()
            if timings is not None:
                timings.append(dict(chunk=i, marshal_s=stage.get(("marshal", i)), plan_s=stage.get(("plan", i)),
                                    wait_s=t1 - t0, upload_s=t2 - t1))
            yield p, a


def synthesize_to_wav(calls, paths, sampling_rates, device=0, return_float=False):
    """soundgen(..., savePath = path) for a batch: synthesize on the GPU, convert
    every call to 16-bit PCM on the GPU (half the bytes cross PCIe), write one
    WAV file per call (R/soundgen.R:854-856). Returns the int16 arrays; with
    return_float also the fp32 waveforms of the same execute: (pcm, waves)."""
    import torch
    from . import api
    ctx = native.default_context(device)
    plan = Plan(calls, ctx)
    plan.upload()
    dev = "cuda:%d" % device
    out = torch.empty(max(plan.total, 1), dtype=torch.float32, device=dev)
    pcm = torch.zeros(max(plan.total, 1), dtype=torch.int16, device=dev)
    sptr = torch.cuda.current_stream(device).cuda_stream
    plan.execute(out.data_ptr(), sptr)
    plan.pcm16(out.data_ptr(), pcm.data_ptr(), sptr)
    torch.cuda.synchronize(device)
    host = pcm.cpu().numpy()
    hostf = out.cpu().numpy() if return_float else None
    res, waves = [], []
    for i in range(plan.n):
        if plan.status[i] != 0:
            err = native.SoundgenError(int(plan.status[i]), plan.message(i))
            res.append(err)
            waves.append(err)
            continue
        y = host[plan.offsets[i]:plan.offsets[i] + plan.lengths[i]].copy()
        api.write_wav(paths[i], y, sampling_rates[i] if hasattr(sampling_rates, "__len__") else sampling_rates)
        res.append(y)
        if return_float:
            waves.append(hostf[plan.offsets[i]:plan.offsets[i] + plan.lengths[i]].copy())
    plan.close()
    return (res, waves) if return_float else res


def synthesize_packed(calls, device=0):
    """Plan + run a batch on one GPU and keep the outputs packed in HBM: returns
    (float32 device tensor, offsets, lengths), call i at offsets[i] with
    lengths[i] samples, -1 for a call the planner refused (dist.gather_packed
    sends this buffer as is)."""
    import torch
    ctx = native.default_context(device)
    plan = Plan(calls, ctx)
    plan.upload()
    out = torch.empty(max(plan.total, 1), dtype=torch.float32, device="cuda:%d" % device)
    plan.execute(out.data_ptr(), torch.cuda.current_stream(device).cuda_stream)
    torch.cuda.synchronize(device)
    lens = np.where(plan.status == 0, plan.lengths, -1).astype(np.int64)
    offs = plan.offsets.astype(np.int64).copy()
    plan.close()
    return out[:plan.total], offs, lens


def synthesize(calls, device=0):
    """Plan + run a batch on one GPU; returns a list of float32 numpy arrays."""
    import torch
    ctx = native.default_context(device)
    plan = Plan(calls, ctx)
    plan.upload()
    out = torch.empty(max(plan.total, 1), dtype=torch.float32, device="cuda:%d" % device)
    stream = torch.cuda.current_stream(device)
    plan.execute(out.data_ptr(), stream.cuda_stream)
    # sg_execute launches on torch's current stream (handle 0 = the null stream)
    torch.cuda.synchronize(device)
    host = out.cpu().numpy()
    res = []
    for i in range(plan.n):
        if plan.status[i] != 0:
            res.append(native.SoundgenError(int(plan.status[i]), plan.message(i)))
        else:
            res.append(host[plan.offsets[i]:plan.offsets[i] + plan.lengths[i]].copy())
    return res
