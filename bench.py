"""bench.py — synthesized audio samples/s of the soundgen hot path on MI355X.

Workload (BASELINE.json configs[1], the config the metric is quoted on, fits
one GPU): C2 = 1024 x generateHarmonics(pitch = rep(f0, 3500),
samplingRate = 44100, temperature = 0, nonlinBalance = 0, rolloff = -12,
rolloffOct = -12, rolloffKHz = -6, pitchFloor = 50), f0 log-uniform in
[80, 400] Hz, numpy PCG64 seed 20261015.

A "step" = one pass of the hot path over the whole batch (plan/upload happen
before the timed region; inputs are resident in HBM). With N ranks each rank
synthesizes its own 1024-call shard (weak scaling, no data-path collective);
time = max over ranks, value = samples of all ranks / time.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SEED = 20261015
METRIC = "synthesized audio samples/sec (whole node) @44.1 kHz; RMS error vs R ref"
C2_PARAMS = dict(samplingRate=44100, pitchSamplingRate=3500, temperature=0, nonlinBalance=0, attackLen=50,
                 rolloff=-12, rolloffOct=-12, rolloffKHz=-6, rolloffParab=0, rolloffParabHarm=3, pitchFloor=50,
                 pitchCeiling=3500, throwaway=-120)
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
VALU_PEAK_OPS = 256 * 4 * 32 * 2.4e9  # wave64 VALU lane-ops/s (78.6e12)


def c2_calls(n_calls, rank=0):
    rng = np.random.Generator(np.random.PCG64(SEED + 7919 * rank))
    f0 = np.exp(rng.uniform(np.log(80.0), np.log(400.0), n_calls))
    return [{"kind": "harmonics", "pitch": np.full(3500, f), "params": C2_PARAMS} for f in f0]


def cpu_baseline(calls, budget_s):
    """Oracle (C restatement of the R algorithm), 1 thread, bounded sample."""
    from oracle import oracle as O
    O.lib()
    t0 = time.perf_counter()
    n_samples = n = 0
    for c in calls:
        n_samples += len(O.generate_harmonics(c["pitch"], **c["params"]))
        n += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": n_samples / dt, "unit": "samples/s", "cores": 1, "kind": "port",
            "sample": "%d of the C2 calls (%d samples) through oracle/sg_oracle.c, single thread" % (n, n_samples)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--calls", type=int, default=1024)
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from soundgen_beta_amd import batch, native
    calls = c2_calls(args.calls, rank)
    ctx = native.Context(local)
    plan = batch.Plan(calls, ctx)
    assert (plan.status == 0).all(), [plan.message(i) for i in np.nonzero(plan.status)[0][:3]]
    plan.upload()
    out = torch.empty(plan.total, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream

    for _ in range(args.warmup):
        plan.execute(out.data_ptr(), sptr)
    torch.cuda.synchronize(dev)
    L = native.lib()
    L.sg_set_profiling(ctx.ptr, 1)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        plan.execute(out.data_ptr(), sptr)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    L.sg_set_profiling(ctx.ptr, 0)
    import ctypes as C
    sine_ms, nprof = C.c_double(), C.c_int64()
    native.check(L.sg_profile_read(ctx.ptr, C.byref(sine_ms), C.byref(nprof)), ctx.ptr)

    samples_rank = plan.total
    if dist:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        s = torch.tensor([samples_rank], device=dev, dtype=torch.float64)
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        samples_all = float(s.item())
    else:
        samples_all = float(samples_rank)
    value = samples_all * args.steps / dt

    if rank == 0:
        st = plan.stats()
        # algorithmic bytes of one sine-bank launch: fp32 epoch
        # waveform write + amplitude matrices + pitch segments/knots
        n_gc = sum(int(np.ceil(c["pitch"].size)) for c in calls[:0])
        launches = max(1, nprof.value // args.steps)  # sine-bank launches per step (batch slices)
        alg_bytes = (4 * st["harm_samples"] + st["harm_amp_bytes"]) / launches
        sine_s = sine_ms.value / 1e3
        achieved = alg_bytes / sine_s / 1e9 if sine_s > 0 else 0.0
        # VALU: per (sample, row) the kernel issues 3 instructions (ISA, C=2 path)
        valu_ops = 2.0 * st["harm_terms"] / launches
        host = out[: min(plan.total, 4 * 50000)].cpu().numpy()
        from oracle import oracle as O
        rms = []
        for i in range(min(4, plan.n)):
            y = host[plan.offsets[i]:plan.offsets[i] + plan.lengths[i]].astype(np.float64)
            if plan.offsets[i] + plan.lengths[i] > host.size:
                break
            ref = O.generate_harmonics(calls[i]["pitch"], **calls[i]["params"])
            rms.append(float(np.sqrt(np.mean((y - ref) ** 2))) if len(ref) == len(y) else float("inf"))
        res = {
            "metric": METRIC, "value": value, "unit": "samples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32 (fp64 phase)", "data": "synthetic",
            "config": {"workload": "C2: %d x 1 s static-f0 tones, generateHarmonics, 44.1 kHz, harmonics only"
                       % args.calls, "calls_per_gpu": args.calls, "samples_per_gpu": samples_rank,
                       "sampling_rate": 44100, "parallelism": "dp%d (independent shards)" % world},
            "rms_error_vs_oracle": max(rms) if rms else None,
            "roofline": {"bound": "hbm", "kernel": "sg_sine_bank", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "alg_bytes_per_launch": alg_bytes, "avg_launch_ms": sine_ms.value,
                         "launches_timed": nprof.value,
                         "valu": {"ops_per_launch": valu_ops, "achieved_ops_s": valu_ops / sine_s if sine_s else 0,
                                  "peak_ops_s": VALU_PEAK_OPS,
                                  "frac": valu_ops / sine_s / VALU_PEAK_OPS if sine_s else 0}},
        }
        if not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(calls, args.cpu_budget)
        print(json.dumps(res), flush=True)
    plan.close()
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
