"""bench.py — synthesized audio samples/s of the soundgen hot path on MI355X.

Default workload (BASELINE.json configs[1], the config the metric is quoted
on, fits one GPU): C2 = 1024 x generateHarmonics(pitch = rep(f0, 3500),
samplingRate = 44100, temperature = 0, nonlinBalance = 0, rolloff = -12,
rolloffOct = -12, rolloffKHz = -6, pitchFloor = 50), f0 log-uniform in
[80, 400] Hz, numpy PCG64 seed 20261015.
--config c3 / c4 run the other single-GPU configs:
  C3 1024 x 2 s vowels, formant filter + breathing noise (uniform draws injected)
  C4 512 x 3 s, subharmonics + jitter/shimmer, temperature 0.05 (draws injected)

A "step" = one pass of the hot path over the whole batch (planning and upload
happen before the timed region; inputs are resident in HBM). With N ranks each
rank synthesizes its own shard (weak scaling, no data-path collective);
time = max over ranks, value = samples of all ranks / time.
"""
import argparse
import ctypes as C
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
HBM_PEAK_GBS = 8000.0                 # MI355X_MICROARCH.md chip table (spec)
VALU_PEAK_OPS = 157.3e12  # f32 lane-ops/s at the packed rate (v_pk_fma_f32 / v_pk_add_f32), which the sine bank uses
FP32_PEAK_TFLOPS = 157.3              # MI355X FP32 vector (packed FMA)


def _rng(rank, salt):
    return np.random.Generator(np.random.PCG64(SEED + 7919 * rank + salt))


def c2_calls(n_calls, rank=0):
    rng = _rng(rank, 0)
    f0 = np.exp(rng.uniform(np.log(80.0), np.log(400.0), n_calls))
    return [{"kind": "harmonics", "pitch": np.full(3500, f), "params": C2_PARAMS} for f in f0]


def c3_calls(n_calls, rank=0):
    rng = _rng(rank, 3)
    vowels = np.array(list("aoieu0"))
    v = rng.choice(vowels, n_calls)
    a = np.exp(rng.uniform(np.log(90), np.log(250), n_calls))
    b = np.exp(rng.uniform(np.log(90), np.log(250), n_calls))
    n = rng.uniform(-40, -10, n_calls)
    per = 1102 * 170  # noise spectrum uniforms per call (1102 bins x ~165 frames)
    U = rng.uniform(size=per * n_calls)
    calls = []
    for i in range(n_calls):
        args = dict(sylLen=2000, samplingRate=44100, temperature=0, addSilence=0, windowLength=50, overlap=75,
                    formants=str(v[i]), pitchAnchors=[float(a[i]), float(b[i])],
                    noiseAnchors={"time": [0, 2000], "value": [float(n[i]), float(n[i])]}, formantsNoise=None)
        calls.append({"kind": "soundgen", "args": args, "uniforms": U[i * per:(i + 1) * per]})
    return calls


def c4_calls(n_calls, rank=0):
    rng = _rng(rank, 4)
    s = rng.uniform(60, 200, n_calls)
    d = rng.uniform(40, 150, n_calls)
    j = rng.uniform(0.3, 2, n_calls)
    l = rng.uniform(1, 20, n_calls)
    h = rng.uniform(5, 20, n_calls)
    a = np.exp(rng.uniform(np.log(150), np.log(600), n_calls))
    b = np.exp(rng.uniform(np.log(150), np.log(600), n_calls))
    pn, pu = 40000, 20000
    Z = rng.standard_normal(pn * n_calls)
    U = rng.uniform(size=pu * n_calls)
    calls = []
    for i in range(n_calls):
        args = dict(sylLen=3000, samplingRate=44100, nonlinBalance=100, temperature=0.05, subFreq=float(s[i]),
                    subDep=float(d[i]), jitterDep=float(j[i]), jitterLen=float(l[i]), shimmerDep=float(h[i]),
                    shortestEpoch=300, pitchAnchors=[float(a[i]), float(b[i])], addSilence=0)
        calls.append({"kind": "soundgen", "args": args, "normals": Z[i * pn:(i + 1) * pn],
                      "uniforms": U[i * pu:(i + 1) * pu]})
    return calls


def c5_calls(n_calls, rank=0):
    """C5: calls drawn uniformly from the 33 presets (R/presets.R:158-399,
    extracted to soundgen_beta_amd/presets.json); sylLen x U(0.5, 2) clamped to [20, 5000],
    pitch anchor values x 2^U(-0.5, 0.5), samplingRate 44100, addSilence 0, the
    preset's own temperature. Random draws come from one shared pre-drawn stream
    (every call reads it from the start; synthetic data)."""
    from soundgen_beta_amd import presets as P
    rng = _rng(rank, 5)
    names = P.names()
    base = {k: P.args(*k) for k in names}  # one copy per preset: calls share its formant lists
    Z = rng.standard_normal(200000)
    U = rng.uniform(size=4000000)
    calls = []
    for i in range(n_calls):
        spk, nm = names[int(rng.integers(len(names)))]
        a = dict(base[(spk, nm)])
        a["sylLen"] = float(np.clip(a.get("sylLen", 300) * rng.uniform(0.5, 2), 20, 5000))
        pa = a.get("pitchAnchors", "default")
        f = 2 ** rng.uniform(-0.5, 0.5)
        if pa == "default":
            a["pitchAnchors"] = {"time": [0, .1, .9, 1], "value": [100 * f, 150 * f, 135 * f, 100 * f]}
        elif pa is not None:
            a["pitchAnchors"] = {"time": pa["time"], "value": list(np.asarray(pa["value"], float) * f)}
        a["samplingRate"] = 44100
        a["addSilence"] = 0
        calls.append({"kind": "soundgen", "args": a, "normals": Z, "uniforms": U, "preset": spk + "$" + nm})
    return calls


CONFIGS = {
    "c2": (c2_calls, 1024, "C2: %d x 1 s static-f0 tones, generateHarmonics, 44.1 kHz, harmonics only"),
    "c3": (c3_calls, 1024, "C3: %d x 2 s vowels, soundgen() with formant filter + breathing noise, 44.1 kHz"),
    "c4": (c4_calls, 512, "C4: %d x 3 s soundgen() with subharmonics, jitter, shimmer, temperature 0.05, 44.1 kHz"),
    "c5": (c5_calls, 8192, "C5: %d calls per GPU drawn from the 33 presets (65,536 over 8 GPUs), 44.1 kHz"),
}


def oracle_call(O, c):
    if c["kind"] == "harmonics":
        return O.generate_harmonics(c["pitch"], normals=c.get("normals"), uniforms=c.get("uniforms"), **c["params"])
    return O.soundgen(normals=c.get("normals"), uniforms=c.get("uniforms"), **c["args"])


def cpu_baseline(calls, budget_s):
    """Oracle (C restatement of the R algorithm), 1 thread, bounded sample."""
    from oracle import oracle as O
    O.lib()
    t0 = time.perf_counter()
    n_samples = n = 0
    for c in calls:
        try:
            n_samples += len(oracle_call(O, c))
        except Exception:  # same unsupported calls as the GPU path
            continue
        n += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": n_samples / dt, "unit": "samples/s", "cores": 1, "kind": "port",
            "sample": "%d of the workload's calls (%d samples) through oracle/sg_oracle.c, single thread"
                      % (n, n_samples)}


def traffic_from_profiles(config, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary of
    this workload (profiles/rNN_<config>_traffic.json, tools/gpu_traffic.sh:
    separate FETCH_SIZE / WRITE_SIZE passes, gfx950 FETCH_SIZE doubled)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_%s_traffic.json" % config)))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    hits = [v["hbm_bytes"] for k, v in d.get("kernels", {}).items() if k.split(" ")[0] == kernel and "hbm_bytes" in v]
    if not hits:
        return None, None
    return max(hits), os.path.relpath(files[-1], ROOT)


def roofline(st, prof, steps, config):
    """Roofline of the step's dominant kernel (the one with the most event time):
    achieved = algorithmic bytes per launch / average launch duration (HIP events on
    the launch stream), SURVEY.md §8d per-unit bytes."""
    tot = {k: v[0] * v[1] for k, v in prof.items()}
    kern = max(tot, key=tot.get) if any(tot.values()) else "sg_sine_bank"
    ms, n = prof[kern]
    launches = max(1, n // steps)
    sec = ms / 1e3
    if kern == "sg_sine_bank":
        # fp32 epoch waveform write + the amplitude blocks it reads (A and dA columns)
        alg = (4 * st["harm_samples"] + st["harm_amp_bytes"]) / launches
        valu_ops = 2.0 * st["harm_terms"] / launches  # Clenshaw: 2 lane-ops per (sample, row, chain)
        extra = {"valu": {"ops_per_launch": valu_ops, "achieved_ops_s": valu_ops / sec if sec else 0,
                          "peak_ops_s": VALU_PEAK_OPS, "frac": valu_ops / sec / VALU_PEAK_OPS if sec else 0}}
    else:
        # source / uniforms + envelope columns read, trimmed output written
        alg = st["stft_bytes"] / launches
        fl = st["stft_flops"] / launches
        extra = {"flops": {"nominal_per_launch": fl, "achieved_tflops": fl / sec / 1e12 if sec else 0,
                           "peak_tflops": FP32_PEAK_TFLOPS,
                           "frac": fl / sec / 1e12 / FP32_PEAK_TFLOPS if sec else 0}}
    achieved = alg / sec / 1e9 if sec > 0 else 0.0
    traffic, src = traffic_from_profiles(config, kern)
    r = {"bound": "hbm", "kernel": kern, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "alg_bytes_per_launch": alg,
         "avg_launch_ms": ms, "launches_timed": n}
    if src:
        r["traffic_source"] = src
    r.update(extra)
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--calls", type=int, default=0, help="calls per GPU (default: the config's)")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gather", action="store_true",
                    help="after the timed steps, time the packed-output gather to rank 0 (RCCL point-to-point)")
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
    make, n_default, desc = CONFIGS[args.config]
    n_calls = args.calls or n_default
    calls = make(n_calls, rank)
    ctx = native.Context(local)
    t_plan = time.perf_counter()
    plan = batch.Plan(calls, ctx)
    t_plan = time.perf_counter() - t_plan
    failed = int((plan.status != 0).sum())
    if failed:  # e.g. loess-smoothed contours (3-10 anchors) are SG_E_UNSUPPORTED; their slots stay empty
        print("bench: %d of %d calls not synthesized: %s" % (failed, plan.n, plan.message(int(np.nonzero(plan.status)[0][0]))),
              file=sys.stderr)
    plan.upload()
    out = torch.empty(max(plan.total, 1), dtype=torch.float32, device=dev)
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
    prof = {}
    for kid, name in ((0, "sg_sine_bank"), (1, "sg_stft_ola")):
        ms, n = C.c_double(), C.c_int64()
        native.check(L.sg_profile_read_kernel(ctx.ptr, kid, C.byref(ms), C.byref(n)), ctx.ptr)
        prof[name] = (ms.value, n.value)

    samples_rank = int(plan.lengths.sum())  # synthesized samples (slot padding excluded)
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

    gather_ms = None
    if args.gather and dist:
        # SURVEY §8e exchange step: every peer sends its packed output to rank 0
        # concurrently (one xGMI link each); rank 0 receives into one buffer
        n_loc = torch.tensor([plan.total], device=dev, dtype=torch.int64)
        counts = [torch.zeros_like(n_loc) for _ in range(world)]
        dist.all_gather(counts, n_loc)
        counts = [int(c.item()) for c in counts]
        dist.barrier()
        torch.cuda.synchronize(dev)
        tg = time.perf_counter()
        if rank == 0:
            bufs = [torch.empty(max(counts[r], 1), dtype=torch.float32, device=dev) for r in range(1, world)]
            ops = [dist.P2POp(dist.irecv, bufs[r - 1][:counts[r]], r) for r in range(1, world) if counts[r]]
        else:
            ops = [dist.P2POp(dist.isend, out[:plan.total], 0)] if plan.total else []
        for w in (dist.batch_isend_irecv(ops) if ops else []):
            w.wait()
        torch.cuda.synchronize(dev)
        dist.barrier()
        gather_ms = (time.perf_counter() - tg) * 1e3

    if rank == 0:
        st = plan.stats()
        roof = roofline(st, prof, args.steps, args.config)
        from oracle import oracle as O
        rms = []
        host = None
        for i in [k for k in range(plan.n) if plan.status[k] == 0][:3]:
            lo, n = int(plan.offsets[i]), int(plan.lengths[i])
            y = out[lo:lo + n].double().cpu().numpy()
            ref = oracle_call(O, calls[i])
            rms.append(float(np.sqrt(np.mean((y - ref) ** 2))) if len(ref) == len(y) else float("inf"))
        res = {
            "metric": METRIC, "value": value, "unit": "samples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32 (fp64 phase)", "data": "synthetic",
            "config": {"workload": desc % n_calls, "calls_per_gpu": n_calls, "samples_per_gpu": samples_rank,
                       "sampling_rate": 44100, "parallelism": "dp%d (independent shards)" % world,
                       "plan_s": t_plan, "failed_calls": failed},
            "rms_error_vs_oracle": max(rms) if rms else None,
            "roofline": roof,
        }
        if gather_ms is not None:
            res["gather_ms"] = gather_ms
        if not args.no_cpu_baseline and world == 1:  # the CPU leg runs at N=1 only
            res["cpu_baseline"] = cpu_baseline(calls, args.cpu_budget)
        print(json.dumps(res), flush=True)
    plan.close()
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
