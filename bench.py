"""bench.py — synthesized audio samples/s of the soundgen hot path on MI355X.

Default workload: C5 (BASELINE.json configs[4], the config the
metric "(whole node)" is quoted on): ONE batch of 65,536 soundgen() calls drawn
from the 33 presets (R/presets.R:158-399, soundgen_beta_amd/presets.json),
sylLen x U(0.5, 2) clamped to [20, 5000] ms, pitch anchors x 2^U(-0.5, 0.5),
44.1 kHz, numpy PCG64 seed 20261015, random draws injected. It fits one
MI355X (288 GB of HBM; the arena takes ~40 GB per 16,384 calls), so N=1 runs all of it; with N ranks the SAME batch is
split by LPT over an analytic per-call cost (soundgen_beta_amd/dist.py), no
data-path collective: "scaling": "strong".
--config c2|c3|c4 run the other single-GPU configs (C2 1024 x 1 s tones,
C3 1024 x 2 s vowels with formant filter + breathing noise, C4 512 x 3 s
subharmonics/jitter/shimmer at temperature 0.05).

A "step" = one pass of the hot path over the whole batch: every kernel from
the envelopes and the sine bank to the final mix, inputs resident in HBM
(planning and upload happen before the timed region; plan time is reported),
ending with every waveform copied into pinned host memory ("from
sg_execute entry to waveforms resident in host memory"); each plan chunk's
copy overlaps the kernels of the chunks after it.
value = samples of all ranks / max over ranks of the timed wall time.
value_device_resident times the same steps without the copy.

With --gpus N and no WORLD_SIZE in the environment, bench.py starts itself
under torch.distributed.run with N ranks (one per GPU) before touching the GPU.
"""
import argparse
import ctypes as C
import json
import os
import subprocess
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
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
# VALU issue peak in f32 lane-operations/s at the packed rate: 256 CU x 4 SIMD x
# 16 lanes x 2.4 GHz = 39.3e12 lane-instructions/s, x 2 for v_pk_* (an FMA
# counted as ONE op; the 157.3 TFLOP/s figure counts it as two flops)
VALU_PEAK_OPS = 78.6e12
FP32_PEAK_TFLOPS = 157.3  # MI355X FP32 vector (packed FMA, 2 flops each)


def _rng(salt):
    return np.random.Generator(np.random.PCG64(SEED + salt))


def c2_calls(n_calls):
    rng = _rng(0)
    f0 = np.exp(rng.uniform(np.log(80.0), np.log(400.0), n_calls))
    return [{"kind": "harmonics", "pitch": np.full(3500, f), "params": C2_PARAMS} for f in f0]


def c3_calls(n_calls):
    rng = _rng(3)
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


def c4_calls(n_calls):
    rng = _rng(4)
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


def c5_calls(n_calls):
    """C5: calls drawn uniformly from the 33 presets (R/presets.R:158-399,
    extracted to soundgen_beta_amd/presets.json); sylLen x U(0.5, 2) clamped to [20, 5000],
    pitch anchor values x 2^U(-0.5, 0.5), samplingRate 44100, addSilence 0, the
    preset's own temperature. Random draws: every call reads its own window of one
    pre-drawn stream (a per-call offset from a second generator, so the call
    parameters are those of earlier rounds; synthetic data)."""
    from soundgen_beta_amd import presets as P
    rng = _rng(5)
    names = P.names()
    base = {k: P.args(*k) for k in names}  # one copy per preset: calls share its formant lists
    Z = rng.standard_normal(200000)
    U = rng.uniform(size=4000000)
    orng = _rng(55)  # window offsets: <= 100k of the 200k normals, <= 2M of the 4M uniforms
    oz = orng.integers(0, 100000, size=n_calls)
    ou = orng.integers(0, 2000000, size=n_calls)
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
        calls.append({"kind": "soundgen", "args": a, "normals": Z[oz[i]:], "uniforms": U[ou[i]:],
                      "preset": spk + "$" + nm})
    return calls


CONFIGS = {
    "c2": (c2_calls, 1024, "C2: %d x 1 s static-f0 tones, generateHarmonics, 44.1 kHz, harmonics only"),
    "c3": (c3_calls, 1024, "C3: %d x 2 s vowels, soundgen() with formant filter + breathing noise, 44.1 kHz"),
    "c4": (c4_calls, 512, "C4: %d x 3 s soundgen() with subharmonics, jitter, shimmer, temperature 0.05, 44.1 kHz"),
    "c5": (c5_calls, 65536, "C5: %d soundgen() calls drawn from the 33 presets (mixed sylLen and pitch contours), "
                            "44.1 kHz"),
}


def oracle_call(O, c):
    if c["kind"] == "harmonics":
        return O.generate_harmonics(c["pitch"], normals=c.get("normals"), uniforms=c.get("uniforms"), **c["params"])
    return O.soundgen(normals=c.get("normals"), uniforms=c.get("uniforms"), **c["args"])


def host_cores():
    """Host threads this job may use (the box exports its CPU share as
    OMP_NUM_THREADS; os.cpu_count() shows the whole machine there)."""
    n = os.cpu_count() or 1
    try:
        n = min(n, int(os.environ.get("OMP_NUM_THREADS", n)))
    except ValueError:
        pass
    return max(1, n)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(calls, budget_s):
    """The oracle (oracle/sg_oracle.c, a C restatement of the R algorithm) on a
    bounded sample of the same calls: one thread, then all host cores (a thread
    pool over calls; the oracle releases the GIL inside its C call)."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as O
    O.lib()

    def one(c):
        try:
            return len(oracle_call(O, c))
        except Exception:  # a call the oracle refuses counts no samples
            return 0

    t0 = time.perf_counter()
    n1 = s1 = 0
    for c in calls:
        s1 += one(c)
        n1 += 1
        if time.perf_counter() - t0 > budget_s / 2:
            break
    dt1 = time.perf_counter() - t0
    cores = host_cores()
    t0 = time.perf_counter()
    with ThreadPoolExecutor(cores) as ex:
        futs = []
        for c in calls:
            # keep 4 calls per thread in flight; stop submitting at the time budget
            while sum(not f.done() for f in futs[-8 * cores:]) >= 4 * cores:
                time.sleep(0.0005)
            if time.perf_counter() - t0 > budget_s / 2:
                break
            futs.append(ex.submit(one, c))
        sm = sum(f.result() for f in futs)
    dtm = time.perf_counter() - t0
    return {"value": sm / dtm, "unit": "samples/s", "cores": cores, "kind": "port",
            "sample": "the first %d calls of the workload (%d samples) through oracle/sg_oracle.c on a %d-thread pool"
                      % (len(futs), sm, cores),
            "single_thread": {"value": s1 / dt1, "sample": "the first %d calls (%d samples), 1 thread" % (n1, s1)},
            "host": {"nproc": os.cpu_count(), "cores_used": cores, "model": cpu_model()},
            "note": "R unavailable; CPU baseline = C restatement of the R algorithm"}


def rms_check(plans, out, calls, n_check):
    """RMS error vs the oracle (after the timed region) of n_check calls spread
    evenly over every plan's synthesized calls, on the /max-normalised waveform
    both return (R/soundgen.R:807); lengths must match exactly. The calls the
    planner sent to the fp64 filter path are all included when present."""
    if n_check <= 0:
        return None
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as O
    O.lib()
    per = max(1, -(-n_check // max(1, len(plans))))
    picks = []  # (global offset, length, call index, fp64 path)
    for p, b, ix in plans:
        ok = np.nonzero(p.status == 0)[0]
        if not len(ok):
            continue
        hp = p.precision()[0]
        sel = set(ok[np.linspace(0, len(ok) - 1, min(per, len(ok))).round().astype(int)].tolist())
        sel |= set(ok[hp[ok] > 0][:2].tolist())  # fp64-path calls, two per plan
        picks += [(b + int(p.offsets[i]), int(p.lengths[i]), int(ix[i]), bool(hp[i] > 0)) for i in sorted(sel)]
    ys = [out[lo:lo + n].double().cpu().numpy() for lo, n, _, _ in picks]

    def one(k):
        ref = oracle_call(O, calls[picks[k][2]])
        y = ys[k]
        return float(np.sqrt(np.mean((y - ref) ** 2))) if len(ref) == len(y) else float("inf")
    with ThreadPoolExecutor(host_cores()) as ex:
        errs = list(ex.map(one, range(len(picks))))
    if not errs:
        return None
    presets = sorted({calls[pk[2]].get("preset", calls[pk[2]].get("kind")) for pk in picks})
    return {"calls": len(errs), "plans": len(plans), "max": max(errs), "median": float(np.median(errs)),
            "fp64_path_calls": int(sum(pk[3] for pk in picks)), "presets": len(presets),
            "tolerance": 1e-5, "within_tolerance": int(sum(e <= 1e-5 for e in errs))}


def traffic_from_profiles(config, kernels, launches_per_step):
    """HBM bytes per launch of the kernel group `kernels` (one launch of each per
    plan) from the committed rocprofv3 PMC summary of this workload
    (profiles/rNN_<config>_traffic.json by tools/gpu_traffic.sh: separate
    FETCH_SIZE / WRITE_SIZE passes, gfx950 FETCH_SIZE doubled): the sum over the
    group's launches of one execute, per launch of the group."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_%s_traffic.json" % config)))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    ex = d.get("executes")
    hits = [(v["hbm_bytes"], v.get("launches")) for k, v in d.get("kernels", {}).items()
            if k.split(" ")[0] in kernels and "hbm_bytes" in v]
    if not hits or not ex or any(n is None for _, n in hits):
        return None, None
    per_step = sum(b * n for b, n in hits) / ex
    return per_step / max(1, launches_per_step), os.path.relpath(files[-1], ROOT)


def pmc_from_profiles(config, kernel):
    """Issue profile of `kernel` from the newest committed rocprofv3 SQ-counter
    summary of this workload (profiles/rNN_<config>_pmc.json, tools/pmc_summary.py),
    averaged over its launches:
      valu/lds_issue_per_wave  SQ_ACTIVE_INST_VALU / _LDS over SQ_WAVE_CYCLES (both
                               quad-cycles): the share of a wave's life issuing them
      waitcnt_per_wave         SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
      waves_per_simd           ACHIEVED occupancy: SQ_WAVE_CYCLES (quad-cycles summed
                               over waves) / SQ_BUSY_CU_CYCLES (cycles summed over CUs)
                               = mean waves resident per SIMD while the CUs are busy
      valu_busy_per_simd       SQ_ACTIVE_INST_VALU / SQ_BUSY_CU_CYCLES: the share of a
                               SIMD's cycles issuing VALU (waves x issue share)
      mfma_busy_per_simd       SQ_VALU_MFMA_BUSY_CYCLES / (4 SQ_BUSY_CU_CYCLES)
      lds_conflicts_per_instr  SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS (summed over launches)
      lds_conflict_share       SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE: the conflicts' share of
                               the LDS array's busy cycles
      lds_array_busy           SQ_LDS_IDX_ACTIVE / SQ_BUSY_CU_CYCLES
    The busy-cycle ratios need SQ_BUSY_CU_CYCLES in the summary (tools/gpu_pmc_head.sh since
    round 5), the LDS ones its third pass (round 6)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_%s_pmc.json" % config)))
    if not files:
        return None
    d = json.load(open(files[-1]))
    acc = {}
    lds = {}
    for k, v in d.get("kernels", {}).items():
        if k.split(" ")[0] != kernel or not v.get("SQ_WAVE_CYCLES"):
            continue
        for c in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_ANY"):
            if c in v:
                acc.setdefault(c, []).append(v[c] / v["SQ_WAVE_CYCLES"])
        busy = v.get("SQ_BUSY_CU_CYCLES")
        if busy:
            acc.setdefault("waves", []).append(v["SQ_WAVE_CYCLES"] / busy)
            if "SQ_ACTIVE_INST_VALU" in v:
                acc.setdefault("valu_busy", []).append(v["SQ_ACTIVE_INST_VALU"] / busy)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in v:
                acc.setdefault("mfma_busy", []).append(v["SQ_VALU_MFMA_BUSY_CYCLES"] / (4 * busy))
            if "SQ_LDS_IDX_ACTIVE" in v:
                acc.setdefault("lds_busy", []).append(v["SQ_LDS_IDX_ACTIVE"] / busy)
        n = v.get("launches", 1)
        for c in ("SQ_LDS_BANK_CONFLICT", "SQ_INSTS_LDS", "SQ_LDS_IDX_ACTIVE"):
            if c in v:
                lds[c] = lds.get(c, 0.0) + v[c] * n
    if not acc:
        return None
    m = {c: float(np.mean(x)) for c, x in acc.items()}
    conf = lds.get("SQ_LDS_BANK_CONFLICT")
    m["lds_conf_instr"] = conf / lds["SQ_INSTS_LDS"] if conf is not None and lds.get("SQ_INSTS_LDS") else None
    m["lds_conf_share"] = conf / lds["SQ_LDS_IDX_ACTIVE"] if conf is not None and lds.get("SQ_LDS_IDX_ACTIVE") else None
    return {"valu_issue_per_wave": m.get("SQ_ACTIVE_INST_VALU"), "lds_issue_per_wave": m.get("SQ_ACTIVE_INST_LDS"),
            "waitcnt_per_wave": m.get("SQ_WAIT_INST_ANY"), "waves_per_simd": m.get("waves"),
            "valu_busy_per_simd": m.get("valu_busy"), "mfma_busy_per_simd": m.get("mfma_busy"),
            "lds_conflicts_per_instr": m.get("lds_conf_instr"), "lds_conflict_share": m.get("lds_conf_share"),
            "lds_array_busy": m.get("lds_busy"), "source": os.path.relpath(files[-1], ROOT)}


SG_WTASK_BYTES = 128  # sizeof(SgWTask), sg_dev.h


def roofline(st, prof, steps, config, kern):
    """Roofline of one profiled kernel group: achieved = algorithmic bytes per launch
    (SURVEY.md §8d per-unit bytes) / average launch duration (HIP events
    on the launch stream, every kernel alone: profiling serialises the two streams).
    `bound` names the unit whose fraction is the larger: HBM bytes against 8 TB/s, or
    the VALU's work (sine bank: 2 lane-ops per (sample, row, chain) against the packed
    issue peak; STFT: the nominal 5 wl log2 wl flops per transform against the fp32
    peak). `frac` is always the HBM fraction of the algorithmic bytes."""
    ms, n = prof[kern]
    lps = max(1, n // steps)  # launches per step
    sec = ms / 1e3
    desc = 0.0
    if kern == "sg_sine_bank":
        # fp32 epoch waveform write + the amplitude columns it reads (each once) + the 128-B
        # task descriptors of the fp32 class kernels (each read once, by scalar loads)
        desc = SG_WTASK_BYTES * sum(st.get(k, 0) for k in ("tasks_long", "tasks_short", "tasks_tall",
                                                             "tasks_tallp")) / lps
        alg = (4 * st["harm_samples"] + st["harm_amp_bytes"]) / lps + desc
        # Clenshaw: 2 lane-ops per (sample, row, chain) of the tasks on the row recurrence;
        # the wavetable spans' samples (one table read + 3 FMAs each) are not priced here
        valu_ops = 2.0 * (st["harm_terms"] - st.get("tab_terms", 0)) / lps
        vfrac = valu_ops / sec / VALU_PEAK_OPS if sec else 0
        extra = {"valu": {"ops_per_launch": valu_ops, "achieved_ops_s": valu_ops / sec if sec else 0,
                          "peak_ops_s": VALU_PEAK_OPS, "frac": vfrac,
                          "wavetable": {"spans": st.get("tab_spans", 0) / lps,
                                        "samples": st.get("tab_samples", 0) / lps,
                                        "terms_replaced": st.get("tab_terms", 0) / lps}}}
        kernels = ("sg_sine_bank", "sg_sine_bank_pairs", "sg_sine_bank_tall", "sg_sine_bank_tall_pairs",
                   "sg_sine_bank_tab")
        name = " + ".join(kernels)
    else:
        # source / uniforms + envelope columns read, trimmed output written
        alg = st["stft_bytes"] / lps
        fl = st["stft_flops"] / lps
        vfrac = fl / sec / 1e12 / FP32_PEAK_TFLOPS if sec else 0
        extra = {"flops": {"nominal_per_launch": fl, "achieved_tflops": fl / sec / 1e12 if sec else 0,
                           "peak_tflops": FP32_PEAK_TFLOPS, "frac": vfrac}}
        kernels = ("sg_stft_ola", "sg_stft_ola_noise")
        name = "sg_stft_ola + sg_stft_ola_noise"
    achieved = alg / sec / 1e9 if sec > 0 else 0.0
    hfrac = achieved / HBM_PEAK_GBS
    traffic, src = traffic_from_profiles(config, kernels, lps)
    if traffic is not None and desc:
        # FETCH_SIZE counts a 128-B scalar (s_load) descriptor read at its true size, where the
        # gfx950 doubling applies only to vector reads (tools/calib/fetch_calib.hip,
        # profiles/r05o_fetch_calib.json: factor 1.00 for desc128, 0.50 for 4-B and 16-B lanes):
        # the doubled total holds the descriptors twice
        traffic -= desc
    r = {"bound": "valu" if vfrac > hfrac else "hbm", "kernel": name, "achieved": achieved, "peak": HBM_PEAK_GBS,
         "unit": "GB/s", "frac": hfrac, "traffic": traffic, "alg_bytes_per_launch": alg, "avg_launch_ms": ms,
         "launches_timed": n,
         "rocprof_check": (("avg_launch_ms = (TotalDurationNs of %s) / (their Calls)" if kern != "sg_sine_bank" else
                            "avg_launch_ms = (sum of TotalDurationNs of %s) / (Calls of one of them: one launch "
                            "of each class per plan)") % " + ".join(kernels)
                           + " in the SG_OVERLAP=0 kernel-stats summary")}
    if src:
        r["traffic_source"] = src
    if desc:
        r["traffic_correction"] = ("- %.0f B per launch: the task descriptors, which FETCH_SIZE counts once "
                                   "(scalar loads; tools/calib/fetch_calib.hip)" % desc)
    r.update(extra)
    issue = {k: pmc_from_profiles(config, k) for k in kernels}
    issue = {k: v for k, v in issue.items() if v}
    if issue:
        r["issue"] = issue
    if kern == "sg_stft_ola":
        r["binding"] = ("latency at 2 waves/SIMD (221 VGPRs; the LDS array ~0.4 busy, DESIGN.md section 5): radix-29 "
                        "stage on the matrix pipe (MFMA), radix 19 on the VALU, radix 2 fused with the untangle and "
                        "the window; workgroups of equal-length segments; see issue")
    return r


def relaunch(args):
    """--gpus N without a launcher: start N ranks under torch.distributed.run as a
    child process (no GPU call has happened in this process) and return its status."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def node_bench(args):
    """The whole-node path behind the C ABI (sg_node_plan_batch + sg_node_execute_to_host[_f32],
    soundgen_batch()'s path from R): one process, every device of --node-devices, the batch
    sharded by calls inside the library (LPT), each shard pipelined by chunk (the D2H of a
    chunk beside the compute of the later ones). Timed: sg_node_execute_to_host entry to
    every call's samples in the caller's host buffer at its whole-batch offset (a plain
    numpy array: pageable memory, as a C or R caller holds it)."""
    from soundgen_beta_amd import batch, native
    devs = [int(x) for x in args.node_devices.split(",") if x.strip()]
    make, n_default, desc = CONFIGS[args.config]
    n_calls = args.calls or n_default
    calls = make(n_calls)
    node = native.Node(devs)
    t_plan = time.perf_counter()
    plan = batch.NodePlan(calls, node)
    t_plan = time.perf_counter() - t_plan
    native.lib().sg_host_cache_trim()
    dtype = np.float64 if args.node_f64 else np.float32
    host = np.empty(max(plan.total, 1), dtype=dtype)
    L = native.lib()
    if args.node_f64:
        fn, ptr = L.sg_node_execute_to_host, host.ctypes.data_as(C.POINTER(C.c_double))
    else:
        fn, ptr = L.sg_node_execute_to_host_f32, host.ctypes.data_as(C.POINTER(C.c_float))

    def step():
        node.check(fn(node.ptr, plan.ptr, ptr))
    for _ in range(args.warmup):
        step()
    t = time.perf_counter()
    for _ in range(args.steps):
        step()
    dt = time.perf_counter() - t
    samples = int(plan.lengths[plan.status == 0].sum())
    failed = int((plan.status != 0).sum())
    rms = None
    if args.rms_calls > 0:  # the timed outputs against the oracle, calls spread over the batch
        from concurrent.futures import ThreadPoolExecutor
        from oracle import oracle as O
        O.lib()
        ok = np.nonzero(plan.status == 0)[0]
        pick = ok[np.linspace(0, len(ok) - 1, min(args.rms_calls, len(ok))).round().astype(int)] if len(ok) else []

        def one(i):
            ref = oracle_call(O, calls[int(i)])
            y = host[plan.offsets[i]:plan.offsets[i] + plan.lengths[i]].astype(np.float64)
            return float(np.sqrt(np.mean((y - ref) ** 2))) if len(ref) == len(y) else float("inf")
        with ThreadPoolExecutor(host_cores()) as ex:
            errs = list(ex.map(one, pick))
        rms = {"calls": len(errs), "max": max(errs) if errs else None, "tolerance": 1e-5,
               "within_tolerance": int(sum(e <= 1e-5 for e in errs))}
    res = {"metric": METRIC, "value": samples * args.steps / dt, "unit": "samples/s", "n_gpus": len(devs),
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
           "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "fp32 (fp64 phase)",
           "data": "synthetic (PCG64 seed %d; random draws injected)" % SEED,
           "config": {"workload": desc % n_calls, "calls": n_calls, "samples": samples, "failed_calls": failed,
                      "parallelism": "node: one process over devices %s (sg_node, LPT shards)" % devs,
                      "chunks_per_shard": [plan.chunks(k) for k in range(len(devs))]},
           "path": "sg_node_plan_batch + sg_node_execute_to_host%s (the C-ABI whole-node path; soundgen_batch() "
                   "from R)" % ("" if args.node_f64 else "_f32"),
           "timing": "sg_node_execute_to_host entry to every call's samples in the caller's pageable %s host "
                     "buffer at its whole-batch offset" % ("float64" if args.node_f64 else "float32"),
           "plan_s": t_plan, "value_incl_planning": samples / (t_plan + dt / args.steps),
           "rms_error_vs_oracle": rms["max"] if rms else None, "rms_check": rms}
    print(json.dumps(res), flush=True)
    plan.close()
    node.close()
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c5", choices=sorted(CONFIGS))
    ap.add_argument("--calls", type=int, default=0, help="calls in the whole batch (default: the config's)")
    ap.add_argument("--plan-chunk", type=int, default=16384,
                    help="calls per plan (each uploaded, then its host copy freed)")
    ap.add_argument("--no-plan-ramp", action="store_true",
                    help="equal plan chunks (default: a first chunk of plan-chunk / 4 calls, a short pipeline fill)")
    ap.add_argument("--no-d2h", action="store_true",
                    help="profiling runs only: the timed steps leave the outputs in HBM (no copy kernels beside them)")
    ap.add_argument("--device-steps", type=int, default=5,
                    help="extra steps timed with the outputs left in HBM (value_device_resident; 0: skip)")
    ap.add_argument("--cpu-budget", type=float, default=16.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true",
                    help="N>1: skip the timed gather of every rank's packed output to rank 0 after the timed steps")
    ap.add_argument("--rms-calls", type=int, default=66,
                    help="calls checked against the oracle after timing, spread over every plan")
    ap.add_argument("--node", action="store_true",
                    help="the whole-node C-ABI path R reaches (sg_node_*): one process, --node-devices, "
                         "the batch planned once and executed into a caller's (pageable) host buffer")
    ap.add_argument("--node-devices", default="0", help="--node: comma-separated device ordinals")
    ap.add_argument("--node-f64", action="store_true", help="--node: into doubles (R's numeric vectors)")
    args = ap.parse_args()
    if args.node:
        return node_bench(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch(args))

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)

    from soundgen_beta_amd import batch, native
    from soundgen_beta_amd import dist as sharding
    make, n_default, desc = CONFIGS[args.config]
    n_calls = args.calls or n_default
    t_gen = time.perf_counter()
    calls = make(n_calls)  # the same batch on every rank
    t_gen = time.perf_counter() - t_gen
    if world > 1:
        idx, mine, _ = sharding.shard(calls, rank, world)
    else:
        idx, mine = np.arange(n_calls), calls
    ctx = native.Context(local)
    plans = []  # (plan, output base, the calls' indices in the batch)
    t_plan = time.perf_counter()
    base = 0
    failed = 0
    first_msg = None
    # chunk k + 1 plans on the host while chunk k uploads (batch.plan_uploaded)
    plan_stages = []
    sizes = batch.chunk_sizes(len(mine), args.plan_chunk, ramp=not args.no_plan_ramp)
    for p, a in batch.plan_uploaded(mine, ctx, sizes, plan_stages):
        bad = np.nonzero(p.status)[0]
        failed += len(bad)
        if len(bad) and first_msg is None:
            first_msg = p.message(int(bad[0]))
        plans.append((p, base, idx[a:a + p.n]))
        base += (p.total + 63) // 64 * 64
        if rank == 0:
            print("bench: planned + uploaded %d/%d calls (%.1f s)" % (a + p.n, len(mine),
                                                                      time.perf_counter() - t_plan), file=sys.stderr)
    t_plan = time.perf_counter() - t_plan
    native.lib().sg_host_cache_trim()  # planning is over: give the planner's cached host blocks back
    if failed:
        print("bench: %d of %d calls not synthesized: %s" % (failed, len(mine), first_msg), file=sys.stderr)
    out = torch.empty(max(base, 1), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream

    def step():
        for p, b, _ in plans:
            p.execute(out.data_ptr() + 4 * b, sptr)

    # the metric's timing: from sg_execute entry to waveforms resident
    # in host memory. Every plan's outputs are copied into pinned host memory on a
    # second stream while the following plans compute; plan c of the next step
    # waits only for the copy of its own region.
    try:
        host = torch.empty(max(base, 1), dtype=torch.float32, pin_memory=True)
        pinned = True
    except RuntimeError:
        host = torch.empty(max(base, 1), dtype=torch.float32)
        pinned = False
    cstream = torch.cuda.Stream(dev)
    ends = [b + (p.total + 63) // 64 * 64 for p, b, _ in plans]
    copied = [None] * len(plans)

    def step_to_host():
        for i, ((p, b, _), e) in enumerate(zip(plans, ends)):
            if copied[i] is not None:
                stream.wait_event(copied[i])  # plan i's region is free again
            p.execute(out.data_ptr() + 4 * b, sptr)
            done = torch.cuda.Event()
            done.record(stream)
            cstream.wait_event(done)
            with torch.cuda.stream(cstream):
                host[b:e].copy_(out[b:e], non_blocking=pinned)
            copied[i] = torch.cuda.Event()
            copied[i].record(cstream)

    def timed(fn, k):
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        return time.perf_counter() - t

    main_step = step if args.no_d2h else step_to_host
    for _ in range(args.warmup):
        main_step()
    torch.cuda.synchronize(dev)
    dt = timed(main_step, args.steps)  # the headline: host-resident
    # the same steps with the outputs left in HBM (no D2H copy)
    dt_dev = timed(step, args.device_steps) if args.device_steps > 0 else None
    L = native.lib()
    # per-kernel HIP events (roofline) over the same number of extra steps, outside the
    # timed region: with profiling on, the harmonic chain and the noise phase run one
    # after the other, so each launch's duration is its own, not shared with a
    # concurrent kernel
    L.sg_set_profiling(ctx.ptr, 1)
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    L.sg_set_profiling(ctx.ptr, 0)
    prof = {}
    for kid, name in ((0, "sg_sine_bank"), (1, "sg_stft_ola")):
        ms, n = C.c_double(), C.c_int64()
        native.check(L.sg_profile_read_kernel(ctx.ptr, kid, C.byref(ms), C.byref(n)), ctx.ptr)
        prof[name] = (ms.value, n.value)
    del host

    samples_rank = int(sum(int(p.lengths.sum()) for p, _, _ in plans))  # synthesized samples (padding excluded)
    vals = [dt, t_plan, float(dt_dev or 0.0)]
    if dist:
        t = torch.tensor(vals, device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        vals = [float(x) for x in t.tolist()]
        s = torch.tensor([samples_rank, failed], device=dev, dtype=torch.float64)
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        samples_all, failed_all = float(s[0].item()), int(s[1].item())
    else:
        samples_all, failed_all = float(samples_rank), failed
    dt, t_plan_max, dt_dev = vals[0], vals[1], (vals[2] if args.device_steps > 0 else None)
    value = samples_all * args.steps / dt

    gather_ms = gather_error = None
    if dist and not args.no_gather:
        # SURVEY §8e exchange step, after the timed steps: every peer sends its packed
        # output and (offset, length) table to rank 0 (dist.gather_packed: one RCCL
        # point-to-point transfer per peer, each on its own xGMI link). Not part of
        # `value` (every rank's outputs already reached its own pinned host memory
        # over its own PCIe link); gathering to rank 0 and copying from there would
        # put the whole node behind one link.
        offs = np.concatenate([b + p.offsets for p, b, _ in plans]) if plans else np.zeros(0, np.int64)
        lens = np.concatenate([np.where(p.status == 0, p.lengths, -1) for p, _, _ in plans]) if plans else \
            np.zeros(0, np.int64)
        try:
            got, gather_ms = sharding.gather_timed(out[:max(base, 1)], offs, lens, calls, rank, world)
            if rank == 0:  # the gathered batch is complete and in call order
                gathered_samples = sum(int(g.numel()) for g in got if not isinstance(g, Exception))
                if len(got) != n_calls or gathered_samples != int(samples_all):
                    gather_error = "gathered %d calls / %d samples, expected %d / %d" % (
                        len(got), gathered_samples, n_calls, int(samples_all))
            del got
        except Exception as e:  # the measured value stands; the exchange's failure is reported beside it
            gather_error = "%s: %s" % (type(e).__name__, e)
            gather_ms = None

    if rank == 0:
        st = {}
        for p, _, _ in plans:
            for k, v in p.stats().items():
                st[k] = st.get(k, 0) + v
            # task descriptors per class (128 B each, read once by their class kernel)
            for k, v in zip(("tasks_long", "tasks_short", "tasks_tall", "tasks_tallp", "tasks_hp"), p.sine_tasks()):
                st[k] = st.get(k, 0) + v
            tabs, tab_samples, tab_terms = p.table_stats()  # wavetable spans (no row recurrence)
            st["tab_spans"] = st.get("tab_spans", 0) + tabs
            st["tab_samples"] = st.get("tab_samples", 0) + tab_samples
            st["tab_terms"] = st.get("tab_terms", 0) + tab_terms
        tot = {k: v[0] * v[1] for k, v in prof.items()}
        dom = max(tot, key=tot.get) if any(tot.values()) else "sg_sine_bank"
        roof = roofline(st, prof, args.steps, args.config, dom)
        other = [k for k in prof if k != dom and prof[k][1] > 0]
        rms = rms_check(plans, out, calls, args.rms_calls)
        res = {
            "metric": METRIC, "value": value, "unit": "samples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "fp32 (fp64 phase)",
            "data": "synthetic (PCG64 seed %d; random draws injected)" % SEED,
            "config": {"workload": desc % n_calls, "calls": n_calls, "calls_rank0": len(mine),
                       "samples": int(samples_all), "sampling_rate": 44100,
                       "parallelism": "dp%d (one batch split by calls, LPT)" % world,
                       "plans_per_rank": len(plans), "failed_calls": failed_all},
            "timing": ("outputs left in HBM (--no-d2h profiling run)" if args.no_d2h else
                       "sg_execute entry to waveforms resident in pinned host memory (SURVEY 8d)"),
            "value_device_resident": (samples_all * args.device_steps / dt_dev) if dt_dev else None,
            "ms_per_step_device_resident": (dt_dev / args.device_steps * 1e3) if dt_dev else None,
            "plan_s": t_plan_max, "calls_gen_s": t_gen,
            "plan_stages": [{k: (round(v, 3) if isinstance(v, float) else v) for k, v in t.items()} for t in plan_stages],
            "value_incl_planning": samples_all / (t_plan_max + dt / args.steps),
            "rms_error_vs_oracle": rms["max"] if rms else None,
            "rms_check": rms,
            "roofline": roof,
        }
        for k in other:  # the other profiled kernel group (C5: the sine-bank classes)
            res["roofline_" + ("sine_bank" if k == "sg_sine_bank" else "stft_ola")] = \
                roofline(st, prof, args.steps, args.config, k)
        if dist and not args.no_gather:
            res["gather_ms"] = gather_ms
            res["gather"] = ("every rank's packed outputs sent to rank 0 over RCCL point-to-point after the timed "
                             "steps (dist.gather_timed); not part of value (DESIGN.md §7)")
            if gather_error:
                res["gather_error"] = gather_error
        if not args.no_cpu_baseline and world == 1:  # the CPU leg runs at N=1 only
            res["cpu_baseline"] = cpu_baseline(calls, args.cpu_budget)
        print(json.dumps(res), flush=True)
    for p, _, _ in plans:
        p.close()
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
