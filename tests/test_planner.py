"""CPU: the product library's host planner (libsoundgen_hip.so, no GPU needed)
does all integer bookkeeping of generateHarmonics() — glottal cycles, gcLen,
subharmonic epochs, kept rows, crossFade zero-crossing trims, fades — and
must agree with the oracle sample-for-sample (bit-exact lengths)."""
import numpy as np
import pytest

from soundgen_beta_amd import batch

RNG = np.random.default_rng(20261015)
NORMALS = RNG.standard_normal(20000)
UNIFORMS = RNG.uniform(size=20000)

C2 = dict(samplingRate=44100, temperature=0, nonlinBalance=0, rolloff=-12, rolloffOct=-12, rolloffKHz=-6,
          pitchFloor=50)
t3500 = np.linspace(0, 1, 3500)
CASES = [
    ("c2_80", np.full(3500, 80.0), C2),
    ("c2_400", np.full(3500, 400.0), C2),
    ("c2_237", np.full(3500, 237.0), C2),
    ("sweep", 150 + 100 * t3500, C2),
    ("vibrato", np.full(3500, 220.0), dict(C2, vibratoDep=1, vibratoFreq=6)),
    ("sr16k", np.full(2000, 140.0), dict(samplingRate=16000)),
    ("high_f0", np.full(700, 1000.0), C2),
    ("near_ceiling", np.full(500, 3400.0), C2),
    ("parab", np.full(3500, 300.0), dict(C2, rolloffParab=-10, rolloffParabHarm=5)),
    ("subharm", np.full(7000, 300.0), dict(C2, nonlinBalance=100, subFreq=100, subDep=80)),
    ("subharm_contour", 250 + 200 * t3500, dict(C2, nonlinBalance=100, subFreq=150, subDep=100,
                                                shortestEpoch=50)),
    ("jitter_shimmer", 180 + 40 * t3500, dict(C2, nonlinBalance=100, jitterDep=1.5, jitterLen=5,
                                              shimmerDep=10)),
    ("temp", np.full(3500, 200.0), dict(C2, temperature=0.05, nonlinBalance=100, subFreq=120, subDep=60,
                                        jitterDep=1, shimmerDep=8)),
    ("temp_balance50", np.full(3500, 200.0), dict(C2, temperature=0.1, nonlinBalance=50, jitterDep=1)),
]


@pytest.mark.parametrize("name,pitch,params", CASES, ids=[c[0] for c in CASES])
def test_plan_lengths_match_oracle(oracle, name, pitch, params):
    calls = [{"kind": "harmonics", "pitch": pitch, "params": params, "normals": NORMALS, "uniforms": UNIFORMS}]
    plan = batch.Plan(calls, None)
    assert plan.status[0] == 0, plan.message(0)
    ref = oracle.generate_harmonics(pitch, normals=NORMALS, uniforms=UNIFORMS, **params)
    assert plan.lengths[0] == len(ref)


def test_ampl_anchors_length(oracle):
    pitch = np.full(3500, 180.0)
    aa = {"time": [0, 1], "value": [110, 60]}  # 2 anchors: linear (3-10 would need loess)
    plan = batch.Plan([{"kind": "harmonics", "pitch": pitch, "params": C2, "amplAnchors": aa}], None)
    ref = oracle.generate_harmonics(pitch, amplAnchors=aa, **C2)
    assert plan.status[0] == 0 and plan.lengths[0] == len(ref)


def test_batch_offsets_and_failed_slot():
    good = {"kind": "harmonics", "pitch": np.full(3500, 150.0), "params": C2}
    bad = {"kind": "harmonics", "pitch": np.full(1, 150.0), "params": C2}  # too short: R errors
    plan = batch.Plan([good, bad, good], None)
    assert list(plan.status) == [0, -2, 0]
    assert plan.lengths[1] == 0
    assert plan.lengths[0] == plan.lengths[2]
    # 256-B aligned slots
    assert all(o % 64 == 0 for o in plan.offsets)
    assert plan.offsets[2] >= plan.offsets[0] + plan.lengths[0]


def test_random_stream_exhaustion_is_an_error():
    call = {"kind": "harmonics", "pitch": np.full(3500, 200.0),
            "params": dict(C2, temperature=0.05, nonlinBalance=100, jitterDep=1), "normals": NORMALS[:3]}
    plan = batch.Plan([call], None)
    assert plan.status[0] == -3  # SG_E_RANDOM


def test_plan_stats_and_device_bytes():
    calls = [{"kind": "harmonics", "pitch": np.full(3500, f), "params": C2} for f in (90.0, 210.0, 390.0)]
    plan = batch.Plan(calls, None)
    st = plan.stats()
    assert st["harm_samples"] >= sum(plan.lengths)
    assert st["harm_terms"] >= st["harm_samples"]
    assert plan.device_bytes() > 4 * st["harm_samples"]


def test_rng_callbacks_follow_the_same_draw_order(oracle):
    """With draws from callbacks (how the R shim binds norm_rand/unif_rand/
    rgamma), planner and oracle consume identical sequences."""
    p = 200 + 60 * t3500
    prm = dict(C2, temperature=0.1, nonlinBalance=100, subFreq=120, subDep=60, jitterDep=1, shimmerDep=8)
    plan = batch.Plan([{"kind": "harmonics", "pitch": p, "params": prm, "rng": np.random.default_rng(5)}], None)
    ref = oracle.generate_harmonics(p, rng=np.random.default_rng(5), **prm)
    assert plan.status[0] == 0 and plan.lengths[0] == len(ref)


def _mixed_calls(n5=96):
    import bench
    calls = bench.c5_calls(n5) + bench.c4_calls(8) + bench.c2_calls(8)
    bad = {"kind": "harmonics", "pitch": np.full(1, 150.0), "params": C2}  # refused slot in the middle
    return calls[:40] + [bad] + calls[40:]


def test_parallel_planning_equals_serial(monkeypatch):
    """sg_plan_batch plans chunks of calls on host threads and concatenates them
    (sg_api.cpp merge_parts); lengths, offsets, statuses and kernel work must be
    exactly those of serial planning."""
    calls = _mixed_calls()
    monkeypatch.setenv("SG_PLAN_THREADS", "1")
    p1 = batch.Plan(calls, None)
    monkeypatch.setenv("SG_PLAN_THREADS", "7")
    p7 = batch.Plan(calls, None)
    assert (p1.status == p7.status).all() and p1.status[40] == -2
    assert (p1.lengths == p7.lengths).all() and (p1.offsets == p7.offsets).all()
    assert p1.total == p7.total
    s1, s7 = p1.stats(), p7.stats()
    for k in ("harm_samples", "harm_terms", "harm_amp_bytes", "fft_frames", "stft_samples", "stft_bytes"):
        assert s1[k] == s7[k], k


def test_fast_zero_crossing_search_equals_exact(tmp_path):
    """The crossFade zero-crossing search evaluates the epoch waveform by Clenshaw
    with an error bound and falls back to R's row-by-row sum near zero
    (sg_plan_harm.cpp HostEpoch::Wsign); every planned length and offset equals
    the exact-only planner's (SG_XFADE_EXACT)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys, numpy as np; sys.path.insert(0, %r); import bench; from soundgen_beta_amd import batch; "
            "p = batch.Plan(bench.c5_calls(384) + bench.c4_calls(48)); np.save(sys.argv[1], np.stack([p.lengths, p.offsets]))"
            % root)
    outs = []
    for exact in (False, True):
        env = dict(os.environ)
        env.pop("SG_XFADE_EXACT", None)
        if exact:
            env["SG_XFADE_EXACT"] = "1"
        f = str(tmp_path / ("x%d.npy" % exact))
        subprocess.run([sys.executable, "-c", code, f], check=True, env=env, timeout=600)
        outs.append(np.load(f))
    assert np.array_equal(outs[0], outs[1])


def _bench():
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    return bench


def test_precision_path_flags_ill_conditioned_presets():
    """The planner's conditioning estimate (filter_conditioning,
    sg_plan_soundgen.cpp) sends Misc$Cow's bouts (fp32 round-off through its
    envelope reached 1-3e-5 RMS) to the fp64 filter path and no other preset of
    the C5 sample; lengths and offsets do not depend on the path."""
    import os
    bench = _bench()
    calls = bench.c5_calls(400)
    plan = batch.Plan(calls, None)
    assert (plan.status == 0).all()
    hp, frames, tasks = plan.precision()
    presets = np.array([c["preset"] for c in calls])
    assert hp[presets == "Misc$Cow"].min() >= 1
    flagged = set(presets[hp > 0])
    assert flagged <= {"Misc$Cow", "M1$Sigh", "Misc$Elephant"}, flagged
    assert frames > 0 and tasks > 0
    from soundgen_beta_amd import native
    L = native.lib()
    assert L.sg_set_fp64_policy(0, native.HP_RHO_DEFAULT) == 0
    try:
        p0 = batch.Plan(calls, None)
        h0, f0, t0 = p0.precision()
        assert h0.sum() == 0 and f0 == 0 and t0 == 0
        assert np.array_equal(p0.lengths, plan.lengths) and np.array_equal(p0.offsets, plan.offsets)
        assert L.sg_set_fp64_policy(2, native.HP_RHO_DEFAULT) == 0
        p2 = batch.Plan(calls, None)
        h2, f2, t2 = p2.precision()
        assert (h2 >= hp).all() and f2 >= frames and t2 > tasks
        assert np.array_equal(p2.lengths, plan.lengths) and np.array_equal(p2.offsets, plan.offsets)
        assert L.sg_set_fp64_policy(3, native.HP_RHO_DEFAULT) != 0
    finally:
        L.sg_set_fp64_policy(1, native.HP_RHO_DEFAULT)


def _decode_args(s):
    """Every field of an sg_soundgen_args, pointers followed to their values."""
    import ctypes as C

    from soundgen_beta_amd import _abi
    out = []
    for name, t in _abi.sg_soundgen_args._fields_:
        v = getattr(s, name)
        if t is _abi.sg_anchors:
            out.append((v.n, [v.time[i] for i in range(v.n)], [v.value[i] for i in range(v.n)]))
        elif t is _abi.sg_formants:
            if v.n_formants == 0:
                out.append((0, v.f1_index))
                continue
            npnt = [v.n_points[i] for i in range(v.n_formants)]
            out.append((v.n_formants, v.f1_index, npnt,
                        [[getattr(v, k)[i] for i in range(sum(npnt))] for k in ("time", "freq", "amp", "width")]))
        elif t is C.c_double:
            out.append(np.float64(v).tobytes())  # NaN-safe
        elif name == "tempEffects":
            out.append(np.asarray(list(v)).tobytes())
        else:
            out.append(v)
    return out


def test_bulk_marshalling_equals_per_call_fill():
    """batch.Marshalled's bulk writer (rargs.ArgsWriter + the descriptor view)
    fills the same argument values, draws and descriptors as the per-call
    fill_soundgen_args, on a mixed batch: C3/C4/C5 calls, NA and numeric anchors,
    vowel strings, tempEffects, harmonics calls and draw callbacks."""
    import ctypes as C

    import bench
    from soundgen_beta_amd import rargs
    rng = np.random.default_rng(3)
    calls = bench.c5_calls(300)[::3] + bench.c3_calls(12) + bench.c4_calls(6)
    calls += [{"kind": "soundgen", "args": {"pitchAnchors": [120, 180, 90], "noiseAnchors": None,
                                            "tempEffects": {"formDrift": 0.5}, "formants": "aoi",
                                            "amplAnchors": {"time": 0, "value": 50}}},
              {"kind": "harmonics", "pitch": np.full(300, 150.0), "params": {"samplingRate": 44100}},
              {"kind": "soundgen", "args": {"sylLen": 100, "temperature": 0.1}, "rng": rng},
              {"kind": "soundgen", "args": {"sylLen": 120, "pitchAnchors": {"time": [0, 1], "value": [200, 300]}},
               "normals": [0.1, -0.2], "uniforms": np.zeros(0)}]
    m = batch.Marshalled(calls)
    h = rargs.Holder()
    for i, c in enumerate(calls):
        d = m.descs[i]
        if c.get("kind") == "harmonics":
            assert d.kind == 1
            continue
        assert d.kind == 0
        assert _decode_args(d.args.contents) == _decode_args(rargs.fill_soundgen_args(h, c.get("args", {})))
        for key, p, n in (("normals", d.random.normals, d.random.n_normals),
                          ("uniforms", d.random.uniforms, d.random.n_uniforms)):
            x = c.get(key)
            if x is None:
                assert n == 0
                continue
            x = np.asarray(x, dtype=np.float64)
            assert n == len(x)
            if n:
                assert np.array_equal(np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_double)), (n,)), x)


def test_uniform_gather_plans_the_same_calls():
    """With the noise uniforms gathered at upload (sg_set_uniform_gather(1)) the
    plan's lengths, offsets, status and kernel work equal the per-item copy's
    (the GPU test compares the synthesized bytes)."""
    import bench
    from soundgen_beta_amd import native
    L = native.lib()
    calls = bench.c5_calls(240) + bench.c3_calls(6)
    res = []
    for on in (0, 1):
        assert L.sg_set_uniform_gather(on) == 0
        try:
            p = batch.Plan(calls, None)
            res.append((p.lengths.copy(), p.offsets.copy(), p.status.copy(), p.stats()))
            p.close()
        finally:
            L.sg_set_uniform_gather(1)
    (l0, o0, s0, st0), (l1, o1, s1, st1) = res
    assert np.array_equal(l0, l1) and np.array_equal(o0, o1) and np.array_equal(s0, s1)
    assert st0 == st1
    assert L.sg_set_uniform_gather(2) != 0


def test_host_cache_trim_between_plans():
    """sg_host_cache_trim releases the planner's cached host blocks; the next plan
    refills the cache and plans the same batch."""
    import time

    import bench
    from soundgen_beta_amd import native
    L = native.lib()
    calls = bench.c5_calls(1200)
    p = batch.Plan(calls, None)
    want = (p.lengths.copy(), p.offsets.copy(), p.stats())
    p.close()
    released = 0
    for _ in range(40):  # large host arrays are freed on a detached thread after close
        released += L.sg_host_cache_trim()
        if released:
            break
        time.sleep(0.05)
    assert released >= 0 and L.sg_host_cache_trim() >= 0
    q = batch.Plan(calls, None)
    assert np.array_equal(q.lengths, want[0]) and np.array_equal(q.offsets, want[1]) and q.stats() == want[2]
    q.close()
