"""GPU parity: the HIP path (libsoundgen_hip.so through the C-ABI) vs the CPU
oracle on the same inputs and injected random draws.
Tolerance: RMS <= 1e-5 on the normalised waveform (BASELINE.json north star);
sample counts bit-exact."""
import numpy as np
import pytest

from test_planner import CASES, NORMALS, UNIFORMS

pytestmark = pytest.mark.gpu

C2 = dict(samplingRate=44100, temperature=0, nonlinBalance=0, rolloff=-12, rolloffOct=-12, rolloffKHz=-6,
          pitchFloor=50)
TOL = 1e-5


def _rms(a, b):
    return float(np.sqrt(np.mean((np.asarray(a, np.float64) - b) ** 2)))


def test_c2_tones_batch(oracle):
    from soundgen_beta_amd import batch
    rng = np.random.Generator(np.random.PCG64(20261015))
    f0 = np.exp(rng.uniform(np.log(80), np.log(400), 24))
    calls = [{"kind": "harmonics", "pitch": np.full(3500, f), "params": C2} for f in f0]
    outs = batch.synthesize(calls)
    for c, y in zip(calls, outs):
        ref = oracle.generate_harmonics(c["pitch"], **c["params"])
        assert len(y) == len(ref)
        assert _rms(y, ref) <= TOL


def test_sine_table_path_vs_recurrence(oracle):
    """Static tones (the wavetable path, sg_sine_bank_tab) against the same
    plan on the row recurrence (sg_set_sine_table(0)) and the oracle, over f0
    from 55 Hz (many rows) to 1.5 kHz, flat and steep rolloffs, 16 and 44.1 kHz."""
    from soundgen_beta_amd import batch, native
    L = native.lib()
    calls = []
    for f in (55.0, 80.0, 123.4, 250.0, 399.0, 1500.0):
        for roll in (-12, -3):
            prm = dict(C2, rolloff=roll, rolloffOct=0 if roll == -3 else C2["rolloffOct"])
            calls.append({"kind": "harmonics", "pitch": np.full(3500, f), "params": prm})
    calls.append({"kind": "harmonics", "pitch": np.full(1500, 190.0), "params": dict(C2, samplingRate=16000)})
    # 2 s: 88 tasks, more than one table job (SG_TAB_TASKS), so the span goes through W
    calls.append({"kind": "harmonics", "pitch": np.full(7000, 201.0), "params": C2})
    outs = {}
    try:
        for on in (1, 0):
            assert L.sg_set_sine_table(on) == 0
            plan = batch.Plan(calls, native.default_context(0))
            plan.upload()
            tabs, samples, _ = plan.table_stats()
            assert (tabs >= 8 and samples > 0.5 * plan.total) if on else tabs == 0  # 55 / 80 Hz at -3 dB: tall rows
            outs[on] = batch.synthesize(calls)
    finally:
        L.sg_set_sine_table(1)
    rows = []
    for c, y1, y0 in zip(calls, outs[1], outs[0]):
        assert len(y1) == len(y0)
        ref = oracle.generate_harmonics(c["pitch"], **c["params"])
        e1, e0 = np.asarray(y1, np.float64) - ref, np.asarray(y0, np.float64) - ref
        rows.append((np.sqrt(np.mean(e1 ** 2)), np.sqrt(np.mean(e0 ** 2)), np.abs(e1).max(), np.abs(e0).max()))
    for r in rows:
        print("table rms %.3g max %.3g | recurrence rms %.3g max %.3g" % (r[0], r[2], r[1], r[3]))
    for r in rows:  # the table within the tolerance, and no worse than the fp32 recurrence by more than 1e-6
        assert r[0] <= TOL and r[2] <= r[3] + 1e-6, r


def test_sine_table_direct_output_equals_w_path():
    """Whole-syllable table spans write their final samples themselves
    (SG_TAB_DIRECT, no W round trip, no sg_harm_copy pass; the max from a full
    evaluation pass): bit-identical to the same spans through W + sg_syl_max +
    sg_harm_copy (SG_TAB_DIRECT=0), including attack/release fades and a batch
    mixing direct and non-direct syllables."""
    import os
    import torch
    from soundgen_beta_amd import batch, native
    # 441 Hz and 2205 Hz: phase grids of 100 and 20 points per cycle (f0 / fs = 1 / 100, 1 / 20),
    # coarser than the table: the max pass evaluates every sample on that grid
    calls = [{"kind": "harmonics", "pitch": np.full(n, f), "params": dict(C2, attackLen=a)}
             for f, n, a in ((97.0, 3500, 50), (210.0, 1200, 10), (333.3, 5000, 0), (150.0, 800, 300),
                             (441.0, 2000, 50), (2205.0, 2000, 50), (1000.0, 3000, 20), (201.0, 7000, 50))]
    calls.append({"kind": "harmonics", "pitch": np.linspace(120, 260, 2000), "params": C2})  # not a static span
    outs = []
    for direct in ("1", "0"):
        os.environ["SG_TAB_DIRECT"] = direct
        try:
            plan = batch.Plan(calls, native.default_context(0))
            plan.upload()
            assert plan.table_stats()[0] >= 4
            out = torch.full((plan.total,), float("nan"), dtype=torch.float32, device="cuda")
            plan.execute(out.data_ptr(), torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            outs.append((out.cpu().numpy(), plan.offsets.copy(), plan.lengths.copy()))
        finally:
            os.environ.pop("SG_TAB_DIRECT", None)
    (a, oa, la), (b, ob, lb) = outs
    assert np.array_equal(oa, ob) and np.array_equal(la, lb)
    for o, n in zip(oa, la):
        assert np.array_equal(a[o:o + n], b[o:o + n]), o
        assert np.isfinite(a[o:o + n]).all()


def test_sine_table_direct_into_filtered_bout(oracle):
    """A direct table syllable of a FILTERED bout writes into the pre-filter
    scratch fs (obase = fs), on the harmonic stream, before the noise copies and
    the join: soundgen() calls with a static pitch, temperature 0 and formants,
    some with breathing noise in the same bout. Byte-equal with SG_TAB_DIRECT=1
    and =0, and within the tolerance of the oracle."""
    import os
    import torch
    from soundgen_beta_amd import batch, native
    from test_spectral_cpu import N, U
    base = dict(samplingRate=44100, temperature=0, addSilence=0, formants="a", attackLen=30)
    cases = [dict(base, sylLen=300, pitchAnchors=[180, 180], noiseAnchors=None),
             dict(base, sylLen=450, pitchAnchors=[123.4, 123.4], noiseAnchors=None, formants="o"),
             dict(base, sylLen=350, pitchAnchors=[220, 220],
                  noiseAnchors={"time": [0, 350], "value": [-25, -25]}),
             dict(base, sylLen=250, pitchAnchors=[150, 150], noiseAnchors=None, repeatBout=2, pauseLen=40)]
    calls = [{"kind": "soundgen", "args": a, "normals": N, "uniforms": U} for a in cases]
    outs = []
    for direct in ("1", "0"):
        os.environ["SG_TAB_DIRECT"] = direct
        try:
            plan = batch.Plan(calls, native.default_context(0))
            plan.upload()
            assert plan.table_stats()[0] >= len(cases)
            out = torch.full((plan.total,), float("nan"), dtype=torch.float32, device="cuda")
            plan.execute(out.data_ptr(), torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            outs.append((out.cpu().numpy(), plan.offsets.copy(), plan.lengths.copy()))
        finally:
            os.environ.pop("SG_TAB_DIRECT", None)
    (a, oa, la), (b, ob, lb) = outs
    assert np.array_equal(oa, ob) and np.array_equal(la, lb)
    for args, o, n in zip(cases, oa, la):
        assert np.array_equal(a[o:o + n], b[o:o + n]), args
        ref = oracle.soundgen(normals=N, uniforms=U, **args)
        assert n == len(ref)
        assert _rms(a[o:o + n], ref) <= TOL, args


def test_planner_cases_one_batch(oracle):
    """Every planner case (vibrato, subharmonic epochs + crossfades, jitter,
    shimmer, temperature random walks, 16 kHz, near-ceiling f0) in ONE batch."""
    from soundgen_beta_amd import batch
    calls = [{"kind": "harmonics", "pitch": p, "params": prm, "normals": NORMALS, "uniforms": UNIFORMS}
             for _, p, prm in CASES]
    outs = batch.synthesize(calls)
    worst = 0.0
    for (name, p, prm), y in zip(CASES, outs):
        ref = oracle.generate_harmonics(p, normals=NORMALS, uniforms=UNIFORMS, **prm)
        assert len(y) == len(ref), name
        r = _rms(y, ref)
        worst = max(worst, r)
        assert r <= TOL, (name, r)
    print("worst rms", worst)


def test_ampl_anchors_and_contours(oracle):
    from soundgen_beta_amd import batch
    t = np.linspace(0, 1, 3500)
    calls = [
        {"kind": "harmonics", "pitch": np.full(3500, 180.0), "params": C2,
         "amplAnchors": {"time": [0, 1], "value": [110, 60]}},
        {"kind": "harmonics", "pitch": 300 - 120 * t ** 2, "params": C2},
        {"kind": "harmonics", "pitch": 220 * 2 ** (0.5 * np.sin(2 * np.pi * 3 * t)), "params": C2},
        {"kind": "harmonics", "pitch": 150 + 100 * t, "params": dict(samplingRate=16000)},
    ]
    for c, y in zip(calls, batch.synthesize(calls)):
        ref = oracle.generate_harmonics(c["pitch"], amplAnchors=c.get("amplAnchors"), **c["params"])
        assert len(y) == len(ref)
        assert _rms(y, ref) <= TOL


def test_edge_single_and_empty_batches(oracle):
    from soundgen_beta_amd import batch
    c = {"kind": "harmonics", "pitch": np.full(40, 500.0), "params": C2}  # very short: few glottal cycles
    out = batch.synthesize([c])
    ref = oracle.generate_harmonics(c["pitch"], **c["params"])
    assert len(out[0]) == len(ref) and _rms(out[0], ref) <= TOL
    assert batch.synthesize([]) == []


def test_c2_full_batch_properties():
    """C2 at its full size (1024 x 1 s tones, bench.c2_calls), checked by
    size-independent properties: every call's signed max is 1 after R's
    wave / max(wave) (R/source.R:449; up to the fades at the ends), two
    executions of one plan are bit-identical (deterministic max reduction, no
    atomics), and every call's length is the planner's bit-exact length."""
    import os
    import sys
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from soundgen_beta_amd import batch, native
    calls = bench.c2_calls(1024)
    ctx = native.default_context(0)
    plan = batch.Plan(calls, ctx)
    assert (plan.status == 0).all()
    plan.upload()
    outs = []
    for _ in range(2):
        out = torch.full((plan.total,), float("nan"), dtype=torch.float32, device="cuda")
        plan.execute(out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        outs.append(out.cpu().numpy())
    assert np.array_equal(outs[0], outs[1], equal_nan=True)  # slot padding stays NaN
    y = outs[0]
    for i in range(plan.n):
        lo, n = int(plan.offsets[i]), int(plan.lengths[i])
        seg = y[lo:lo + n]
        assert np.isfinite(seg).all(), i
        # <= 1 exactly up to rounding; a fade can shave the largest peak, the next
        # peak of a sampled sinusoid is within ~1e-5 of it
        assert 1.0 - 1e-4 <= float(seg.max()) <= 1.0 + 1e-6, (i, float(seg.max()))


def test_api_plans_once_with_r_rng(oracle):
    """api.soundgen / api.generateHarmonics plan a call once: a
    stochastic 2.5 s sound drawn from R's generator (RRng, set.seed) matches the
    oracle fed by a fresh RRng with the same seed, sample for sample."""
    from soundgen_beta_amd import api
    from soundgen_beta_amd.rrng import RRng
    args = dict(sylLen=2500, samplingRate=44100, temperature=0.1, pitchAnchors=[180, 240], jitterDep=1,
                shimmerDep=5, nonlinBalance=50, subDep=60, addSilence=0)
    y = api.soundgen(rng=RRng(42), **args)
    ref = oracle.soundgen(rng=RRng(42), **args)
    assert len(y) == len(ref) > 1.5 * 44100
    assert _rms(y, ref) <= TOL
    prm = dict(samplingRate=44100, temperature=0.1, jitterDep=1, shimmerDep=5, pitchFloor=50)
    p = np.full(7000, 150.0)
    y = api.generateHarmonics(p, rng=RRng(9), **prm)
    ref = oracle.generate_harmonics(p, rng=RRng(9), **prm)
    assert len(y) == len(ref)
    assert _rms(y, ref) <= TOL


def test_parallel_plan_output_byte_equal(monkeypatch):
    """A batch planned on 7 host threads (chunks concatenated by merge_parts)
    synthesizes exactly the bytes of the same batch planned serially."""
    import torch
    from test_planner import _mixed_calls
    from soundgen_beta_amd import batch, native
    calls = _mixed_calls()
    ctx = native.default_context(0)
    outs = []
    for t in ("1", "7"):
        monkeypatch.setenv("SG_PLAN_THREADS", t)
        plan = batch.Plan(calls, ctx)
        plan.upload()
        out = torch.zeros(plan.total, dtype=torch.float32, device="cuda")
        plan.execute(out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        outs.append((plan.offsets.copy(), plan.lengths.copy(), out.cpu().numpy()))
        plan.close()
    (o1, l1, y1), (o7, l7, y7) = outs
    assert (o1 == o7).all() and (l1 == l7).all()
    assert np.array_equal(y1.view(np.uint32), y7.view(np.uint32))


def test_sharded_batch_byte_equal():
    """bench.py's strong scaling splits ONE batch over ranks (dist.shard, LPT).
    Every call synthesizes the same bytes whether planned in the whole batch or in
    either rank's shard (per-call normalisation, deterministic reductions), so the
    N=2 outputs equal the N=1 outputs call for call."""
    import os
    import sys
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from soundgen_beta_amd import batch, dist, native
    calls = bench.c5_calls(192) + bench.c4_calls(8)
    ctx = native.default_context(0)

    def run(cs):
        plan = batch.Plan(cs, ctx)
        assert (plan.status == 0).all()
        plan.upload()
        out = torch.zeros(max(plan.total, 1), dtype=torch.float32, device="cuda")
        plan.execute(out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        y = out.cpu().numpy()
        res = [y[o:o + n].copy() for o, n in zip(plan.offsets, plan.lengths)]
        plan.close()
        return res

    whole = run(calls)
    for r in range(2):
        idx, mine, owner = dist.shard(calls, r, 2)
        assert 0 < len(idx) < len(calls)
        for i, y in zip(idx, run(mine)):
            assert np.array_equal(y.view(np.uint32), whole[i].view(np.uint32)), (r, int(i))


def test_plan_uploaded_pipeline_byte_equal():
    """batch.plan_uploaded (chunk k + 1 planned on a worker thread while chunk k
    uploads) yields, in order, plans whose outputs equal those of plans built and
    uploaded one after another."""
    import os
    import sys
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from soundgen_beta_amd import batch, native
    calls = bench.c5_calls(70)
    ctx = native.default_context(0)
    sptr = torch.cuda.current_stream().cuda_stream
    got = list(batch.plan_uploaded(calls, ctx, 32))
    assert [a for _, a in got] == [0, 32, 64]
    for p, a in got:
        ref = batch.Plan(calls[a:a + 32], ctx)
        assert ref.total == p.total and (ref.lengths == p.lengths).all() and (p.status == 0).all()
        ref.upload()
        o1 = torch.zeros(max(p.total, 1), dtype=torch.float32, device="cuda")
        o2 = torch.zeros_like(o1)
        p.execute(o1.data_ptr(), sptr)
        ref.execute(o2.data_ptr(), sptr)
        torch.cuda.synchronize()
        assert torch.equal(o1.view(torch.int32), o2.view(torch.int32))
        ref.close()
        p.close()


def test_execute_plans_equals_per_plan_execute():
    """sg_execute_plans (several uploaded plans as one batch, the harmonic chains of
    later plans overlapping the spectral phases of earlier ones on the context's
    second stream) writes exactly the bytes of a loop of sg_execute; the overlap
    knob (SG_OVERLAP, read once per process) does not enter the comparison."""
    import os
    import sys
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from soundgen_beta_amd import batch, native
    calls = bench.c5_calls(96)
    chunks = [calls[0:40], calls[40:41], calls[41:96]]
    ctx = native.default_context(0)
    plans = [batch.Plan(c, ctx) for c in chunks]
    for p in plans:
        assert (p.status == 0).all()
        p.upload()
    outs = [torch.zeros(max(p.total, 1), dtype=torch.float32, device="cuda") for p in plans]
    ref = [torch.zeros_like(o) for o in outs]
    sptr = torch.cuda.current_stream().cuda_stream
    for p, o in zip(plans, ref):
        p.execute(o.data_ptr(), sptr)
    batch.execute_plans(ctx, plans, [o.data_ptr() for o in outs], sptr)
    torch.cuda.synchronize()
    for o, r in zip(outs, ref):
        assert torch.equal(o.view(torch.int32), r.view(torch.int32))
    with pytest.raises(native.SoundgenError):  # a plan listed twice is refused
        batch.execute_plans(ctx, [plans[0], plans[0]], [outs[0].data_ptr()] * 2, sptr)
    for p in plans:
        p.close()


def test_gathered_noise_uniforms_byte_equal():
    """generateNoise()'s uniforms expanded on the device at upload from the union
    of the injected draw ranges (sg_set_uniform_gather(1), the default) synthesize
    the same bytes as the per-item host copy (0): C5 calls reading windows of one
    stream, C3 vowels with breathing noise, and calls on separate arrays."""
    import bench
    from soundgen_beta_amd import batch, native
    rng = np.random.default_rng(11)
    calls = bench.c5_calls(400)[::2] + bench.c3_calls(8)
    calls += [{"kind": "soundgen", "args": {"sylLen": 300, "noiseAnchors": {"time": [0, 300], "value": [-20, -30]},
                                            "samplingRate": 44100, "addSilence": 0},
               "normals": rng.standard_normal(20000), "uniforms": rng.uniform(size=200000)} for _ in range(3)]
    L = native.lib()
    outs = []
    for on in (0, 1):
        assert L.sg_set_uniform_gather(on) == 0
        try:
            outs.append(batch.synthesize(calls))
        finally:
            L.sg_set_uniform_gather(1)
    for a, b in zip(*outs):
        assert a.tobytes() == b.tobytes()
