"""GPU parity of the spectral path (sg_fft.hip) and of whole soundgen() calls
against the oracle, same inputs and draws. Tolerance: RMS <= 1e-5 on the
normalised waveform (north star); lengths bit-exact."""
import numpy as np
import pytest

from test_spectral_cpu import FORMANTS_A, MOVING, N, SOUNDGEN_CASES, U

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _rms(a, b):
    return float(np.sqrt(np.mean((np.asarray(a, np.float64) - b) ** 2)))


@pytest.mark.parametrize("wl", [8, 64, 440, 800, 1000, 1764, 2048, 2204, 2400])
def test_wave_fft_vs_numpy(wl):
    """The wavefront FFT stages (radices 2, 4, odd primes) against numpy, both
    directions; wl = 2204 also with its radix-29 stage on the VALU (the noise
    kernel's) as well as on the matrix pipe (the filter kernel's)."""
    import ctypes as C
    from soundgen_beta_amd import native
    M, nf = wl // 2, 3
    rng = np.random.default_rng(wl)
    x = (rng.normal(size=(nf, M)) + 1j * rng.normal(size=(nf, M))).astype(np.complex64)
    ctx = native.Context(0)
    try:
        for inv in ((0, 1, 2, 3) if wl == 2204 else (0, 1)):
            src = np.ascontiguousarray(x).view(np.float32).ravel()
            dst = np.zeros_like(src)
            fp = C.POINTER(C.c_float)
            rc = native.lib().sg_debug_wave_fft(ctx.ptr, wl, inv, nf, src.ctypes.data_as(fp), dst.ctypes.data_as(fp))
            if rc == -4:  # SG_E_UNSUPPORTED: not a wavefront-path geometry
                pytest.skip("wl %d runs the workgroup FFT" % wl)
            native.check(rc, ctx.ptr)
            got = dst.view(np.complex64).reshape(nf, M)
            want = np.fft.ifft(x, axis=1) * M if inv & 1 else np.fft.fft(x, axis=1)
            err = np.abs(got - want).max() / np.abs(want).max()
            assert err < 2e-6 * np.log2(M) + 1e-6, (wl, inv, err)
    finally:
        ctx.close()


# odd wl (441, 1101, 2203, 2205): windowLength_points = floor(L / 2) for short
# sounds (R/soundgen.R:743); seewave inverts wl - 1 points against a wl-point window
@pytest.mark.parametrize("wl", [440, 800, 1764, 2204, 2038, 1998, 6000, 441, 1101, 2203, 2205])
def test_formant_filter_vs_oracle(oracle, wl):
    from soundgen_beta_amd import api
    rng = np.random.default_rng(wl)
    sound = np.sin(np.cumsum(rng.uniform(0.01, 0.2, 20 * wl))) + 0.1 * rng.normal(size=20 * wl)
    nr = wl // 2
    step = np.arange(1, max(1, len(sound) - wl) + 1e-9, wl * 0.25)  # seq(1, L - wl, by = hop)
    for env in (np.abs(rng.normal(1, 0.3, size=(nr, 1))), np.abs(rng.normal(1, 0.3, size=(nr, len(step))))):
        got = api.formantFilter(sound, env, wl, 75)
        want = oracle.formant_filter(sound, env, wl, 75)
        assert len(got) == len(want)
        assert _rms(got, want) <= TOL


@pytest.mark.parametrize("wl,sr", [(800, 16000), (2204, 44100), (440, 44100), (1442, 44100), (2203, 44100),
                                   (441, 44100)])
def test_generate_noise_vs_oracle(oracle, wl, sr):
    from soundgen_beta_amd import api
    na = {"time": [0, 1000], "value": [-30, -10]}
    for L, filt in ((sr, None), (sr // 3, np.abs(np.random.default_rng(3).normal(1, .5, size=(wl // 2, 5))))):
        got = api.generateNoise(L, na, rolloffNoise=-6, attackLen=20, windowLength_points=wl, samplingRate=sr,
                                filterNoise=filt, uniforms=U)
        want = oracle.generate_noise(L, na, rolloffNoise=-6, attackLen=20, windowLength_points=wl, samplingRate=sr,
                                     filterNoise=filt, uniforms=U)
        assert len(got) == len(want)
        assert _rms(got, want) <= TOL


def test_soundgen_cases_one_batch(oracle):
    from soundgen_beta_amd import batch
    names = sorted(SOUNDGEN_CASES)
    calls = [{"kind": "soundgen", "args": SOUNDGEN_CASES[n], "normals": N, "uniforms": U} for n in names]
    outs = batch.synthesize(calls)
    for n, y in zip(names, outs):
        ref = oracle.soundgen(normals=N, uniforms=U, **SOUNDGEN_CASES[n])
        assert len(y) == len(ref), n
        r = _rms(y, ref)
        print(n, "rms", r)
        assert r <= TOL, (n, r)


def test_short_sounds_odd_windows(oracle):
    """Syllables of 40-52 ms at 44.1 kHz: the formant filter's window shrinks to
    floor(L / 2) points (R/soundgen.R:743), odd for about half of them, and the
    shrink persists into the second bout's noise (repeatBout = 2)."""
    from soundgen_beta_amd import batch
    cases = []
    for ms in range(40, 53):
        cases.append(dict(sylLen=ms, samplingRate=44100, temperature=0, addSilence=0, pitchAnchors=[300, 350],
                          formants="a", repeatBout=2, pauseLen=30,
                          noiseAnchors={"time": [0, ms], "value": [-20, -20]}, formantsNoise="s"))
    calls = [{"kind": "soundgen", "args": a, "normals": N, "uniforms": U} for a in cases]
    outs = batch.synthesize(calls)
    for a, y in zip(cases, outs):
        assert not isinstance(y, Exception), (a["sylLen"], y)
        ref = oracle.soundgen(normals=N, uniforms=U, **a)
        assert len(y) == len(ref), a["sylLen"]
        assert _rms(y, ref) <= TOL, (a["sylLen"], _rms(y, ref))


def _bench():
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    return bench


def test_c4_calls_vs_oracle(oracle):
    """C4: the whole 512-call batch (3 s, 44.1 kHz, nonlinBalance 100,
    subharmonics, jitter/shimmer random walks at temperature 0.05, injected draws)
    is planned and synthesized with no refused call; 32 calls spread over the batch
    are compared with the oracle (RMS <= 1e-5, exact lengths)."""
    bench = _bench()
    from soundgen_beta_amd import batch
    calls = bench.c4_calls(512)
    outs = batch.synthesize(calls)
    bad = [i for i, y in enumerate(outs) if isinstance(y, Exception)]
    assert not bad, [(i, str(outs[i])) for i in bad[:5]]
    worst = 0.0
    for i in range(0, 512, 16):
        ref = bench.oracle_call(oracle, calls[i])
        assert len(outs[i]) == len(ref), i
        r = _rms(outs[i], ref)
        worst = max(worst, r)
        assert r <= TOL, (i, r)
    print("C4 worst rms", worst)


def test_c5_presets_one_batch(oracle):
    """C5: calls drawn from the 33 presets of R/presets.R with scaled
    sylLen and pitch, 44.1 kHz, the presets' own temperatures and separately
    filtered noise (formantsNoise), subharmonic sidebands up to ~400 rows
    (sg_sine_bank_tall). No call is refused (zero-width loess fits take R's
    span + 0.1 retry, odd windows run the odd-length DFT path); every call is
    compared with the oracle at RMS <= 1e-5, Misc$Cow included (its bouts take
    the fp64 filter path the planner's conditioning estimate selects)."""
    bench = _bench()
    from soundgen_beta_amd import batch
    calls = bench.c5_calls(128)
    plan = batch.Plan(calls, None)
    assert (plan.status == 0).all(), [(i, plan.message(i)) for i in np.nonzero(plan.status)[0][:5]]
    outs = batch.synthesize(calls)
    worst = 0.0
    for i, y in enumerate(outs):
        ref = bench.oracle_call(oracle, calls[i])
        assert len(y) == len(ref), calls[i]["preset"]
        r = _rms(y, ref)
        worst = max(worst, r)
        assert r <= TOL, (i, calls[i]["preset"], r)
    print("C5 worst rms", worst, "over", len(outs), "calls")


def test_c5_1024_calls_spread_over_the_batch(oracle):
    """1,024 calls spread over the 65,536-call C5 batch (every 64th, each reading its own
    draw window) planned as one batch and compared with the oracle at RMS <= 1e-5 with
    exact lengths; the oracle runs on a 16-thread pool (its ctypes calls release the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    bench = _bench()
    from soundgen_beta_amd import batch
    calls = bench.c5_calls(65536)[::64]
    outs = batch.synthesize(calls)
    bad = [i for i, y in enumerate(outs) if isinstance(y, Exception)]
    assert not bad, [(i, str(outs[i])) for i in bad[:5]]
    with ThreadPoolExecutor(16) as ex:
        refs = list(ex.map(lambda c: bench.oracle_call(oracle, c), calls))
    worst, where = 0.0, None
    for i, (y, ref) in enumerate(zip(outs, refs)):
        assert len(y) == len(ref), (i, calls[i]["preset"])
        r = _rms(y, ref)
        if r > worst:
            worst, where = r, calls[i]["preset"]
        assert r <= TOL, (i, calls[i]["preset"], r)
    print("C5 1024 calls: worst rms", worst, where)


def _per_preset(bench, k):
    """The first k calls of each of the 33 presets in the C5 stream."""
    calls, seen = [], {}
    for c in bench.c5_calls(4000):
        if seen.get(c["preset"], 0) < k:
            seen[c["preset"]] = seen.get(c["preset"], 0) + 1
            calls.append(c)
    assert len(seen) == 33 and min(seen.values()) == k
    return calls


@pytest.mark.parametrize("policy", [1, 2], ids=["default", "fp64_all"])
def test_c5_every_preset_vs_oracle(oracle, policy):
    """Two calls of EACH of the 33 presets against the oracle at RMS <= 1e-5.
    policy 1: the default (fp64 filter path where the planner's conditioning
    estimate exceeds native.HP_RHO_DEFAULT: Misc$Cow, Misc$Elephant); policy 2: every filtered bout on the fp64
    path (sg_sine_bank_hp, sg_harm_finalize_hp, sg_mix_hp, sg_fft_frames64)."""
    bench = _bench()
    from soundgen_beta_amd import batch, native
    calls = _per_preset(bench, 2)
    L = native.lib()
    assert L.sg_set_fp64_policy(policy, native.HP_RHO_DEFAULT) == 0
    try:
        plan = batch.Plan(calls, None)
        hp, nfr, ntk = plan.precision()
        outs = batch.synthesize(calls)
    finally:
        L.sg_set_fp64_policy(1, native.HP_RHO_DEFAULT)
    cow = [i for i, c in enumerate(calls) if c["preset"] == "Misc$Cow"]
    assert all(hp[i] > 0 for i in cow)
    worst = {}
    for i, y in enumerate(outs):
        ref = bench.oracle_call(oracle, calls[i])
        assert len(y) == len(ref), calls[i]["preset"]
        r = _rms(y, ref)
        p = calls[i]["preset"]
        worst[p] = max(worst.get(p, 0.0), r)
        assert r <= TOL, (i, p, r, int(hp[i]))
    print("policy", policy, "fp64 calls", int((hp > 0).sum()), "frames", nfr, "tasks", ntk)
    print(sorted(worst.items(), key=lambda kv: -kv[1])[:6])


def test_c3_all_vowels_vs_oracle(oracle):
    """C3: 36 calls of bench.c3_calls(1024) covering all six vowels
    a/o/i/e/u/0 (R/presets.R:176-212), 2 s at 44.1 kHz with breathing noise,
    against the oracle (RMS <= 1e-5, exact lengths)."""
    bench = _bench()
    from soundgen_beta_amd import batch
    allc = bench.c3_calls(1024)
    pick, seen = [], {}
    for i, c in enumerate(allc):
        v = c["args"]["formants"]
        if seen.get(v, 0) < 6:
            seen[v] = seen.get(v, 0) + 1
            pick.append(i)
    assert sorted(seen) == sorted("aoieu0") and len(pick) == 36
    calls = [allc[i] for i in pick]
    outs = batch.synthesize(calls)
    worst = 0.0
    for c, y in zip(calls, outs):
        ref = bench.oracle_call(oracle, c)
        assert len(y) == len(ref), c["args"]["formants"]
        r = _rms(y, ref)
        worst = max(worst, r)
        assert r <= TOL, (c["args"]["formants"], r)
    print("C3 worst rms", worst)

# getSpectralEnvelope's matrix comes from sg_spec_env (fp32 terms, fp32 2^(dB/10)):
# per-bin relative error vs the fp64 oracle <= 1e-5 (the waveform bar is RMS <= 1e-5)
ENV_RTOL = 1e-5


def _api():
    from soundgen_beta_amd import api
    return api


@pytest.mark.parametrize("fm,nc,extra", [
    (FORMANTS_A, 1, {}),
    (MOVING, 37, {}),
    ("a", 1, dict(vocalTract=15.5)),
    ("u", 25, dict(mouthAnchors={"time": [0, 1], "value": [0, 0.8]}, mouthOpenThres=0.2, openMouthBoost=5)),
    (None, 1, dict(vocalTract=17)),  # schwa from vocalTract
])
def test_spectral_envelope_matches_oracle(oracle, fm, nc, extra):
    kw = dict(formants=fm, samplingRate=44100, **extra)
    got = _api().getSpectralEnvelope(1102, nc, **kw)
    want = oracle.spectral_envelope(1102, nc, **kw)
    np.testing.assert_allclose(got, want, rtol=ENV_RTOL, atol=0)


def test_spectral_envelope_stochastic_same_draws(oracle):
    kw = dict(formants=FORMANTS_A, samplingRate=16000, temperature=0.1, vocalTract=15)
    got = _api().getSpectralEnvelope(400, 9, rng=np.random.default_rng(9), **kw)
    want = oracle.spectral_envelope(400, 9, rng=np.random.default_rng(9), **kw)
    np.testing.assert_allclose(got, want, rtol=ENV_RTOL)




def test_spectral_envelope_stochastic_formants_44k(oracle):
    """temperature > 0 at 44.1 kHz adds stochastic formants up to sr/2 - 1000
    (R/sourceSpectrum.R:347-415): ~20 tracks per column, narrow and wide."""
    for seed in range(4):
        kw = dict(formants=MOVING, samplingRate=44100, temperature=0.2, vocalTract=16)
        got = _api().getSpectralEnvelope(1102, 61, rng=np.random.default_rng(seed), **kw)
        want = oracle.spectral_envelope(1102, 61, rng=np.random.default_rng(seed), **kw)
        np.testing.assert_allclose(got, want, rtol=ENV_RTOL)
