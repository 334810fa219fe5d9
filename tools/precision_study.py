"""Where does fp32 round-off enter the formant filter's output? (diagnostic)

For preset calls of the C5 workload, the oracle's formant-filter input (the
fp64 pre-filter sound and envelope, captured with or_debug_capture) is run
through a numpy restatement of seewave stft x env -> istft with chosen stages
in fp32 (scipy.fft computes complex64 in single precision), and compared with
the all-fp64 result (RMS on the /max-normalised output, the parity metric):

  src32    sound rounded to fp32, filter in fp64
  srcnoise sound + white noise of eps32 x |sound|max / 2 (a Clenshaw-like compute error)
  fwd32    fp32 forward STFT + envelope multiply, fp64 inverse
  inv32    fp64 forward, fp32 inverse
  all32    everything fp32

    python tools/precision_study.py [preset ...]
"""
import ctypes as C
import os
import sys

import numpy as np
import scipy.fft as sfft

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def capture(O, call):
    L = O.lib()
    L.or_debug_capture.argtypes = [C.c_int]
    L.or_debug_captured.restype = C.c_int64
    L.or_debug_capture(1)
    y = O.soundgen(normals=call.get("normals"), uniforms=call.get("uniforms"), **call["args"])
    n = L.or_debug_captured(None, None, None, None)
    nc, wl = C.c_int64(), C.c_int64()
    L.or_debug_captured(None, None, C.byref(nc), C.byref(wl))
    s = np.zeros(n)
    e = np.zeros(nc.value * (wl.value // 2))
    L.or_debug_captured(s.ctypes.data_as(C.POINTER(C.c_double)), e.ctypes.data_as(C.POINTER(C.c_double)), None, None)
    L.or_debug_capture(0)
    return y, s, e.reshape(nc.value, wl.value // 2), wl.value


def filt(sound, env, wl, fwd=np.float64, inv=np.float64, overlap=75, norm=True):
    L = len(sound)
    nr = wl // 2
    h = wl * (100 - overlap) / 100
    step = np.arange(1, max(1, L - wl) + 1e-9, h)
    nc = len(step)
    i = np.arange(wl)
    ham = 0.54 - 0.46 * np.cos(2 * np.pi * i / (wl - 1))
    han = 0.5 - 0.5 * np.cos(2 * np.pi * i / (wl - 1))
    idx = (step[:, None] + i[None, :]).astype(np.int64) - 1
    fr = (sound[idx] * ham).astype(fwd)
    Z = sfft.fft(fr, axis=1)[:, :nr] / fwd(wl)
    E = env if env.shape[0] == nc else np.repeat(env, nc, axis=0)
    Z = (Z * E.astype(fwd)).astype(np.complex64 if inv == np.float32 else np.complex128)
    X = np.concatenate([Z, Z[:, nr - 1:nr].real + 0j, np.conj(Z[:, 1:][:, ::-1])], axis=1)
    y = sfft.ifft(X, axis=1).real / inv(2 * nr) * han.astype(inv)
    xlen = int(wl + (nc - 1) * h)
    out = np.zeros(xlen, np.float64)
    for f in range(nc):
        b = int(f * h)
        out[b:b + wl] += y[f].astype(np.float64)
    out = out * h / np.sum(han ** 2)
    return out / out.max() if norm else out


def rms(a, b):
    return float(np.sqrt(np.mean((a - b) ** 2)))


def main(presets):
    import bench
    from oracle import oracle as O
    calls = [c for c in bench.c5_calls(3000) if not presets or c["preset"] in presets]
    seen = {}
    for c in calls:
        if seen.get(c["preset"], 0) >= 2:
            continue
        seen[c["preset"]] = seen.get(c["preset"], 0) + 1
        try:
            y, s, e, wl = capture(O, c)
        except Exception as ex:  # noqa: BLE001
            print(c["preset"], "oracle refused:", ex)
            continue
        if len(s) == 0:
            print(c["preset"], "no filter")
            continue
        ref = filt(s, e, wl)
        rng = np.random.default_rng(1)
        res = {
            "src32": rms(filt(s.astype(np.float32).astype(np.float64), e, wl), ref),
            "srcnoise": rms(filt(s + rng.standard_normal(len(s)) * 6e-8 * np.abs(s).max() / 2, e, wl), ref),
            "fwd32": rms(filt(s, e, wl, fwd=np.float32), ref),
            "inv32": rms(filt(s, e, wl, inv=np.float32), ref),
            "all32": rms(filt(s.astype(np.float32).astype(np.float64), e, wl, np.float32, np.float32), ref),
        }
        ed = 10 * np.log2(e.max() / np.median(e)) if e.size else 0
        # noise gain / signal gain: white source noise through the envelope vs the source itself
        yr = filt(s, e, wl, norm=False)
        pred = float(np.sqrt(np.mean(e ** 2)) * np.sqrt(np.mean(s ** 2)) / np.sqrt(np.mean(yr ** 2)))
        res["pred"] = pred
        # planner-style estimate: per envelope column, rms over bins of env / source-power-weighted
        # rms of env (source power from the fp64 STFT of the sound)
        nr = wl // 2
        h = wl // 4
        step = np.arange(1, max(1, len(s) - wl) + 1e-9, wl * 0.25)
        i = np.arange(wl)
        ham = 0.54 - 0.46 * np.cos(2 * np.pi * i / (wl - 1))
        idx = (step[:, None] + i[None, :]).astype(np.int64) - 1
        P = np.abs(np.fft.fft(s[idx] * ham, axis=1)[:, :nr]) ** 2
        E = e if e.shape[0] == len(step) else np.repeat(e, len(step), axis=0)
        ng = np.sqrt(np.mean(E ** 2, axis=1))
        sg = np.sqrt(np.sum(P * E ** 2, axis=1) / np.maximum(np.sum(P, axis=1), 1e-300))
        w = np.sum(P, axis=1)
        rho_all = ng / sg
        res["rho_max"] = float(np.max(rho_all[w > 1e-6 * w.max()]))
        res["rho_g"] = float(np.sqrt(np.sum(ng ** 2 * w) / np.sum(sg ** 2 * w)))
        print("%-22s wl %5d nc %4d env dB range %6.1f  " % (c["preset"], wl, e.shape[0], ed) +
              " ".join("%s %.2e" % kv for kv in res.items()), flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
