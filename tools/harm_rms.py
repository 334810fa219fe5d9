"""Diagnostic: generateHarmonics() GPU vs oracle for a Misc$Cow-like contour
(low f0, steep rolloff, temperature 0.05) under parameter variants."""
import copy, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from soundgen_beta_amd import batch
from oracle import oracle as O

rng = np.random.default_rng(5)
Z = rng.standard_normal(200000)
U = rng.uniform(size=4000000)
t = np.linspace(0, 1, 6000)
pitch = np.interp(t, [0, .61, .85, 1], [60, 85, 165, 160])
base = dict(samplingRate=44100, temperature=0.05, rolloff=-24, rolloffKHz=-10, rolloffOct=0, nonlinBalance=66,
            subDep=50, shortestEpoch=125, jitterDep=2, pitchFloor=50, attackLen=50)
variants = {"as is": {}, "no nonlin": {"nonlinBalance": 0}, "no jitter": {"jitterDep": 0},
            "no drift": {"pitchDriftDep": 0}, "temp0": {"temperature": 0},
            "no nonlin/jitter": {"nonlinBalance": 0, "jitterDep": 0},
            "rolloff -12": {"rolloff": -12}, "rolloff -36": {"rolloff": -36}}
calls = []
for lab, mod in variants.items():
    p = copy.deepcopy(base)
    p.update(mod)
    calls.append({"kind": "harmonics", "pitch": pitch, "params": p, "normals": Z, "uniforms": U})
outs = batch.synthesize(calls)
for (lab, _), c, y in zip(variants.items(), calls, outs):
    ref = O.generate_harmonics(c["pitch"], normals=Z, uniforms=U, **c["params"])
    if isinstance(y, Exception) or len(y) != len(ref):
        print(lab, "mismatch", y if isinstance(y, Exception) else (len(y), len(ref)))
        continue
    e = y - ref
    k = int(np.abs(e).argmax())
    print("%-20s rms %.3e maxabs %.2e at %d/%d" % (lab, np.sqrt(np.mean(e ** 2)), abs(e[k]), k, len(y)))
