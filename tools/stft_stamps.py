"""Diagnostic: cycles per section of sg_stft_ola's frame loop, from a library
built with -DSG_STFT_STAMPS (tools/build_variant.sh stamps -DSG_STFT_STAMPS,
SRC=sg_fft.hip).  SG_HIP_LIB=.../exp_stamps.so python tools/stft_stamps.py c3 [calls]
Sections (per wave, summed over frames), reported separately for the filter
kernel (sg_stft_ola) and the noise kernel (sg_stft_ola_noise): 0 descriptor +
input loads + hamming store (filter frames), 1-3 forward FFT stages (filter
frames; stage 3 = all stages after the second), 4 untangle x envelope (filter)
or input loads + the noise spectrum (noise), 5-7 inverse FFT stages, 8 hanning
+ carry add, 9 output + next carry.
"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import bench  # noqa: E402
from soundgen_beta_amd import batch, native  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
make, n_default, _ = bench.CONFIGS[cfg]
n = int(sys.argv[2]) if len(sys.argv) > 2 else n_default
calls = make(n)
ctx = native.Context(0)
p = batch.Plan(calls, ctx)
p.upload()
out = torch.empty((p.total + 63) // 64 * 64, dtype=torch.float32, device="cuda:0")
L = native.lib()
f = L.sg_debug_stft_stamps
f.argtypes = [C.POINTER(C.c_ulonglong)]
buf = (C.c_ulonglong * 32)()
p.execute(out.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
f(buf)  # drop the warmup
reps = 3
for _ in range(reps):
    p.execute(out.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
f(buf)
names = ["loads+ham", "fwd_s1", "fwd_s2", "fwd_s3+", "untangle", "inv_s1", "inv_s2", "inv_s3+", "han+carry",
         "out+carry"]
res = {"config": cfg, "calls": n}
for kern, base in (("sg_stft_ola", 0), ("sg_stft_ola_noise", 16)):
    v = list(buf)[base:base + 16]
    frames, waves = v[10], v[11]
    tot = sum(v[:10])
    res[kern] = {"frames": frames, "waves": waves, "cycles_per_frame_total": tot / max(frames, 1),
                 "cycles_per_frame": {k: v[i] / max(frames, 1) for i, k in enumerate(names)},
                 "share": {k: v[i] / max(tot, 1) for i, k in enumerate(names)}}
print(json.dumps(res, indent=1))
