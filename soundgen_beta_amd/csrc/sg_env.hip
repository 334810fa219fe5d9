// sg_env.hip — getSpectralEnvelope() on the device (K7): the formant-filter
// envelope nr x nc of R/sourceSpectrum.R:507-541 (dgamma per formant track and
// column, normalised by the column max, times amplitude, summed, times
// formantDep; lip radiation, open-mouth boost, 2^(dB / 10)), and the same for
// the noise filter of generateNoise() with its rolloff slope (R/source.R:103-105).
//
// One wave per task = SG_ENV_COLS columns of one job. Lanes own bins: for each
// chunk of 64 bins the wave computes log2(k) once (fp64), then per column sums
// the formant terms whose planner-computed bin range [klo, khi] meets the chunk
// (wave-uniform skip: a formant's term is nonzero within a band of ~25 widths)
// and writes 64 consecutive fp32 values (coalesced). The log-density difference
// A log2 k - Rr k - Lm is formed in fp64 (its two products are ~1e6 for narrow
// formants, so fp32 would lose the difference); the power of two and the sum
// over formants run in fp32.
//
// Bound: neither HBM (4 B written per bin and column, ~48 B read per formant and
// column) nor transcendental rate dominates; per active term 2 fp64 FMA +
// cvt + v_exp_f32 + FMA.
#include <hip/hip_runtime.h>

#include "sg_dev.h"

extern "C" __global__ __launch_bounds__(256) void sg_spec_env(const SgEnvTask* __restrict__ tasks, int64_t ntask,
                                                              const SgEnvJob* __restrict__ jobs,
                                                              const SgEnvTerm* __restrict__ terms,
                                                              const SgEnvCol* __restrict__ cols,
                                                              float* __restrict__ fe) {
  const int64_t w = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (w >= ntask) return;
  const int lane = threadIdx.x & 63;
  const SgEnvTask T = tasks[w];
  const SgEnvJob J = jobs[T.job];
  const int c1 = T.c0 + SG_ENV_COLS < J.nc ? T.c0 + SG_ENV_COLS : J.nc;
  const double thr = -80.0 * 1.4426950408889634;  // e^-80 of the column max, in log2 units
#pragma unroll 1
  for (int k0 = 0; k0 < J.nr; k0 += 64) {
    const int k = k0 + lane;
    const double x = (double)(k + 1);
    const double lx = log2(x);
    const float lxf = (float)lx;
#pragma unroll 1
    for (int c = T.c0; c < c1; ++c) {
      const SgEnvTerm* __restrict__ tm = terms + J.term0 + (int64_t)c * J.ntr;
      float acc = 0.f;
#pragma unroll 1
      for (int t = 0; t < J.ntr; ++t) {
        const SgEnvTerm& e = tm[t];
        if (e.khi < k0 + 1 || e.klo > k0 + 64) continue;  // band misses the chunk
        const double d = fma(e.A, lx, fma(-e.Rr, x, -e.Lm));
        if (d > thr) acc = fmaf((float)e.amp, exp2f((float)d), acc);
      }
      const SgEnvCol C = cols[J.col0 + c];
      const float v = fmaf(fmaf(C.lip, lxf, acc), C.boost, J.slope * lxf);
      if (k < J.nr) fe[J.out + (int64_t)c * J.nr + k] = exp2f(v * 0.1f);
    }
  }
}

#include "sg_exec.h"

namespace sg {
void launch_spec_env(const DevicePlan& D, const Batch& B, hipStream_t s) {
  const int64_t n = (int64_t)B.envtasks.size();
  if (n <= 0) return;
  hipLaunchKernelGGL(sg_spec_env, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, D.envtasks, n, D.envjobs, D.eterms,
                     D.ecols, D.fl + B.fe_base);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw SgError(SG_E_DEVICE, std::string("launch sg_spec_env: ") + hipGetErrorString(e));
}
}  // namespace sg
