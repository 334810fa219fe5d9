// sg_env.hip — getSpectralEnvelope() on the device (K7): the formant-filter
// envelope nr x nc of R/sourceSpectrum.R:507-541 (dgamma per formant track and
// column, normalised by the column max, times amplitude, summed, times
// formantDep; lip radiation, open-mouth boost, 2^(dB / 10)), and the same for
// the noise filter of generateNoise() with its rolloff slope (R/source.R:103-105).
//
// One wave per task = SG_ENV_COLS columns of one job. Per column, lane t holds
// the band of track t (and t + 64). Lanes then own bins, two per lane in chunks of
// 128 (env_column2; env_column is the 64-bin form): a ballot over the tracks' bands
// gives the tracks that reach the chunk (a formant is nonzero within a band of a few
// tens of bins), and only those are summed, each track's parameters and fp32
// amplitude by scalar loads. The log-density difference A log2 k - Rr k - Lm is
// formed in fp64 from a log2(k) table (its two products reach ~1e6 for narrow
// formants, so fp32 would lose the difference); the power of two and the sum over
// formants run in fp32. Each chunk ends with coalesced fp32 stores.
//
// Work per selected (chunk, track): per bin 2 fp64 FMA + cvt + v_exp_f32 + FMA, and
// per track ~8 scalar instructions (ballot walk, address, loads) shared by the two
// bins. Output 4 B per bin and column, ~48 B per track and column read once: issue-
// bound (vector and scalar), not HBM-bound.
#include <hip/hip_runtime.h>

#include "sg_dev.h"

constexpr int SG_ENV_LG_LDS = 2048;  // log2(k) table entries staged in LDS per workgroup (r02: 4.9 -> 3.8 ms)

// One column of a job: per 64-bin chunk, the tracks whose bands reach it (ballot),
// their parameters by scalar loads; LG: log2(k) from the LDS copy.
template <bool LG>
__device__ __forceinline__ void env_column(const SgEnvJob& J, int c, const SgEnvTerm* __restrict__ tm,
                                           const SgEnvCol& C, const double* __restrict__ lg2, const double* lgs,
                                           float* __restrict__ fe, int lane) {
  const float thrf = -SG_ENV_CUT;  // log2 units
  // lane t: term t (group 0) and term 64 + t (group 1); absent terms get an empty range
  float amp[2];
  int klo[2], khi[2];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int t = g * 64 + lane;
    const bool in = t < J.ntr;
    const SgEnvTerm& e = tm[in ? t : 0];
    amp[g] = (float)e.amp;
    klo[g] = in ? e.klo : 1 << 30;
    khi[g] = in ? e.khi : -1;
  }
  float* __restrict__ dst = fe + J.out + (int64_t)c * J.nr;
  const char* __restrict__ tb = reinterpret_cast<const char*>(tm);
#pragma unroll 1
  for (int k0 = 0; k0 < J.nr; k0 += 64) {
    const int k = k0 + lane;
    const double x = (double)(k + 1);
    const double lx = LG ? lgs[k] : lg2[k];
    float acc = 0.f;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      uint64_t m = __ballot(klo[g] <= k0 + 64 && khi[g] >= k0 + 1);
      while (m) {
        const int t = __builtin_ctzll(m);
        m ^= 1ull << t;
        // wave-uniform: scalar loads into SGPRs, at a 32-bit byte offset from the column's terms
        const SgEnvTerm* __restrict__ e =
            reinterpret_cast<const SgEnvTerm*>(tb + (unsigned)(g * 64 + t) * (unsigned)sizeof(SgEnvTerm));
        const double a = e->A, r = e->Rr, l = e->Lm;
        const float am = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, amp[g]), t));
        const double d = fma(a, lx, fma(-r, x, -l));
        // d > thr >= -126: the raw v_exp_f32 is exact enough and never denormal
        const float df = (float)d;
        if (df > thrf) acc = fmaf(am, __builtin_amdgcn_exp2f(df), acc);
      }
    }
    const float lxf = (float)lx;
    const float v = fmaf(fmaf(C.lip, lxf, acc), C.boost, J.slope * lxf);
    if (k < J.nr) dst[k] = exp2f(v * 0.1f);
  }
}

// Two bins per lane (SG_ENV_K2): chunks of 128 bins, lane l owns bins k0 + l and
// k0 + 64 + l. The per-track scalar work (ballot walk, term address, scalar loads,
// amplitude broadcast) is shared by both bins: the pair loop issued ~11 SALU next to
// ~9 VALU per (chunk, track), so the scalar pipe bounded it as much as the vector pipe.
// SG_ENV_NOCUT: a selected track adds its term at every bin of the chunk, with no
// per-bin cut (a compare and a select per bin fewer). Outside its band a term is below
// 2^-SG_ENV_CUT of its column max (the band is a superset of the bins within the cut),
// so a bin's dB sum moves by less than |amp| 2^-30 against the cut form (which took the
// 64-bin form's terms exactly); the oracle sums every term.
#ifndef SG_ENV_K2
#define SG_ENV_K2 1
#endif
#ifndef SG_ENV_AMPF
#define SG_ENV_AMPF 1
#endif
#ifndef SG_ENV_NOCUT  // r06v: 2.377 -> 2.213 ms per C5 launch without the per-bin cut
#define SG_ENV_NOCUT 1
#endif
template <bool LG>
__device__ __forceinline__ void env_column2(const SgEnvJob& J, int c, const SgEnvTerm* __restrict__ tm,
                                            const SgEnvCol& C, const double* __restrict__ lg2, const double* lgs,
                                            float* __restrict__ fe, int lane) {
  const float thrf = -SG_ENV_CUT;
  float amp[2];
  int klo[2], khi[2];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int t = g * 64 + lane;
    const bool in = t < J.ntr;
    const SgEnvTerm& e = tm[in ? t : 0];
    amp[g] = (float)e.amp;
    klo[g] = in ? e.klo : 1 << 30;
    khi[g] = in ? e.khi : -1;
  }
  float* __restrict__ dst = fe + J.out + (int64_t)c * J.nr;
  const char* __restrict__ tb = reinterpret_cast<const char*>(tm);
#pragma unroll 1
  for (int k0 = 0; k0 < J.nr; k0 += 128) {
    const int ka = k0 + lane, kb = ka + 64;
    const int ca = ka < J.nr ? ka : J.nr - 1, cb = kb < J.nr ? kb : J.nr - 1;  // table reads in range
    const double xa = (double)(ka + 1), xb = (double)(kb + 1);
    const double lxa = LG ? lgs[ca] : lg2[ca], lxb = LG ? lgs[cb] : lg2[cb];
    float acca = 0.f, accb = 0.f;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      uint64_t m = __ballot(klo[g] <= k0 + 128 && khi[g] >= k0 + 1);
      while (m) {
        const int t = __builtin_ctzll(m);
        m ^= 1ull << t;
        const SgEnvTerm* __restrict__ e =
            reinterpret_cast<const SgEnvTerm*>(tb + (unsigned)(g * 64 + t) * (unsigned)sizeof(SgEnvTerm));
        const double a = e->A, r = e->Rr, l = e->Lm;
        // the amplitude as a scalar load (the planner's (float)amp) or broadcast from its lane
        const float am = SG_ENV_AMPF ? e->ampf
                                     : __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, amp[g]), t));
        const double da = fma(a, lxa, fma(-r, xa, -l)), db = fma(a, lxb, fma(-r, xb, -l));
        const float dfa = (float)da, dfb = (float)db;
        if (SG_ENV_NOCUT) {  // every selected track's term at both bins (below the cut they add < 2^-30 amp)
          acca = fmaf(am, __builtin_amdgcn_exp2f(dfa), acca);
          accb = fmaf(am, __builtin_amdgcn_exp2f(dfb), accb);
        } else {
          if (dfa > thrf) acca = fmaf(am, __builtin_amdgcn_exp2f(dfa), acca);
          if (dfb > thrf) accb = fmaf(am, __builtin_amdgcn_exp2f(dfb), accb);
        }
      }
    }
    const float lfa = (float)lxa, lfb = (float)lxb;
    const float va = fmaf(fmaf(C.lip, lfa, acca), C.boost, J.slope * lfa);
    const float vb = fmaf(fmaf(C.lip, lfb, accb), C.boost, J.slope * lfb);
    if (ka < J.nr) dst[ka] = exp2f(va * 0.1f);
    if (kb < J.nr) dst[kb] = exp2f(vb * 0.1f);
  }
}

extern "C" __global__ __launch_bounds__(256) void sg_spec_env(const SgEnvTask* __restrict__ tasks, int64_t ntask,
                                                              const SgEnvJob* __restrict__ jobs,
                                                              const SgEnvTerm* __restrict__ terms,
                                                              const SgEnvCol* __restrict__ cols,
                                                              const double* __restrict__ lg2, int64_t nlg,
                                                              float* __restrict__ fe) {
  const int64_t w = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const SgEnvTask T = tasks[w < ntask ? w : ntask - 1];
  const SgEnvJob J = jobs[T.job];
  // the log2(k) table is common to every job: one LDS copy per workgroup, as far
  // as the workgroup's longest column reaches (whole 64-bin chunks)
  __shared__ double lgs[SG_ENV_LG_LDS];
  __shared__ int nrw[4];
  if (lane == 0) nrw[threadIdx.x >> 6] = (J.nr + 63) / 64 * 64;
  __syncthreads();
  int need = nrw[0] > nrw[1] ? nrw[0] : nrw[1];
  need = need > nrw[2] ? need : nrw[2];
  need = need > nrw[3] ? need : nrw[3];
  const int cap = nlg < SG_ENV_LG_LDS ? (int)nlg : SG_ENV_LG_LDS;
  const int nst = need < cap ? need : cap;
  for (int i = threadIdx.x; i < nst; i += 256) lgs[i] = lg2[i];
  __syncthreads();
  if (w >= ntask) return;
  const int c1 = T.c0 + SG_ENV_COLS < J.nc ? T.c0 + SG_ENV_COLS : J.nc;
  const bool lds = (J.nr + 63) / 64 * 64 <= nst;  // every chunk's k inside the staged table
#pragma unroll 1
  for (int c = T.c0; c < c1; ++c) {
    const SgEnvTerm* __restrict__ tm = terms + J.term0 + (int64_t)c * J.ntr;
    const SgEnvCol C = cols[J.col0 + c];
    if (SG_ENV_K2) {
      if (lds) env_column2<true>(J, c, tm, C, lg2, lgs, fe, lane);
      else env_column2<false>(J, c, tm, C, lg2, lgs, fe, lane);
    } else {
      if (lds) env_column<true>(J, c, tm, C, lg2, lgs, fe, lane);
      else env_column<false>(J, c, tm, C, lg2, lgs, fe, lane);
    }
  }
}

#include "sg_exec.h"

namespace sg {
void launch_spec_env(const DevicePlan& D, const Batch& B, hipStream_t s) {
  const int64_t n = (int64_t)B.envtasks.size();
  if (n <= 0) return;
  hipLaunchKernelGGL(sg_spec_env, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, D.envtasks, n, D.envjobs, D.eterms,
                     D.ecols, D.elog2, (int64_t)B.elog2.size(), D.fl + B.fe_base);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw SgError(SG_E_DEVICE, std::string("launch sg_spec_env: ") + hipGetErrorString(e));
}
}  // namespace sg
