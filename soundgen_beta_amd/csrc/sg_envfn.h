// sg_envfn.h — one bin of a spectral-envelope column (R/sourceSpectrum.R:507-541, the
// restatement in sg_dev.h above SgEnvTerm), evaluated by a wavefront. Shared by
// sg_spec_env (materialised columns) and sg_stft_ola (columns evaluated in the frame
// that uses them), so that both give the same bits.
//
// A bin's value is the sum over the column's tracks in track order of the terms that
// pass the cut (d > -SG_ENV_CUT). A wave evaluates the bins of a 1-based range [a, b]
// and sums only the tracks whose band [klo, khi] meets the range (ballot); a band
// contains every bin where its term passes the cut, so the skipped tracks add nothing
// at any bin of the range, and the value does not depend on the range.
#pragma once
#include <hip/hip_runtime.h>

#include "sg_dev.h"

namespace sgd {

// lane t's copy of tracks t and 64 + t (G = 2; G = 1: columns of <= 64 tracks) of a
// column (absent tracks: an empty band). REG: the log-density parameters too, which
// env_bin then broadcasts by v_readlane instead of scalar loads -- for a wave that
// runs alone on its SIMD (sg_stft_ola) each scalar load's latency was exposed per
// (chunk, track), and its s_waitcnt also drained the LDS reads in flight.
template <int G = 2, bool REG = false>
struct EnvLane {
  float amp[G];
  int klo[G], khi[G];
  double A[REG ? G : 1], Rr[REG ? G : 1], Lm[REG ? G : 1];
};

template <int G = 2, bool REG = false>
__device__ __forceinline__ EnvLane<G, REG> env_lane(const SgEnvTerm* __restrict__ tm, int ntr, int lane) {
  EnvLane<G, REG> L;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int t = g * 64 + lane;
    const bool in = t < ntr;
    const SgEnvTerm& e = tm[in ? t : 0];
    L.amp[g] = (float)e.amp;
    L.klo[g] = in ? e.klo : 1 << 30;
    L.khi[g] = in ? e.khi : -1;
    if constexpr (REG) {
      L.A[g] = e.A;
      L.Rr[g] = e.Rr;
      L.Lm[g] = e.Lm;
    }
  }
  return L;
}

__device__ __forceinline__ double lane_f64(double v, int t) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, t);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), t);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// env(k) at the 0-based bin k (lx = log2(k + 1)); [a, b] (1-based, wave-uniform)
// contains k + 1 for every lane. Every lane of the wave must call it (ballot).
template <int G, bool REG>
__device__ __forceinline__ float env_bin(const EnvLane<G, REG>& L, const SgEnvTerm* __restrict__ tm, float lip,
                                         float boost, float slope, int k, double lx, int a, int b) {
  const float thrf = -SG_ENV_CUT;  // log2 units
  const double x = (double)(k + 1);
  float acc = 0.f;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    uint64_t m = __ballot(L.klo[g] <= b && L.khi[g] >= a);
    while (m) {
      const int t = __builtin_ctzll(m);
      m &= m - 1;
      double A, r, l;
      if constexpr (REG) {
        A = lane_f64(L.A[g], t);
        r = lane_f64(L.Rr[g], t);
        l = lane_f64(L.Lm[g], t);
      } else {
        const SgEnvTerm* __restrict__ e = tm + g * 64 + t;  // wave-uniform: scalar loads into SGPRs
        A = e->A;
        r = e->Rr;
        l = e->Lm;
      }
      const float am = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, L.amp[g]), t));
      // the products reach ~1e6 for narrow formants: the difference is formed in fp64
      const double d = fma(A, lx, fma(-r, x, -l));
      // d > thr >= -126: the raw v_exp_f32 is exact enough and never denormal
      const float df = (float)d;
      if (df > thrf) acc = fmaf(am, __builtin_amdgcn_exp2f(df), acc);
    }
  }
  const float lxf = (float)lx;
  const float v = fmaf(fmaf(lip, lxf, acc), boost, slope * lxf);
  return exp2f(v * 0.1f);
}

}  // namespace sgd
