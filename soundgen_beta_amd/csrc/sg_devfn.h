// sg_devfn.h — device helpers shared by the HIP kernels (contours, approx, reductions).
#pragma once
#include <hip/hip_runtime.h>

#include "sg_dev.h"

namespace sgd {

__device__ __forceinline__ double seqint_at(double from, double to, int n, int i) {
  if (i == 0) return from;
  if (i == n - 1) return to;
  const double by = (to - from) / (double)(n - 1);
  return (i < n / 2) ? from + (double)i * by : to - (double)(n - 1 - i) * by;
}

__device__ __forceinline__ double contour_at(const SgContour& c, const double* __restrict__ ck, int64_t L, int64_t k) {
  double v;
  if (c.kind == 1) v = c.a;
  else if (c.kind == 2) {
    if (k == 0 || c.a == c.b) v = c.a;
    else if (k == L - 1) v = c.b;
    else v = c.a + (double)k * (L == c.L ? c.by : (c.b - c.a) / (double)(L - 1));
  } else {
    const double* x = ck + c.k_off;
    const double* y = x + c.nk;
    const double* b = y + c.nk;
    const double* cc = b + c.nk;
    const double* d = cc + c.nk;
    double u;
    if (k == 0) u = c.a;
    else if (k == L - 1) u = c.b;
    else {
      const double by = L == c.L ? c.by : (c.b - c.a) / (double)(L - 1);
      u = (k < L / 2) ? c.a + (double)k * by : c.b - (double)(L - 1 - k) * by;
    }
    int i = 0, j = c.nk;
    do { int m = (i + j) >> 1; if (u < x[m]) j = m; else i = m; } while (j > i + 1);
    const double dx = u - x[i];
    v = y[i] + dx * (b[i] + dx * (cc[i] + dx * d[i]));
    v = v < c.lo ? c.lo : v;
    v = v > c.hi ? c.hi : v;
  }
  return c.db ? (double)exp2f((float)(v * 0.1)) : v;  // 2^(dB/10); fp32 exp2 (rel. err ~1e-7)
}

// contour_at for a caller-held interval cursor i (start at -1) and k increasing
// between calls: the first call bisects (as contour_at), later calls step forward,
// finding the same interval (the largest i with x[i] <= u) in ~1 load instead of
// log2(nk) dependent loads.
__device__ __forceinline__ double contour_at_cursor(const SgContour& c, const double* __restrict__ ck, int64_t L,
                                                    int64_t k, int& i) {
  if (c.kind != 3) return contour_at(c, ck, L, k);
  const double* x = ck + c.k_off;
  const double* y = x + c.nk;
  const double* b = y + c.nk;
  const double* cc = b + c.nk;
  const double* d = cc + c.nk;
  double u;
  if (k == 0) u = c.a;
  else if (k == L - 1) u = c.b;
  else {
    const double by = L == c.L ? c.by : (c.b - c.a) / (double)(L - 1);
    u = (k < L / 2) ? c.a + (double)k * by : c.b - (double)(L - 1 - k) * by;
  }
  if (i < 0) {
    int a = 0, j = c.nk;
    do { int m = (a + j) >> 1; if (u < x[m]) j = m; else a = m; } while (j > a + 1);
    i = a;
  } else {
    while (i + 1 <= c.nk - 1 && x[i + 1] <= u) ++i;
  }
  const double dx = u - x[i];
  double v = y[i] + dx * (b[i] + dx * (cc[i] + dx * d[i]));
  v = v < c.lo ? c.lo : v;
  v = v > c.hi ? c.hi : v;
  return c.db ? (double)exp2f((float)(v * 0.1)) : v;
}

__device__ __forceinline__ double linear_at(const SgLinear& l, const double* __restrict__ ck, int64_t L, int64_t k) {
  const double* x = ck + l.k_off;
  const double* y = x + l.nk;
  double u;
  if (k == 0) u = l.x0;
  else if (k == L - 1) u = l.x1;
  else {
    const double by = (l.x1 - l.x0) / (double)(L - 1);
    u = (k < L / 2) ? l.x0 + (double)k * by : l.x1 - (double)(L - 1 - k) * by;
  }
  int i = 0, j = l.nk - 1;
  while (i < j - 1) { int ij = (i + j) >> 1; if (u < x[ij]) j = ij; else i = ij; }
  if (u == x[j]) return y[j];
  if (u == x[i]) return y[i];
  return y[i] + (y[j] - y[i]) * ((u - x[i]) / (x[j] - x[i]));
}

// linear_at for monotonically increasing k with a caller-held interval
// cursor i (start at -1): same interval as the bisection above (largest i in
// [0, nk - 2] with x[i] <= u), found by bisection once, then by stepping.
__device__ __forceinline__ double linear_at_cursor(const SgLinear& l, const double* __restrict__ ck, int64_t L,
                                                   int64_t k, int& i) {
  const double* x = ck + l.k_off;
  const double* y = x + l.nk;
  double u;
  if (k == 0) u = l.x0;
  else if (k == L - 1) u = l.x1;
  else {
    const double by = (l.x1 - l.x0) / (double)(L - 1);
    u = (k < L / 2) ? l.x0 + (double)k * by : l.x1 - (double)(L - 1 - k) * by;
  }
  if (i < 0) {
    int a = 0, b = l.nk - 1;
    while (a < b - 1) { int ab = (a + b) >> 1; if (u < x[ab]) b = ab; else a = ab; }
    i = a;
  } else {
    while (i + 1 <= l.nk - 2 && x[i + 1] <= u) ++i;
  }
  const int j = i + 1;
  if (u == x[j]) return y[j];
  if (u == x[i]) return y[i];
  return y[i] + (y[j] - y[i]) * ((u - x[i]) / (x[j] - x[i]));
}

// Max over the wavefront, in every lane: DPP within each 16-lane row (quad_perm
// [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror), then the four rows' values by
// readlane. All VALU: the __shfl_xor form took six ds_bpermute round trips through
// the LDS per reduction (round 6; each short-task sine-bank wave reduces twice).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  const int x = __builtin_bit_cast(int, v);
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(x, x, CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float wave_max(float v) {
#ifdef SG_WAVE_MAX_SHFL
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
#else
  v = fmaxf(v, dpp_f<0xB1>(v));   // quad_perm [1,0,3,2]
  v = fmaxf(v, dpp_f<0x4E>(v));   // quad_perm [2,3,0,1]
  v = fmaxf(v, dpp_f<0x141>(v));  // row_half_mirror: max over 8 lanes
  v = fmaxf(v, dpp_f<0x140>(v));  // row_mirror: max over the row of 16
  const int x = __builtin_bit_cast(int, v);
  const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(x, 0));
  const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(x, 16));
  const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(x, 32));
  const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(x, 48));
  return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
#endif
}

// XCD-aware workgroup order: the dispatcher deals workgroups round-robin over
// the 8 XCDs (b and b + 8 share one, each XCD has its own L2), so consecutive
// workgroups -- which read neighbouring data, e.g. a glottal cycle's amplitude
// column A[i + 1] is also the next cycle's A[i] -- would fetch it from HBM on two
// L2s. This bijection of [0, n) gives each XCD a contiguous run of logical
// indices instead (cdna_hip_programming.md §5.5 T1, bijective for any n). Speed
// only: nothing depends on where a workgroup runs.
__device__ __forceinline__ uint32_t xcd_swizzle(uint32_t b, uint32_t n) {
  const uint32_t x = b & 7u, i = b >> 3, q = n >> 3, r = n & 7u;
  return x * q + (x < r ? x : r) + i;
}

}  // namespace sgd

