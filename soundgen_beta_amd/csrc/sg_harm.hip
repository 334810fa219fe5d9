// sg_harm.hip — gfx950 kernels of the additive harmonic source
// (generateHarmonics(), R/source.R:377-467).
//
// sg_sine_bank: one 256-sample tile per workgroup (4 wave64s). Per sample:
//   integr(u)  = closed-form prefix sum of the FMM pitch spline (fp64)
//   phi        = frac(integr / D) folded to |psi| <= 1/4 (sign sigma)
//   sin(r*phi) via Reinsch's stable 2-term recurrence (2 VALU ops/row)
//   amplitude  = approx() hat weights over the wave's 2-3 knot columns; the
//                columns are wave-uniform so every amplitude is a scalar
//                (SGPR) operand loaded by s_load: no LDS, no per-lane gathers
//   => 2 + C VALU ops per (sample, harmonic row), C = columns (2 or 3)
// It also produces the signed max of the syllable over its direct-copy
// window (the R normalisation waveform / max(waveform)).
#include <hip/hip_runtime.h>

#include "sg_dev.h"

namespace {

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
    else v = c.a + (double)k * ((c.b - c.a) / (double)(L - 1));
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
      const double by = (c.b - c.a) / (double)(L - 1);
      u = (k < L / 2) ? c.a + (double)k * by : c.b - (double)(L - 1 - k) * by;
    }
    int i = 0, j = c.nk;
    do { int m = (i + j) >> 1; if (u < x[m]) j = m; else i = m; } while (j > i + 1);
    const double dx = u - x[i];
    v = y[i] + dx * (b[i] + dx * (cc[i] + dx * d[i]));
    v = v < c.lo ? c.lo : v;
    v = v > c.hi ? c.hi : v;
  }
  return c.db ? exp2(v * 0.1) : v;
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

// Sum over rows with wave-uniform columns ia..ia+C-1 (amplitudes in SGPRs).
template <int C>
__device__ __forceinline__ float rows_uniform(const float* __restrict__ A, int R, int ia, int rel, float t,
                                              float s1, float lam, float sigma) {
  float acc_o[C], acc_e[C];
#pragma unroll
  for (int c = 0; c < C; ++c) { acc_o[c] = 0.f; acc_e[c] = 0.f; }
  float s = s1, d = s1;
  const float* __restrict__ col = A + (size_t)ia * R;
  for (int r0 = 0; r0 < R; r0 += 8) {
    float a[C][8];
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int q = 0; q < 8; ++q) a[c][q] = col[c * R + r0 + q];
#pragma unroll
    for (int q = 0; q < 8; q += 2) {
#pragma unroll
      for (int c = 0; c < C; ++c) acc_o[c] = fmaf(a[c][q], s, acc_o[c]);
      d = fmaf(lam, s, d);
      s = s + d;
#pragma unroll
      for (int c = 0; c < C; ++c) acc_e[c] = fmaf(a[c][q + 1], s, acc_e[c]);
      d = fmaf(lam, s, d);
      s = s + d;
    }
  }
  float y = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const float w = (c == rel) ? 1.f - t : ((c == rel + 1) ? t : 0.f);
    y = fmaf(w, fmaf(sigma, acc_o[c], acc_e[c]), y);
  }
  return y;
}

// Fallback when a wave spans > 3 knot columns (f0 near pitchCeiling):
// per-lane amplitude gathers.
__device__ __forceinline__ float rows_gather(const float* __restrict__ A, int R, int i, float t, float s1,
                                             float lam, float sigma) {
  const float* __restrict__ c0 = A + (size_t)i * R;
  const float* __restrict__ c1 = c0 + R;
  float ao = 0.f, ae = 0.f, s = s1, d = s1;
  for (int r = 0; r < R; r += 2) {
    const float a0 = c0[r], a1 = c1[r], b0 = c0[r + 1], b1 = c1[r + 1];
    ao = fmaf(fmaf(t, a1 - a0, a0), s, ao);
    d = fmaf(lam, s, d);
    s = s + d;
    ae = fmaf(fmaf(t, b1 - b0, b0), s, ae);
    d = fmaf(lam, s, d);
    s = s + d;
  }
  return fmaf(sigma, ao, ae);
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

}  // namespace

// sin(pi*x), cos(pi*x) for |x| <= 1/4 (|pi*x| <= pi/4): Taylor to x^9 / x^10,
// truncation < 2e-9, i.e. below fp32 rounding.
__device__ __forceinline__ void sincospi_q(float x, float& s, float& c) {
  const float a = 3.14159265358979f * x;
  const float a2 = a * a;
  s = a * fmaf(a2, fmaf(a2, fmaf(a2, fmaf(a2, 2.75573192e-6f, -1.98412698e-4f), 8.33333333e-3f), -1.66666667e-1f), 1.f);
  c = fmaf(a2, fmaf(a2, fmaf(a2, fmaf(a2, fmaf(a2, -2.75573192e-7f, 2.48015873e-5f), -1.38888889e-3f),
                          4.16666667e-2f), -0.5f), 1.f);
}

extern "C" __global__ __launch_bounds__(256) void sg_sine_bank(
    const SgTile* __restrict__ tiles, const SgEpoch* __restrict__ epochs, const SgSeg* __restrict__ segs,
    const double* __restrict__ knots, const float* __restrict__ amps, const SgSyllable* __restrict__ syls,
    const double* __restrict__ cknots, float* __restrict__ W, unsigned* __restrict__ maxes) {
  const SgTile tl = tiles[blockIdx.x];
  const SgEpoch ep = epochs[tl.epoch];
  const double* __restrict__ kn = knots + ep.knot_off;
  const SgSeg* __restrict__ sg = segs + ep.seg_off;
  const float* __restrict__ A = amps + ep.amp_off;
  const int half = ep.n >> 1;
  int i = tl.i0, k = tl.k0;
  float tmax = 0.f;
  const bool env = ep.dj1 > ep.dj0 && syls[ep.syl].env.kind != 0;
#pragma unroll 1
  for (int q = 0; q < SG_SINE_TILE / 256; ++q) {
    const int jw = tl.j0 + q * 256;  // wave-group base (uniform)
    if (jw >= ep.n) break;
    const int j = jw + (int)threadIdx.x;
    const bool valid = j < ep.n;
    const int jc = valid ? j : ep.n - 1;
    // amplitude interval: approx() at xo = seq.int(x1, xG, n)[j]
    const double xo = (jc == ep.n - 1) ? ep.xG
                      : (jc < half ? fma((double)jc, ep.xby, ep.x1) : fma(-(double)(ep.n - 1 - jc), ep.xby, ep.xG));
    while (i < ep.G - 2 && kn[i + 1] <= xo) ++i;
    const double xa = kn[i], xb = kn[i + 1];
    const float t = (xo == xb) ? 1.f : ((xo == xa) ? 0.f : (float)(xo - xa) / (float)(xb - xa));
    // phase: integr(u) = cumsum(pitch_up)[u] / sr in closed form per segment
    const double u = (double)(ep.u0 + jc);
    while (k + 1 < ep.nseg && sg[k + 1].t0 < u) ++k;
    const SgSeg S = sg[k];
    const double m = u - S.t0;
    const double S1 = m * (m + 1.0) * 0.5;
    const double S2 = S1 * fma(2.0, m, 1.0) * (1.0 / 3.0);
    const double P = fma(S.d, S1 * S1, fma(S.c, S2, fma(S.b, S1, fma(S.y, m, S.prefix))));
    const double v = P * ep.inv_srD;
    double ph = v - floor(v);
    if (ph >= 0.5) ph -= 1.0;
    float sigma = 1.f;
    if (ph > 0.25) { ph -= 0.5; sigma = -1.f; }
    else if (ph < -0.25) { ph += 0.5; sigma = -1.f; }
    float sh, ch;
    sincospi_q((float)ph, sh, ch);
    const float s1 = 2.f * sh * ch;    // sin(2*pi*psi)
    const float lam = -4.f * sh * sh;  // 2cos(2*pi*psi) - 2 without cancellation
    // wave-uniform knot columns
    const int ia = __builtin_amdgcn_readfirstlane(i);
    const int ib = __builtin_amdgcn_readfirstlane(__shfl(i, 63));
    const int ncol = ib - ia + 2;
    float y;
    if (ncol == 2) y = rows_uniform<2>(A, ep.R, ia, i - ia, t, s1, lam, sigma);
    else if (ncol == 3) y = rows_uniform<3>(A, ep.R, ia, i - ia, t, s1, lam, sigma);
    else y = rows_gather(A, ep.R, i, t, s1, lam, sigma);
    if (valid) {
      W[ep.w_off + j] = y;
      if (j >= ep.dj0 && j < ep.dj1) {
        float cand = y;
        if (env) {
          const SgSyllable& sy = syls[ep.syl];
          cand = (float)((double)y * contour_at(sy.env, cknots, sy.L, ep.dk0 + j));
        }
        tmax = fmaxf(tmax, cand);
      }
    }
  }
  // fused normalisation max over the direct-copy window
  if (ep.dj1 > ep.dj0) {
    __shared__ float red[4];
    const float wm = wave_max(tmax);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = wm;
    __syncthreads();
    if (threadIdx.x == 0) {
      const float bm = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
      if (bm > 0.f) atomicMax(maxes + syls[ep.syl].max_slot, __float_as_uint(bm));
    }
  }
}

namespace {
__device__ __forceinline__ float piece_value(const SgPiece& p, const float* __restrict__ W, int64_t q) {
  if (p.nterms < 0) return W[p.t[0].src + q];
  float v = 0.f;
  const float qf = (float)q;
  for (int t = 0; t < p.nterms; ++t)
    v = fmaf(fmaf(qf, fmaf(qf, p.t[t].w2, p.t[t].w1), p.t[t].w0), W[p.t[t].src + q], v);
  return v;
}
}  // namespace

// max over crossfade pieces (multi-term); tiles list (syl, piece, q0)
extern "C" __global__ __launch_bounds__(256) void sg_piece_max(
    const SgSylTile* __restrict__ ptiles, const SgPiece* __restrict__ pieces, const SgSyllable* __restrict__ syls,
    const double* __restrict__ cknots, const float* __restrict__ W, unsigned* __restrict__ maxes) {
  const SgSylTile tl = ptiles[blockIdx.x];
  const SgPiece& p = pieces[tl.piece];
  const SgSyllable& sy = syls[tl.syl];
  const int64_t q = tl.k0 + threadIdx.x;
  float cand = 0.f;
  if (q < p.len) {
    cand = piece_value(p, W, q);
    if (sy.env.kind != 0) cand = (float)((double)cand * contour_at(sy.env, cknots, sy.L, p.start + q));
  }
  __shared__ float red[4];
  const float wm = wave_max(cand);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = wm;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float bm = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    if (bm > 0.f) atomicMax(maxes + sy.max_slot, __float_as_uint(bm));
  }
}

// out[k] = assembled[k] * env[k] / max * fade[k] * drift[k]   (R/source.R:436-467)
// Each thread owns 4 consecutive samples; a tile lying inside one direct
// piece with a 16-B aligned source and destination moves float4s.
__device__ __forceinline__ float fade_at(int lf, int64_t L, int64_t k) {
  float f = 1.f;
  const float by = 1.f / (float)(lf - 1);
  if (k < lf) f *= (k == lf - 1) ? 1.f : (float)k * by;
  const int64_t kb = L - 1 - k;
  if (kb < lf) f *= (kb == lf - 1) ? 1.f : (float)kb * by;
  return f;
}

extern "C" __global__ __launch_bounds__(256) void sg_harm_finalize(
    const SgSylTile* __restrict__ stiles, const SgPiece* __restrict__ pieces, const SgSyllable* __restrict__ syls,
    const double* __restrict__ cknots, const float* __restrict__ W, const unsigned* __restrict__ maxes,
    float* __restrict__ out) {
  const SgSylTile tl = stiles[blockIdx.x];
  const SgSyllable& sy = syls[tl.syl];
  const float inv_max = 1.f / __uint_as_float(maxes[sy.max_slot]);
  const int pend = sy.piece0 + sy.npiece;
  const int64_t kt = tl.k0 + 4 * (int64_t)threadIdx.x;
  const int64_t tile_end = tl.k0 + 1024 < sy.L ? tl.k0 + 1024 : sy.L;
  const SgPiece& p0 = pieces[tl.piece];
  const bool simple = sy.env.kind == 0 && sy.drift.nk == 0;
  // fast path: whole tile inside one direct piece, aligned, no env/drift
  if (simple && p0.nterms < 0 && p0.start <= tl.k0 && p0.start + p0.len >= tile_end &&
      ((sy.out_off + tl.k0) & 3) == 0 && ((p0.t[0].src + (tl.k0 - p0.start)) & 3) == 0) {
    if (kt >= tile_end) return;
    const float* src = W + p0.t[0].src + (kt - p0.start);
    float* dst = out + sy.out_off + kt;
    if (kt + 4 <= tile_end) {
      float4 v = *reinterpret_cast<const float4*>(src);
      v.x *= inv_max; v.y *= inv_max; v.z *= inv_max; v.w *= inv_max;
      if (sy.fade >= 2 && (kt < sy.fade || kt + 4 > sy.L - sy.fade)) {
        v.x *= fade_at(sy.fade, sy.L, kt); v.y *= fade_at(sy.fade, sy.L, kt + 1);
        v.z *= fade_at(sy.fade, sy.L, kt + 2); v.w *= fade_at(sy.fade, sy.L, kt + 3);
      }
      *reinterpret_cast<float4*>(dst) = v;
    } else {
      for (int64_t k = kt; k < tile_end; ++k) {
        float v = src[k - kt] * inv_max;
        if (sy.fade >= 2) v *= fade_at(sy.fade, sy.L, k);
        dst[k - kt] = v;
      }
    }
    return;
  }
  int p = tl.piece;
  for (int e = 0; e < 4; ++e) {
    const int64_t k = kt + e;
    if (k >= tile_end) break;
    while (p + 1 < pend && pieces[p + 1].start <= k) ++p;
    const SgPiece& pc = pieces[p];
    float v = pc.nterms == 0 ? 0.f : piece_value(pc, W, k - pc.start);
    if (sy.env.kind != 0) v = (float)((double)v * contour_at(sy.env, cknots, sy.L, k));
    v *= inv_max;
    if (sy.fade >= 2) v *= fade_at(sy.fade, sy.L, k);
    if (sy.drift.nk > 0) v = (float)((double)v * linear_at(sy.drift, cknots, sy.L, k));
    out[sy.out_off + k] = v;
  }
}

// ---------------------------------------------------------------- launchers
#include "sg_exec.h"
namespace sg {
void launch_sine_bank(const DevicePlan& D, int64_t n_tiles, hipStream_t s) {
  if (n_tiles <= 0) return;
  hipLaunchKernelGGL(sg_sine_bank, dim3((unsigned)n_tiles), dim3(256), 0, s, D.tiles, D.epochs, D.segs, D.knots,
                     D.amps, D.syls, D.cknots, D.W, D.maxes);
}
void launch_piece_max(const DevicePlan& D, int64_t n_ptiles, hipStream_t s) {
  if (n_ptiles <= 0) return;
  hipLaunchKernelGGL(sg_piece_max, dim3((unsigned)n_ptiles), dim3(256), 0, s, D.ptiles, D.pieces, D.syls, D.cknots,
                     D.W, D.maxes);
}
void launch_harm_finalize(const DevicePlan& D, int64_t n_stiles, float* out, hipStream_t s) {
  if (n_stiles <= 0) return;
  hipLaunchKernelGGL(sg_harm_finalize, dim3((unsigned)n_stiles), dim3(256), 0, s, D.syl_tiles, D.pieces, D.syls,
                     D.cknots, D.W, D.maxes, out);
}
}  // namespace sg
