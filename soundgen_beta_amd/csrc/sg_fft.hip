// sg_fft.hip — gfx950 kernels of the spectral part of the path:
//   seewave::stft (hamming) x spectral envelope -> seewave::istft (hanning OLA)
//     = the formant filter of soundgen(), R/soundgen.R:743-807
//   real random spectrum x filter -> seewave::istft
//     = generateNoise(), R/source.R:88-131
// (seewave_2.0.5.tar.gz::seewave/R/seewave.r:7782-7819 stft, :3447-3486 istft)
//
// sg_fft_frames: a workgroup transforms `fb` frames of one window length wl
// in LDS. A real length-wl transform is a complex M = wl/2 point transform
// (even/odd packing) + an O(M) untangling pass; the complex transform is a
// mixed-radix Stockham FFT (radices 2, 4 and odd primes <= 31, each butterfly
// in registers, symmetric form for odd primes: R-1 real FMAs per output).
// Filter frames go FFT -> /wl x env -> (seewave's Hermitian mirror with the
// Nyquist bin = Re(bin nr-1)) -> inverse -> /wl x hann; noise frames start
// from the real spectrum. Windowed frames go to scratch and sg_ola gathers
// the <= ceil(wl/h) frames covering each output sample (deterministic, no
// atomics), scales by h / sum(hann^2), trims/pads (matchLengths 'central')
// and writes per-tile maxima for the following normalisation.
#include <hip/hip_runtime.h>

#include "sg_dev.h"
#include "sg_devfn.h"
#include "sg_roots.h"

namespace {

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ float2 cmulc(float2 a, float2 b) {  // a * conj(b)
  return make_float2(fmaf(a.x, b.x, a.y * b.y), fmaf(a.y, b.x, -a.x * b.y));
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }

// R-point DFT in registers. INV: exp(+2 pi i rk / R), else exp(-2 pi i rk / R).
template <int R, bool INV>
struct Dft {
  // odd prime R: y_k = x0 + sum_m a_m cos - i sum_m b_m sin, a_m = x_m + x_{R-m}, b_m = x_m - x_{R-m}
  __device__ __forceinline__ static void run(float2 (&v)[R]) {
    constexpr int H = (R - 1) / 2;
    float2 a[H], b[H];
#pragma unroll
    for (int m = 1; m <= H; ++m) {
      a[m - 1] = cadd(v[m], v[R - m]);
      b[m - 1] = csub(v[m], v[R - m]);
    }
    const float2 x0 = v[0];
    float2 y0 = x0;
#pragma unroll
    for (int m = 0; m < H; ++m) y0 = cadd(y0, a[m]);
#pragma unroll
    for (int k = 1; k <= H; ++k) {
      float2 P = x0, Q = make_float2(0.f, 0.f);
#pragma unroll
      for (int m = 1; m <= H; ++m) {
        const int idx = (m * k) % R;
        const float c = SgRoots<R>::c(idx), s = SgRoots<R>::s(idx);
        P.x = fmaf(a[m - 1].x, c, P.x);
        P.y = fmaf(a[m - 1].y, c, P.y);
        Q.x = fmaf(b[m - 1].x, s, Q.x);
        Q.y = fmaf(b[m - 1].y, s, Q.y);
      }
      if (!INV) {  // -i Q = (Q.y, -Q.x)
        v[k] = make_float2(P.x + Q.y, P.y - Q.x);
        v[R - k] = make_float2(P.x - Q.y, P.y + Q.x);
      } else {
        v[k] = make_float2(P.x - Q.y, P.y + Q.x);
        v[R - k] = make_float2(P.x + Q.y, P.y - Q.x);
      }
    }
    v[0] = y0;
  }
};
template <bool INV>
struct Dft<2, INV> {
  __device__ __forceinline__ static void run(float2 (&v)[2]) {
    const float2 a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = csub(a, b);
  }
};
template <bool INV>
struct Dft<4, INV> {
  __device__ __forceinline__ static void run(float2 (&v)[4]) {
    const float2 s02 = cadd(v[0], v[2]), d02 = csub(v[0], v[2]);
    const float2 s13 = cadd(v[1], v[3]), d13 = csub(v[1], v[3]);
    v[0] = cadd(s02, s13);
    v[2] = csub(s02, s13);
    // forward: y1 = d02 - i d13, y3 = d02 + i d13 (inverse swapped)
    const float2 mid = make_float2(d13.y, -d13.x);  // -i d13
    if (!INV) {
      v[1] = cadd(d02, mid);
      v[3] = csub(d02, mid);
    } else {
      v[1] = csub(d02, mid);
      v[3] = cadd(d02, mid);
    }
  }
};

// ISTFT input packing: from the one-sided spectrum Y[0..M) (seewave's mirror:
// Xf[k] = Y[k], Xf[M] = Re(Y[M-1]), Xf[N-k] = conj(Y[k])) build
// Z'[k] = (Xf[k] + Xf[k+M]) + i (Xf[k] - Xf[k+M]) e^{2 pi i k / N}
// whose M-point inverse transform holds y[2n] + i y[2n+1].
__device__ __forceinline__ void pack_pair(float2 yk, float2 ymk, float2 wNk, float2& zk, float2& zmk) {
  // k: Xf[k + M] = conj(Y[M - k]);  M - k: Xf[M - k + M] = conj(Y[k])
  const float2 e = cadd(yk, cconj(ymk));
  const float2 d = csub(yk, cconj(ymk));
  const float2 o = cmulc(d, wNk);  // x e^{+2 pi i k/N}
  zk = make_float2(e.x - o.y, e.y + o.x);
  const float2 e2 = cadd(ymk, cconj(yk));
  const float2 d2 = csub(ymk, cconj(yk));
  const float2 o2 = make_float2(-(d2.x * wNk.x - d2.y * wNk.y), -(d2.x * wNk.y + d2.y * wNk.x));  // x (-W_N^k)
  zmk = make_float2(e2.x - o2.y, e2.y + o2.x);
}

// ---------------------------------------------------------------- FFT v2
// In-place Stockham pass over fb frames of M points held in ONE LDS buffer:
// phase 1 reads each butterfly (twiddled) into registers and reduces it to
// its state (odd primes: x0 and the symmetric sums a_m, b_m; radix 2/4: the
// outputs), barrier, phase 2 produces the outputs and writes them. With
// fb*M <= SG_FFT_SLOTS complex points and SG_FFT_THREADS threads, a thread
// owns at most NB = ceil(SG_FFT_SLOTS / (R * SG_FFT_THREADS)) butterflies.
constexpr int SG_FFT_THREADS = 512;
constexpr int SG_FFT_SLOTS = 8192;  // complex points per workgroup (64 KB of LDS)

template <int R>
struct NbOf {
  static constexpr int value = (SG_FFT_SLOTS / SG_FFT_THREADS + R - 1) / R;
};

template <int R, bool INV>
__device__ __forceinline__ void stage_ip(float2* X, int M, int Ns, const float2* __restrict__ twM, int fb) {
  constexpr int NB = NbOf<R>::value;
  constexpr bool ODD = (R % 2) == 1;
  constexpr int H = ODD ? (R - 1) / 2 : 1;
  const int MR = M / R;
  const int tstep = M / (Ns * R);
  const int total = fb * MR;
  float2 st[NB][ODD ? (2 * H + 1) : R];  // odd: [x0, a_1..a_H, b_1..b_H]; even radix: outputs
  int base_o[NB];
  bool live[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    const int idx = threadIdx.x + q * SG_FFT_THREADS;
    live[q] = idx < total;
    base_o[q] = 0;
    if (!live[q]) continue;
    const int f = idx / MR;
    const int j = idx - f * MR;
    const float2* x = X + f * M;
    float2 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = x[j + r * MR];
    const int jm = j % Ns;
    if (Ns > 1) {
#pragma unroll
      for (int r = 1; r < R; ++r) {
        const float2 w = twM[r * jm * tstep];
        v[r] = INV ? cmulc(v[r], w) : cmul(v[r], w);
      }
    }
    base_o[q] = f * M + (j - jm) * R + jm;
    if constexpr (ODD) {
      st[q][0] = v[0];
#pragma unroll
      for (int m = 1; m <= H; ++m) {
        st[q][m] = cadd(v[m], v[R - m]);
        st[q][H + m] = csub(v[m], v[R - m]);
      }
    } else {
      Dft<R, INV>::run(v);
#pragma unroll
      for (int r = 0; r < R; ++r) st[q][r] = v[r];
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    if (!live[q]) continue;
    float2* y = X + base_o[q];
    if constexpr (ODD) {
      const float2 x0 = st[q][0];
      float2 y0 = x0;
#pragma unroll
      for (int m = 1; m <= H; ++m) y0 = cadd(y0, st[q][m]);
      y[0] = y0;
#pragma unroll
      for (int k = 1; k <= H; ++k) {
        float2 P = x0, Q = make_float2(0.f, 0.f);
#pragma unroll
        for (int m = 1; m <= H; ++m) {
          const int id = (m * k) % R;
          const float c = SgRoots<R>::c(id), s = SgRoots<R>::s(id);
          P.x = fmaf(st[q][m].x, c, P.x);
          P.y = fmaf(st[q][m].y, c, P.y);
          Q.x = fmaf(st[q][H + m].x, s, Q.x);
          Q.y = fmaf(st[q][H + m].y, s, Q.y);
        }
        if (!INV) {
          y[k * Ns] = make_float2(P.x + Q.y, P.y - Q.x);
          y[(R - k) * Ns] = make_float2(P.x - Q.y, P.y + Q.x);
        } else {
          y[k * Ns] = make_float2(P.x - Q.y, P.y + Q.x);
          y[(R - k) * Ns] = make_float2(P.x + Q.y, P.y - Q.x);
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) y[r * Ns] = st[q][r];
    }
  }
  __syncthreads();
}

template <bool INV>
__device__ void fft_ip(float2* X, const SgFftGeom& g, const float2* __restrict__ twM, int fb) {
  int Ns = 1;
  for (int s = 0; s < g.nstages; ++s) {
    const int R = g.radix[s];
    switch (R) {
      case 2: stage_ip<2, INV>(X, g.M, Ns, twM, fb); break;
      case 3: stage_ip<3, INV>(X, g.M, Ns, twM, fb); break;
      case 4: stage_ip<4, INV>(X, g.M, Ns, twM, fb); break;
      case 5: stage_ip<5, INV>(X, g.M, Ns, twM, fb); break;
      case 7: stage_ip<7, INV>(X, g.M, Ns, twM, fb); break;
      case 11: stage_ip<11, INV>(X, g.M, Ns, twM, fb); break;
      case 13: stage_ip<13, INV>(X, g.M, Ns, twM, fb); break;
      case 17: stage_ip<17, INV>(X, g.M, Ns, twM, fb); break;
      case 19: stage_ip<19, INV>(X, g.M, Ns, twM, fb); break;
      case 23: stage_ip<23, INV>(X, g.M, Ns, twM, fb); break;
      case 29: stage_ip<29, INV>(X, g.M, Ns, twM, fb); break;
      case 31: stage_ip<31, INV>(X, g.M, Ns, twM, fb); break;
      default: break;  // the planner only emits the radices above
    }
    Ns *= R;
  }
}

}  // namespace

extern "C" __global__ __launch_bounds__(SG_FFT_THREADS) void sg_fft_frames(
    const SgFrameGroup* __restrict__ groups, const SgFrame* __restrict__ frames, const SgFftGeom* __restrict__ geoms,
    const float* __restrict__ fl, float* __restrict__ fs) {
  extern __shared__ float4 lds4[];
  float2* A = reinterpret_cast<float2*>(lds4);
  const SgFrameGroup G = groups[blockIdx.x];
  const SgFftGeom& g = geoms[G.geom];
  const int M = g.M, N = g.wl, fb = G.nf;
  const float2* twM = reinterpret_cast<const float2*>(fl + g.tw);  // L1/L2 resident
  const float2* twN = twM + M;
  const float* ham = fl + g.win;
  const float* han = ham + N;
  const float invN = 1.f / (float)N;
  const int half = M / 2;
  const int npairs = fb * (half + 1);
  constexpr int NP = SG_FFT_SLOTS / 2 / SG_FFT_THREADS + 1;  // pairs per thread
  if (G.mode == SG_FRAME_FILTER) {
    for (int idx = threadIdx.x; idx < fb * M; idx += SG_FFT_THREADS) {
      const int f = idx / M, n = idx - f * M;
      const float* s = fs + frames[G.f0 + f].src;
      A[idx] = make_float2(s[2 * n] * ham[2 * n], s[2 * n + 1] * ham[2 * n + 1]);
    }
    __syncthreads();
    fft_ip<false>(A, g, twM, fb);
    // untangle the real transform: X[k] = E + W_N^k O, E = (Z_k + conj Z_{M-k})/2,
    // O = -i (Z_k - conj Z_{M-k}) / 2; Y = X / N * env; pack for the inverse
    float2 zk[NP], zm[NP], zh[NP];
    int pk[NP], pf[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const int idx = threadIdx.x + q * SG_FFT_THREADS;
      pk[q] = -1;
      if (idx >= npairs) continue;
      const int f = idx / (half + 1), k = idx - f * (half + 1);
      if (k != 0 && k >= M - k) continue;
      pk[q] = k;
      pf[q] = f;
      const float2* z = A + f * M;
      const float* env = fl + frames[G.f0 + f].env;
      auto X_at = [&](int kk) -> float2 {
        const float2 a = z[kk], b = z[(M - kk) % M];
        const float2 e = make_float2(0.5f * (a.x + b.x), 0.5f * (a.y - b.y));
        const float2 dd = make_float2(a.x - b.x, a.y + b.y);
        const float2 o = make_float2(0.5f * dd.y, -0.5f * dd.x);
        return cadd(e, cmul(o, twN[kk]));
      };
      if (k == 0) {
        const float2 x0 = X_at(0), xl = X_at(M - 1);
        const float y0 = x0.x * invN * env[0];
        const float nyq = xl.x * invN * env[M - 1];
        zk[q] = make_float2(y0 + nyq, y0 - nyq);
        if (M % 2 == 0) {
          const float2 xk = X_at(half);
          const float2 yk = make_float2(xk.x * invN * env[half], xk.y * invN * env[half]);
          float2 t2;
          pack_pair(yk, yk, twN[half], zh[q], t2);
        }
      } else {
        const float2 xk = X_at(k), xm = X_at(M - k);
        const float2 yk = make_float2(xk.x * invN * env[k], xk.y * invN * env[k]);
        const float2 ym = make_float2(xm.x * invN * env[M - k], xm.y * invN * env[M - k]);
        pack_pair(yk, ym, twN[k], zk[q], zm[q]);
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      if (pk[q] < 0) continue;
      float2* out = A + pf[q] * M;
      const int k = pk[q];
      out[k] = zk[q];
      if (k == 0) {
        if (M % 2 == 0) out[half] = zh[q];
      } else {
        out[M - k] = zm[q];
      }
    }
    __syncthreads();
  } else {  // SG_FRAME_NOISE: real spectrum u * filter, packed straight into LDS
    for (int idx = threadIdx.x; idx < npairs; idx += SG_FFT_THREADS) {
      const int f = idx / (half + 1), k = idx - f * (half + 1);
      const SgFrame& F = frames[G.f0 + f];
      const float* u = fl + F.src;
      const float* flt = fl + F.env;
      float2* out = A + f * M;
      if (k == 0) {
        const float y0 = u[0] * flt[0], nyq = u[M - 1] * flt[M - 1];
        out[0] = make_float2(y0 + nyq, y0 - nyq);
        if (M % 2 == 0) {
          const float2 yk = make_float2(u[half] * flt[half], 0.f);
          float2 a, b;
          pack_pair(yk, yk, twN[half], a, b);
          out[half] = a;
        }
      } else if (k < M - k) {
        const float2 yk = make_float2(u[k] * flt[k], 0.f), ym = make_float2(u[M - k] * flt[M - k], 0.f);
        float2 a, b;
        pack_pair(yk, ym, twN[k], a, b);
        out[k] = a;
        out[M - k] = b;
      }
    }
    __syncthreads();
  }
  fft_ip<true>(A, g, twM, fb);
  // windowed frame: Re(ifft)/N x hann, y[2n] = Re z[n], y[2n+1] = Im z[n]
  for (int idx = threadIdx.x; idx < fb * M; idx += SG_FFT_THREADS) {
    const int f = idx / M, n = idx - f * M;
    const float2 v = A[idx];
    float* d = fs + frames[G.f0 + f].dst;
    d[2 * n] = v.x * invN * han[2 * n];
    d[2 * n + 1] = v.y * invN * han[2 * n + 1];
  }
}

using sgd::contour_at;
__device__ __forceinline__ float wave_max_f(float v) { return sgd::wave_max(v); }

// Overlap-add gather: out[q] = scale * sum over frames f covering sample
// p = first + q of frame_f[p - floor(f h)], zero outside [0, xlen).
extern "C" __global__ __launch_bounds__(256) void sg_ola(const SgOlaTile* __restrict__ tiles,
                                                         const SgOla* __restrict__ olas, float* __restrict__ fs,
                                                         float* __restrict__ tilemax) {
  const SgOlaTile T = tiles[blockIdx.x];
  const SgOla& O = olas[T.ola];
  float m = -INFINITY;
  for (int e = 0; e < SG_OLA_TILE / 256; ++e) {
    const int64_t q = T.q0 + e * 256 + threadIdx.x;
    if (q >= O.len) break;
    const int64_t p = O.first + q;
    float acc = 0.f;
    if (p >= 0 && p < O.xlen) {
      // frames f with floor(f h) <= p < floor(f h) + wl
      int64_t fhi = (int64_t)floor((double)p / O.h);
      if (fhi > O.nframes - 1) fhi = O.nframes - 1;
      while (fhi > 0 && (int64_t)floor((double)fhi * O.h) > p) --fhi;
      for (int64_t f = fhi; f >= 0; --f) {
        const int64_t b = (int64_t)floor((double)f * O.h);
        const int64_t i = p - b;
        if (i >= O.wl) break;
        acc += fs[O.frames + f * O.wl + i];
      }
      acc *= O.scale;
    }
    fs[O.out + q] = acc;
    m = fmaxf(m, acc);
  }
  __shared__ float red[4];
  m = wave_max_f(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) tilemax[blockIdx.x] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// max over consecutive tile slots of each OLA
extern "C" __global__ __launch_bounds__(64) void sg_ola_max(const SgOla* __restrict__ olas, int n_olas,
                                                            const float* __restrict__ tilemax,
                                                            float* __restrict__ olamax) {
  const int o = blockIdx.x;
  if (o >= n_olas) return;
  const SgOla& O = olas[o];
  const int nt = (int)((O.len + SG_OLA_TILE - 1) / SG_OLA_TILE);
  float m = -INFINITY;
  for (int i = threadIdx.x; i < nt; i += 64) m = fmaxf(m, tilemax[O.tile0 + i]);
  m = wave_max_f(m);
  if (threadIdx.x == 0) olamax[o] = m;
}

// Output assembly (addVectors / envelopes / AM trill / normalisation),
// R/soundgen.R:699-842 and generateNoise()'s tail R/source.R:124-131.
__device__ __forceinline__ float sigmoid_at(const float* __restrict__ tab, int lo, int64_t k) {
  const int64_t r = k % (2 * (int64_t)lo);
  return r < lo ? tab[r] : tab[2 * lo - 1 - r];
}

__device__ __forceinline__ float fade_in_out(int lf, int64_t L, int64_t k) {  // fadeInOut(), R/utilities_soundgen.R:440-459
  float f = 1.f;
  if (lf < 2) return f;
  const float by = 1.f / (float)(lf - 1);
  if (k < lf) f *= (k == lf - 1) ? 1.f : (float)k * by;
  const int64_t kb = L - 1 - k;
  if (kb < lf) f *= (kb == lf - 1) ? 1.f : (float)kb * by;
  return f;
}

extern "C" __global__ __launch_bounds__(256) void sg_mix(const SgMixTile* __restrict__ tiles,
                                                         const SgMix* __restrict__ mixes,
                                                         const SgNoiseItem* __restrict__ items,
                                                         const float* __restrict__ olamax,
                                                         const double* __restrict__ cknots,
                                                         const float* __restrict__ fl, float* __restrict__ fs,
                                                         float* __restrict__ out) {
  const SgMixTile T = tiles[blockIdx.x];
  const SgMix& X = mixes[T.mix];
  float* __restrict__ dst = X.to_fs ? fs : out;
  for (int e = 0; e < SG_MIX_TILE / 256; ++e) {
    const int64_t k = T.k0 + e * 256 + threadIdx.x;
    if (k >= X.len) break;
    float v = 0.f;
    if (X.base_kind != SG_BASE_NONE && k < X.base_len) {
      v = fs[X.base + k];
      if (X.base_kind == SG_BASE_NORM) v = v / olamax[X.base_ola];
    }
    for (int i = 0; i < X.nitems; ++i) {
      const SgNoiseItem& it = items[X.item0 + i];
      const int64_t j = k - it.off;
      if (j < 0 || j >= it.len) continue;
      float nv = fs[it.raw + j];
      if (it.ola >= 0) nv = nv / olamax[it.ola];
      if (it.strength.kind != 0) nv = (float)((double)nv * contour_at(it.strength, cknots, it.len, j));
      nv *= fade_in_out(it.fade, it.len, j);
      v += nv;
    }
    if (X.mult.kind != 0) v = (float)((double)v * contour_at(X.mult, cknots, X.len, k));
    if (X.am_lo > 0) v *= 1.f - sigmoid_at(fl + X.am_tab, X.am_lo, k) * X.am_dep / 100.f;
    dst[X.dst + k] = v;
  }
}

// ---------------------------------------------------------------- launchers
#include "sg_exec.h"
namespace sg {
void launch_fft_frames(const DevicePlan& D, int64_t g0, int64_t n_groups, int lds_bytes, hipStream_t s) {
  if (n_groups <= 0) return;
  hipLaunchKernelGGL(sg_fft_frames, dim3((unsigned)n_groups), dim3(SG_FFT_THREADS), lds_bytes, s, D.fgroups + g0,
                     D.frames,
                     D.geoms, D.fl, D.fs);
}
void launch_ola(const DevicePlan& D, int64_t t0, int64_t n_tiles, int64_t o0, int64_t n_olas, hipStream_t s) {
  if (n_tiles <= 0) return;
  hipLaunchKernelGGL(sg_ola, dim3((unsigned)n_tiles), dim3(256), 0, s, D.olatiles + t0, D.olas, D.fs,
                     D.olatilemax + t0);
  hipLaunchKernelGGL(sg_ola_max, dim3((unsigned)n_olas), dim3(64), 0, s, D.olas + o0, (int)n_olas, D.olatilemax,
                     D.olamax + o0);
}
void launch_mix(const DevicePlan& D, int64_t t0, int64_t n_tiles, float* out, hipStream_t s) {
  if (n_tiles <= 0) return;
  hipLaunchKernelGGL(sg_mix, dim3((unsigned)n_tiles), dim3(256), 0, s, D.mixtiles + t0, D.mixes, D.items, D.olamax,
                     D.cknots, D.fl, D.fs, out);
}
}  // namespace sg
