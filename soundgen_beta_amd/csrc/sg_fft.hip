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

#include <type_traits>

#include "sg_dev.h"
#include "sg_devfn.h"
#include "sg_roots.h"

namespace {

// Complex values as packed fp32 pairs: gfx950 issues v_pk_fma_f32 / v_pk_mul_f32 /
// v_pk_add_f32 on (re, im) in one instruction, halving the VALU work of the
// butterflies (the odd-prime sums multiply both halves by one real root).
typedef float v2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ v2 V(float2 a) { return v2{a.x, a.y}; }
__device__ __forceinline__ float2 F(v2 a) { return make_float2(a.x, a.y); }
__device__ __forceinline__ v2 pfma(v2 a, v2 b, v2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ v2 splat(float c) { return v2{c, c}; }
// The swizzles and sign flips of a complex product fold into the VOP3P
// op_sel / neg modifiers (the compiler emits separate moves and xors for them)
__device__ __forceinline__ v2 vmul(v2 a, v2 w) {  // a * w = a.x w + a.y (-w.y, w.x)
  v2 t, r;
  __asm__("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(a), "v"(w));
  __asm__("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
          : "=v"(r) : "v"(a), "v"(w), "v"(t));
  return r;
}
__device__ __forceinline__ v2 vmulc(v2 a, v2 w) {  // a * conj(w) = a.x (w.x, -w.y) + a.y (w.y, w.x)
  v2 t, r;
  __asm__("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1] neg_hi:[0,1]" : "=v"(t) : "v"(a), "v"(w));
  __asm__("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1]" : "=v"(r) : "v"(a), "v"(w), "v"(t));
  return r;
}
__device__ __forceinline__ v2 add_miq(v2 p, v2 q) {  // p - i q = (p.x + q.y, p.y - q.x)
  v2 r;
  __asm__("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(p), "v"(q));
  return r;
}
__device__ __forceinline__ v2 add_piq(v2 p, v2 q) {  // p + i q = (p.x - q.y, p.y + q.x)
  v2 r;
  __asm__("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(p), "v"(q));
  return r;
}
__device__ __forceinline__ v2 add_conjb(v2 a, v2 b) {  // a + conj b = (a.x + b.x, a.y - b.y)
  v2 r;
  __asm__("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ v2 sub_conjb(v2 a, v2 b) {  // a - conj b = (a.x - b.x, a.y + b.y)
  v2 r;
  __asm__("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float2 cmul(float2 a, float2 b) { return F(vmul(V(a), V(b))); }
__device__ __forceinline__ float2 cmulc(float2 a, float2 b) { return F(vmulc(V(a), V(b))); }
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return F(V(a) + V(b)); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return F(V(a) - V(b)); }
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }

// Outputs k and R - k of an odd-prime butterfly from its symmetric sums
// (st = [x0, a_1..a_H, b_1..b_H]): P = x0 + sum_m a_m cos(2 pi mk/R),
// Q = sum_m b_m sin(2 pi mk/R); forward y_k = P - iQ, y_{R-k} = P + iQ.
template <int R, bool INV>
__device__ __forceinline__ void odd_out(const v2 (&st)[R], int k, v2& yk, v2& ymk) {
  constexpr int H = (R - 1) / 2;
  v2 P = st[0], Q = v2{0.f, 0.f};
#pragma unroll
  for (int m = 1; m <= H; ++m) {
    const int id = (m * k) % R;
    P = pfma(st[m], splat(SgRoots<R>::c(id)), P);
    Q = pfma(st[H + m], splat(SgRoots<R>::s(id)), Q);
  }
  yk = INV ? add_piq(P, Q) : add_miq(P, Q);
  ymk = INV ? add_miq(P, Q) : add_piq(P, Q);
}

// R-point DFT in registers. INV: exp(+2 pi i rk / R), else exp(-2 pi i rk / R).
template <int R, bool INV>
struct Dft {
  // odd prime R: y_k = x0 + sum_m a_m cos - i sum_m b_m sin, a_m = x_m + x_{R-m}, b_m = x_m - x_{R-m}
  __device__ __forceinline__ static void run(float2 (&v)[R]) {
    constexpr int H = (R - 1) / 2;
    v2 st[R];
    st[0] = V(v[0]);
    v2 y0 = st[0];
#pragma unroll
    for (int m = 1; m <= H; ++m) {
      st[m] = V(v[m]) + V(v[R - m]);
      st[H + m] = V(v[m]) - V(v[R - m]);
      y0 += st[m];
    }
#pragma unroll
    for (int k = 1; k <= H; ++k) {
      v2 a, b;
      odd_out<R, INV>(st, k, a, b);
      v[k] = F(a);
      v[R - k] = F(b);
    }
    v[0] = F(y0);
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

// exact n / d for n * d < 2^32 with magic = ceil(2^32 / d) (planner), magic 0 <=> d == 1
__device__ __forceinline__ int udiv(int n, uint32_t magic) {
  return magic ? (int)__umulhi((uint32_t)n, magic) : n;
}

// twS: the geometry's stage-ordered twiddles (SgFftGeom::tws: stage s with stride Ns
// holds W_{Ns R}^{q jm} at Ns - 1 + (q - 1) Ns + jm), so that consecutive butterflies
// read consecutive entries (a W_M table read at q jm M / (Ns R) put every lane of an
// early stage in the same LDS bank)
template <int R, bool INV>
__device__ __forceinline__ void stage_ip(float2* X, int M, int Ns, const float2* twS, int fb, uint32_t mr_magic,
                                         uint32_t ns_magic) {
  constexpr int NB = NbOf<R>::value;
  constexpr bool ODD = (R % 2) == 1;
  constexpr int H = ODD ? (R - 1) / 2 : 1;
  const int MR = M / R;
  const int total = fb * MR;
  v2 st[NB][R];  // odd: [x0, a_1..a_H, b_1..b_H]; even radix: outputs
  int base_o[NB];
  bool live[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    const int idx = threadIdx.x + q * SG_FFT_THREADS;
    live[q] = idx < total;
    base_o[q] = 0;
    if (!live[q]) continue;
    const int f = udiv(idx, mr_magic);
    const int j = idx - f * MR;
    const float2* x = X + f * M;
    float2 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = x[j + r * MR];
    const int jm = j - udiv(j, ns_magic) * Ns;
    if (Ns > 1) {
      const float2* tw = twS + (Ns - 1) + jm;
#pragma unroll
      for (int r = 1; r < R; ++r) {
        const float2 w = tw[(r - 1) * Ns];
        v[r] = INV ? cmulc(v[r], w) : cmul(v[r], w);
      }
    }
    base_o[q] = f * M + (j - jm) * R + jm;
    if constexpr (ODD) {
      st[q][0] = V(v[0]);
#pragma unroll
      for (int m = 1; m <= H; ++m) {
        st[q][m] = V(v[m]) + V(v[R - m]);
        st[q][H + m] = V(v[m]) - V(v[R - m]);
      }
    } else {
      Dft<R, INV>::run(v);
#pragma unroll
      for (int r = 0; r < R; ++r) st[q][r] = V(v[r]);
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    if (!live[q]) continue;
    float2* y = X + base_o[q];
    if constexpr (ODD) {
      v2 y0 = st[q][0];
#pragma unroll
      for (int m = 1; m <= H; ++m) y0 += st[q][m];
      y[0] = F(y0);
#pragma unroll
      for (int k = 1; k <= H; ++k) {
        v2 a, b;
        odd_out<R, INV>(st[q], k, a, b);
        y[k * Ns] = F(a);
        y[(R - k) * Ns] = F(b);
      }
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) y[r * Ns] = F(st[q][r]);
    }
  }
  __syncthreads();
}

template <bool INV>
__device__ void fft_ip(float2* X, const SgFftGeom& g, const float2* twS, int fb) {
  int Ns = 1;
  for (int s = 0; s < g.nstages; ++s) {
    const int R = g.radix[s];
    const uint32_t mm = g.mr_magic[s], nm = g.ns_magic[s];
    int Ms = g.M;
    Ms = __builtin_amdgcn_readfirstlane(Ms);  // wave-uniform also when called out of line
    switch (R) {
#define SG_STAGE(RR) \
      case RR: stage_ip<RR, INV>(X, Ms, Ns, twS, fb, mm, nm); break;
      SG_STAGE(2) SG_STAGE(3) SG_STAGE(4) SG_STAGE(5) SG_STAGE(7) SG_STAGE(11) SG_STAGE(13) SG_STAGE(17)
      SG_STAGE(19) SG_STAGE(23) SG_STAGE(29) SG_STAGE(31)
#undef SG_STAGE
      default: break;  // the planner only emits the radices above
    }
    Ns *= R;
  }
}

// ---------------------------------------------------------------- FFT v3
// One wavefront transforms one frame: no workgroup barriers between stages.
// A wavefront's LDS operations complete in issue order, so the in-place pass
// only has to keep the compiler from moving the phase-2 writes above the
// phase-1 reads (sg_wave_fence). A lane owns ceil(M / R / 64) <= 32 / R
// butterflies of a stage (planner: SG_FFT_WAVE geometries).
__device__ __forceinline__ void sg_wave_fence() { __asm__ __volatile__("" ::: "memory"); }

template <int R>
struct NbW {
  static constexpr int value = SG_WAVE_STATE / R > 0 ? SG_WAVE_STATE / R : 1;
};

#ifndef SG_R19_REMAP
#define SG_R19_REMAP 1
#endif
// CM, CNS > 0: the frame size and the stage's stride are compile-time constants
// (the dominant geometry's specialisation: index math folds away)
template <int R, bool INV, int CM = 0, int CNS = 0>
__device__ __forceinline__ void stage_w(float2* X, int M_, int Ns_, const float2* twS, uint32_t ns_magic, int lane) {
  constexpr int NB = NbW<R>::value;
  constexpr bool ODD = (R % 2) == 1;
  constexpr int H = ODD ? (R - 1) / 2 : 1;
  const int M = CM ? CM : M_, Ns = CNS ? CNS : Ns_;
  const int MR = M / R;
  // HALVES: a stride of <= 32 butterflies with two blocks (MR = 2 Ns; M = 1102's
  // radix-19 stage: Ns = 29): lane half h takes block h, jm = lane & 31, so a
  // 16-lane quarter's ds_write_b64 never straddles the two blocks' outputs (lanes
  // 29..31 and 61..63 idle; with j = lane, lanes 29..31 wrote block 1's first
  // outputs beside block 0's last: 2-way conflicts, round 6)
  constexpr bool HALVES = SG_R19_REMAP && CM > 0 && CNS > 0 && CNS <= 32 && CM / R == 2 * CNS;
  auto slot = [&](int q, int& j, int& jm) -> bool {
    if constexpr (HALVES) {
      jm = lane & 31;
      j = (lane >> 5) * CNS + jm;
      return q == 0 && jm < CNS;
    }
    j = lane + q * 64;
    if (j >= MR) return false;
    jm = CNS ? j % CNS : j - udiv(j, ns_magic) * Ns;
    return true;
  };
  v2 st[NB][R];
  int base_o[NB];
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    if (q * 64 >= MR) break;
    int j, jm;
    base_o[q] = 0;
    if (!slot(q, j, jm)) continue;
    base_o[q] = (j - jm) * R + jm;
    if constexpr (ODD) {
      // pairs (m, R - m) one at a time: inputs, twiddles and the symmetric
      // sums of one pair live at once (register budget of the fused kernel)
      st[q][0] = V(X[j]);
      const float2* tw = twS + (Ns - 1) + jm;
#pragma unroll
      for (int m = 1; m <= H; ++m) {
        v2 a = V(X[j + m * MR]), b = V(X[j + (R - m) * MR]);
        if (Ns > 1) {
          const v2 wa = V(tw[(m - 1) * Ns]), wb = V(tw[(R - m - 1) * Ns]);
          a = INV ? vmulc(a, wa) : vmul(a, wa);
          b = INV ? vmulc(b, wb) : vmul(b, wb);
        }
        st[q][m] = a + b;
        st[q][H + m] = a - b;
      }
      continue;
    }
    float2 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = X[j + r * MR];
    if (Ns > 1) {
      const float2* tw = twS + (Ns - 1) + jm;  // consecutive lanes, consecutive entries
#pragma unroll
      for (int r = 1; r < R; ++r) {
        const float2 w = tw[(r - 1) * Ns];
        v[r] = INV ? cmulc(v[r], w) : cmul(v[r], w);
      }
    }
    {
      Dft<R, INV>::run(v);
#pragma unroll
      for (int r = 0; r < R; ++r) st[q][r] = V(v[r]);
    }
  }
  sg_wave_fence();
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    if (q * 64 >= MR) break;
    int j, jm;
    if (!slot(q, j, jm)) continue;
    float2* y = X + base_o[q];
    if constexpr (ODD) {
      v2 y0 = st[q][0];
#pragma unroll
      for (int m = 1; m <= H; ++m) y0 += st[q][m];
      y[0] = F(y0);
#pragma unroll
      for (int k = 1; k <= H; ++k) {
        v2 a, b;
        odd_out<R, INV>(st[q], k, a, b);
        y[k * Ns] = F(a);
        y[(R - k) * Ns] = F(b);
      }
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) y[r * Ns] = F(st[q][r]);
    }
  }
  sg_wave_fence();
}

// Diagnostic build only (-DSG_STFT_STAMPS): cycles per section of the
// sg_stft_ola frame loop, accumulated per wave with s_memtime and summed into a
// buffer that nothing else reads (sg_debug_stft_stamps).
#ifdef SG_STFT_STAMPS
__device__ unsigned long long sg_stft_st[32];  // [0, 16): filter frames, [16, 32): noise frames
#define SG_ST(i)                                          \
  do {                                                    \
    if (st_acc) {                                         \
      const uint64_t _t = __builtin_amdgcn_s_memtime();   \
      st_acc[i] += _t - *st_last;                         \
      *st_last = _t;                                      \
    }                                                     \
  } while (0)
#define SG_ST_PARAMS , uint64_t *st_acc = nullptr, uint64_t *st_last = nullptr
#define SG_ST_ARGS , st_acc, st_last
#else
#define SG_ST(i) \
  do {           \
  } while (0)
#define SG_ST_PARAMS
#define SG_ST_ARGS
#endif

template <bool INV>
__device__ __forceinline__ void fft_w(float2* X, const SgFftGeom& g, const float2* twS, int lane SG_ST_PARAMS) {
  int Ns = 1;
  for (int s = 0; s < g.nstages; ++s) {
    const int R = g.radix[s];
    const uint32_t nm = g.ns_magic[s];
    int Ms = g.M;
    __asm__ __volatile__("" : "+s"(Ms));  // keep M / R and its multiples inside the stage (no hoisted SGPRs)
    switch (R) {
#define SG_STAGE(RR) \
      case RR: stage_w<RR, INV>(X, Ms, Ns, twS, nm, lane); break;
      SG_STAGE(2) SG_STAGE(3) SG_STAGE(4) SG_STAGE(5) SG_STAGE(7) SG_STAGE(11) SG_STAGE(13) SG_STAGE(17)
      SG_STAGE(19) SG_STAGE(23) SG_STAGE(29) SG_STAGE(31)
#undef SG_STAGE
      default: break;
    }
    Ns *= R;
    SG_ST((INV ? 5 : 1) + (s < 2 ? s : 2));
  }
}

// ------------------------------------------- radix-29 stage on the matrix pipe
// The first stage (Ns = 1: no twiddles) of the M = 1102 = 29 x 19 x 2 frame:
// 38 butterflies of 29 points, y_k = sum_m x_m W_29^{mk}, in the symmetric form
//   P_k = x_0 + sum_{m=1..14} (x_m + x_{29-m}) cos(2 pi mk / 29)     k = 0..14
//   Q_k =       sum_{m=1..14} (x_m - x_{29-m}) sin(2 pi mk / 29)     k = 1..14
//   forward y_k = P_k - i Q_k, y_{29-k} = P_k + i Q_k (inverse: the signs swap)
// as two real products [16 x 16] x [16 x 80] on v_mfma_f32_16x16x4_f32 (exact
// fp32: a k-ordered fmaf chain, like the VALU form). Rows: k; the cos matrix's
// column m = 0 is 1 (x_0 enters P), row 15 / column 15 are zero padding.
// Columns: the real (c = 0) and imaginary (c = 1) parts of the 38 butterflies.
// Q's operand carries the OTHER component of the same column, so one lane holds
// P_k.c and (Q_k).c' for its column and finishes y_k.c, y_{29-k}.c alone:
// y.re = P.re +- Q.im, y.im = P.im -+ Q.re. Reference: the DFT of seewave's
// stft/istft, seewave.r:7782-7819, :3447-3486 (R's fft).
//
// Layout (round 6; LDS bank rule: ds_read_b64 serves lanes 0-31 and 32-63 as
// two groups over 64 banks, ds_write_b64 four 16-lane quarters over 32 banks,
// ds_write_b32 two groups over 32 banks):
//  - Column groups 0 / 3 hold the real / imaginary parts of butterflies
//    j = col (0..15), groups 1 / 4 those of j = 16 + col: ONE lane holds both
//    components of its butterfly, so its operands are read once for two column
//    groups and y_k, y_{29-k} are written as whole pairs (ds_write_b64; a quarter's
//    16 pairs at a 58-word stride cover the 32 banks once). Group 2 holds both
//    parts of j = 32..37 (col < 6 real, 6 <= col < 12 imaginary, 12..15 padding
//    reading j = 32..35: same addresses, broadcast).
//  - K rows: k-step ks, lane quarter mg takes row m29_row(ks, mg) = 2 ks +
//    (mg >> 1) + 8 (mg & 1): the two quarters of a read group read rows 8 apart,
//    2 x 38 x 8 = 608 = 32 (mod 64) words, the other half of the banks.
//  - D rows: result row i = 4 (lane >> 4) + r is output k = m29_out(i), so the two
//    quarters of a group-2 ds_write_b32 write outputs 8 apart (16 words apart: the
//    other half of the 32 banks for those 6 butterflies' stride).
// Per lane: 24 pair reads, 40 MFMAs (1,280 matrix-pipe cycles per wave), 16 pair
// and 8 single-float writes, instead of ~520 VALU with 38 of 64 lanes busy
// (stage_w<29>). Round 5's layout (16 butterflies' real or imaginary parts per
// group, rows 4 ks + mg) read 40 pairs and wrote 40 floats per lane with 2-way
// conflicts on both: 1.0 conflict cycles per LDS instruction in sg_stft_ola (r05zz).
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ constexpr int m29_row(int ks, int mg) { return 2 * ks + (mg >> 1) + 8 * (mg & 1); }
__device__ __forceinline__ constexpr int m29_out(int i) { return (i & 3) + 8 * ((i >> 2) & 1) + 4 * (i >> 3); }
// The A fragments live in a 2 KB LDS table shared by the workgroup (lane l:
// cos fragments of k-steps 0..3 at tab[l], sin fragments at tab[64 + l]) and
// are read where the stage starts, so they hold no registers across the frame.
constexpr int SG_MAT29_BYTES = 128 * 16;
// Fills the table from the global twN[t] = W_2204^t = (cos, -sin)(2 pi t / 2204),
// t < 1102: W_29^t = W_2204^{76 t}, and W_2204^{t + 1102} = -W_2204^t. Threads
// 0..63 of the workgroup; the caller's barrier publishes it. LDS: after the
// workgroup's frame slices (planner: SG_MAT29_BYTES more for M = 1102).
// A operand of v_mfma_f32_16x16x4_f32: lane t holds A[i = t & 15][kk = t >> 4].
__device__ __forceinline__ void mat29_fill(float4* tab, const float2* twN, int t) {
  if (t >= 64) return;
  const int k = m29_out(t & 15);
  float p[4], q[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int m = m29_row(ks, t >> 4);
    const int idx = 76 * ((m * k) % 29);
    const float2 w = idx < 1102 ? twN[idx] : make_float2(-twN[idx - 1102].x, -twN[idx - 1102].y);
    p[ks] = (k <= 14 && m <= 14) ? w.x : 0.f;
    q[ks] = (k >= 1 && k <= 14 && m >= 1 && m <= 14) ? -w.y : 0.f;
  }
  tab[t] = make_float4(p[0], p[1], p[2], p[3]);
  tab[64 + t] = make_float4(q[0], q[1], q[2], q[3]);
}

template <bool INV>
__device__ __forceinline__ void stage29_mfma(float2* X, const float4* tab, int lane) {
  constexpr int MR = 38;
  const int col = lane & 15, mg = lane >> 4;
  const float4 ap = tab[lane], aq = tab[64 + lane];
  const float Ap[4] = {ap.x, ap.y, ap.z, ap.w}, Aq[4] = {aq.x, aq.y, aq.z, aq.w};
  // row 0: x_0 enters P alone (b weighted 0); rows without a second operand keep the
  // bank image of their group's partner row: row 0's b reads row 8's b address - 32
  // words, row 15 (padding, A's column zero) row 7's addresses + 32 words (finite data)
  const float w0 = mg == 0 ? 0.f : 1.f;
  auto load = [&](int j, float2 (&la)[4], float2 (&lb)[4]) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int m = m29_row(ks, mg);
      const int ia = m == 15 ? MR * 7 + 16 : MR * m;
      const int ib = m == 15 ? MR * 22 + 16 : m == 0 ? MR * 13 : MR * (29 - m);
      la[ks] = X[j + ia];
      lb[ks] = X[j + ib];
    }
  };
  // operand sums of k-step ks: s = a + b (row 0: a), d = a - b
  auto sums = [&](int ks, float2 a, float2 b, v2& s, v2& d) {
    s = ks == 0 ? pfma(V(b), splat(w0), V(a)) : V(a) + V(b);
    d = V(a) - V(b);
  };
  f32x4 P[5], Q[5];
  float2 la[2][4], lb[2][4];
  // butterflies j = 16 g + col, g = 0, 1: column groups g (real) and g + 3 (imaginary)
  load(col, la[0], lb[0]);
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    if (g == 0) load(16 + col, la[1], lb[1]);  // in flight while group 0's MFMAs issue
    else load(32 + (col < 12 ? col % 6 : col - 12), la[0], lb[0]);
    P[g] = Q[g] = P[g + 3] = Q[g + 3] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      v2 s, d;
      sums(ks, la[g][ks], lb[g][ks], s, d);
      P[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(Ap[ks], s.x, P[g], 0, 0, 0);
      Q[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(Aq[ks], d.y, Q[g], 0, 0, 0);
      P[g + 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(Ap[ks], s.y, P[g + 3], 0, 0, 0);
      Q[g + 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(Aq[ks], d.x, Q[g + 3], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  // group 2: butterflies 32..37, the lane's component c2
  const bool c2 = col >= 6;
  P[2] = Q[2] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    v2 s, d;
    sums(ks, la[0][ks], lb[0][ks], s, d);
    P[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(Ap[ks], c2 ? s.y : s.x, P[2], 0, 0, 0);
    Q[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(Aq[ks], c2 ? d.x : d.y, Q[2], 0, 0, 0);
  }
  sg_wave_fence();  // every read above precedes the in-place writes below
  // y_k = P_k -+ i Q_k: forward (re, im) = (P.re + Q.im, P.im - Q.re), the inverse swaps the signs
  const v2 sgn = INV ? v2{-1.f, 1.f} : v2{1.f, -1.f};
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    float2* y = X + 29 * (16 * g + col);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = m29_out(4 * mg + r);  // D layout: column = lane & 15, row = 4 (lane / 16) + r
      if (k > 14) continue;
      const v2 p = v2{P[g][r], P[g + 3][r]}, q = v2{Q[g][r], Q[g + 3][r]};  // p: (P.re, P.im), q: (Q.im, Q.re)
      y[k] = F(pfma(q, sgn, p));  // k = 0: Q_0 = 0
      if (k > 0) y[29 - k] = F(pfma(q, -sgn, p));
    }
  }
  if (col < 12) {
    float* y = reinterpret_cast<float*>(X + 29 * (32 + col % 6)) + (c2 ? 1 : 0);
    const float sg = c2 == INV ? 1.f : -1.f;  // re: P.re + sgn.x Q.im; im: P.im + sgn.y Q.re
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = m29_out(4 * mg + r);
      if (k > 14) continue;
      const float p = P[2][r], q = sg * Q[2][r];
      y[2 * k] = p + q;
      if (k > 0) y[2 * (29 - k)] = p - q;
    }
  }
  sg_wave_fence();
}

// The dominant geometry (C5: 94 % of frames are wl = 2204, M = 1102 = 29 x 19 x 2)
// with every size and stride a compile-time constant. MFMA: the radix-29 first
// stage on the matrix pipe (A29: its fragment table in LDS). Measured per C5
// launch (r05a, profiles/r05a_stft_ab.txt): the filter kernel 9.46 ms (stage
// order 2, 19, 29) -> 9.15 (29 first, VALU) -> 8.88 (29 first, MFMA); the noise
// kernel 2.53 -> 2.44 -> 2.56 (3 waves per SIMD: the MFMA stage's accumulators
// push it into spills), so the noise kernel keeps the VALU stage.
// LAST = false stops before the last stage (the forward M = 1102 filter transform fuses
// it with the untangle, r2_untangle_1102)
template <bool INV, int CM, int R0, int R1, int R2, bool MFMA = true, bool LAST = true>
__device__ __forceinline__ void fft_wc(float2* X, const float2* twS, const float4* A29, int lane SG_ST_PARAMS) {
  if constexpr (MFMA && CM == 1102 && R0 == 29) stage29_mfma<INV>(X, A29, lane);
  else stage_w<R0, INV, CM, 1>(X, CM, 1, twS, 0u, lane);
  SG_ST(INV ? 5 : 1);
  stage_w<R1, INV, CM, R0>(X, CM, R0, twS, 0u, lane);
  SG_ST(INV ? 6 : 2);
  if constexpr (LAST) stage_w<R2, INV, CM, R0 * R1>(X, CM, R0 * R1, twS, 0u, lane);
  SG_ST(INV ? 7 : 3);
}

// Complex n-point DFT of X (LDS, n points, in place) by the workgroup (sg_fft_frames):
// the Stockham FFT of size n, or Bluestein's chirp-z form through two L-point
// FFTs in Z (L points) -- SgCdft, planned by make_cdft (sg_plan_spec.cpp).
// INV: exp(+2 pi i jk / n), computed as conj(DFT(conj x)). tw: >= max(n, L) pairs.
template <bool INV>
__device__ void cdft(float2* X, const SgCdft& c, const SgFftGeom* __restrict__ geoms, const float* __restrict__ fl,
                     float2* Z, float2* tw) {
  const SgFftGeom& gs = geoms[c.geom];
  const int T = c.L ? c.L : c.n;
  const float2* twg = reinterpret_cast<const float2*>(fl + gs.tws);  // stage-ordered, T - 1 pairs
  for (int t = threadIdx.x; t < T - 1; t += SG_FFT_THREADS) tw[t] = twg[t];
  if (!c.L) {
    __syncthreads();
    fft_ip<INV>(X, gs, tw, 1);
    return;
  }
  const int n = c.n, L = c.L;
  const float2* ch = reinterpret_cast<const float2*>(fl + c.chirp);
  const float2* bf = reinterpret_cast<const float2*>(fl + c.bf);
  for (int j = threadIdx.x; j < L; j += SG_FFT_THREADS)
    Z[j] = j < n ? cmul(INV ? cconj(X[j]) : X[j], ch[j]) : make_float2(0.f, 0.f);
  __syncthreads();
  fft_ip<false>(Z, gs, tw, 1);
  for (int k = threadIdx.x; k < L; k += SG_FFT_THREADS) Z[k] = cmul(Z[k], bf[k]);
  __syncthreads();
  fft_ip<true>(Z, gs, tw, 1);
  for (int k = threadIdx.x; k < n; k += SG_FFT_THREADS) {
    const float2 v = cmul(Z[k], ch[k]);
    X[k] = INV ? cconj(v) : v;
  }
  __syncthreads();
}

// One frame of an odd window length N (SG_FFT_ODD): seewave's stft keeps
// M = N %/% 2 bins of the N-point DFT (/N); istft inverts the 2M = N - 1
// point Hermitian extension X = (Y_0..Y_{M-1}, Re Y_{M-1}, conj Y_{M-1}..conj Y_1)
// and recycles it against the N-point Hann window (seewave.r:3468-3479):
//   frame[i] = han[i] / 2M * Re(sum_t X_t e^{+2 pi i n t / 2M}),  n = i mod 2M.
// Both transforms are complex DFTs of the frame buffer B (N points) in place.
__device__ void odd_frame(const SgFrameGroup& G, const SgFrame* __restrict__ frames, const SgFftGeom& g,
                          const SgFftGeom* __restrict__ geoms, const float* __restrict__ fl, float* __restrict__ fs,
                          float4* lds4) {
  const int N = g.wl, M = g.M, N2 = 2 * M;
  const int T = max(g.cd[0].L ? g.cd[0].L : g.cd[0].n, g.cd[1].L ? g.cd[1].L : g.cd[1].n);
  float2* B = reinterpret_cast<float2*>(lds4);  // N points
  float2* Z = B + N;                            // Bluestein work buffer
  float2* tw = Z + T;                           // FFT twiddles
  const SgFrame F = frames[G.f0];
  const float* ham = fl + g.win;
  const float* han = ham + N;
  // Y_k (k < M) into B[k], then the Hermitian extension in place (B[M + 1 ..] hold
  // bins >= M of the forward transform, which nothing reads)
  if (G.mode == SG_FRAME_FILTER) {
    const float* s = fs + F.src;
    for (int n = threadIdx.x; n < N; n += SG_FFT_THREADS) B[n] = make_float2(s[n] * ham[n], 0.f);
    __syncthreads();
    cdft<false>(B, g.cd[0], geoms, fl, Z, tw);
    const float* env = fl + F.env;
    const float invN = 1.f / (float)N;
    for (int k = threadIdx.x; k < M; k += SG_FFT_THREADS) {
      const float sc = invN * env[k];
      const float2 y = make_float2(B[k].x * sc, B[k].y * sc);
      B[k] = y;
      if (k > 0) B[N2 - k] = cconj(y);
      if (k == M - 1) B[M] = make_float2(y.x, 0.f);
    }
  } else {  // SG_FRAME_NOISE: real spectrum u * filter
    const float* u = fl + F.src;
    const float* flt = fl + F.env;
    for (int k = threadIdx.x; k < M; k += SG_FFT_THREADS) {
      const float2 y = make_float2(u[k] * flt[k], 0.f);
      B[k] = y;
      if (k > 0) B[N2 - k] = y;
      if (k == M - 1) B[M] = y;
    }
  }
  __syncthreads();
  cdft<true>(B, g.cd[1], geoms, fl, Z, tw);
  const float invN2 = 1.f / (float)N2;
  float* d = fs + F.dst;
  for (int i = threadIdx.x; i < N; i += SG_FFT_THREADS) d[i] = B[i < N2 ? i : i - N2].x * invN2 * han[i];
}

}  // namespace

extern "C" __global__ __launch_bounds__(SG_FFT_THREADS) void sg_fft_frames(
    const SgFrameGroup* __restrict__ groups, const SgFrame* __restrict__ frames, const SgFftGeom* __restrict__ geoms,
    const float* __restrict__ fl, float* __restrict__ fs) {
  extern __shared__ float4 lds4[];
  float2* A = reinterpret_cast<float2*>(lds4);
  __shared__ SgFrame fr[16];
  const SgFrameGroup G = groups[blockIdx.x];
  const SgFftGeom& g = geoms[G.geom];
  if (g.kind == SG_FFT_ODD) {  // workgroup-uniform
    odd_frame(G, frames, g, geoms, fl, fs, lds4);
    return;
  }
  const int M = g.M, N = g.wl, fb = G.nf;
  const float2* twg = reinterpret_cast<const float2*>(fl + g.tw);
  const float2* twN = twg + M;  // L1/L2 resident (one read per bin pair)
  float2* twM = A + fb * M;     // stage-ordered twiddles in LDS behind the frames (SG_FFT_DFT: the Bluestein buffers)
  if (g.kind != SG_FFT_DFT) {
    const float2* tsg = reinterpret_cast<const float2*>(fl + g.tws);
    for (int t = threadIdx.x; t < M - 1; t += SG_FFT_THREADS) twM[t] = tsg[t];
  }
  if (threadIdx.x < fb) fr[threadIdx.x] = frames[G.f0 + threadIdx.x];
  __syncthreads();
  const float* ham = fl + g.win;
  const float* han = ham + N;
  const float invN = 1.f / (float)N;
  const int half = M / 2;
  const int npairs = fb * (half + 1);
  constexpr int NP = SG_FFT_SLOTS / 2 / SG_FFT_THREADS + 1;  // pairs per thread
  if (G.mode == SG_FRAME_FILTER) {
    for (int idx = threadIdx.x; idx < fb * M; idx += SG_FFT_THREADS) {
      const int f = udiv(idx, g.m_magic), n = idx - f * M;
      const float* s = fs + fr[f].src;
      A[idx] = make_float2(s[2 * n] * ham[2 * n], s[2 * n + 1] * ham[2 * n + 1]);
    }
    __syncthreads();
    if (g.kind == SG_FFT_DFT) cdft<false>(A, g.cd[0], geoms, fl, twM, twM + g.cd[0].L);
    else fft_ip<false>(A, g, twM, fb);
    // untangle the real transform: X[k] = E + W_N^k O, E = (Z_k + conj Z_{M-k})/2,
    // O = -i (Z_k - conj Z_{M-k}) / 2; Y = X / N * env; pack for the inverse
    float2 zk[NP], zm[NP], zh[NP];
    int pk[NP], pf[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const int idx = threadIdx.x + q * SG_FFT_THREADS;
      pk[q] = -1;
      if (idx >= npairs) continue;
      const int f = udiv(idx, g.hp_magic), k = idx - f * (half + 1);
      if (k != 0 && k >= M - k) continue;
      pk[q] = k;
      pf[q] = f;
      const float2* z = A + f * M;
      const float* env = fl + fr[f].env;
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
      const int f = udiv(idx, g.hp_magic), k = idx - f * (half + 1);
      const SgFrame& F = fr[f];
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
  if (g.kind == SG_FFT_DFT) cdft<true>(A, g.cd[0], geoms, fl, twM, twM + g.cd[0].L);
  else fft_ip<true>(A, g, twM, fb);
  // windowed frame: Re(ifft)/N x hann, y[2n] = Re z[n], y[2n+1] = Im z[n]
  for (int idx = threadIdx.x; idx < fb * M; idx += SG_FFT_THREADS) {
    const int f = udiv(idx, g.m_magic), n = idx - f * M;
    const float2 v = A[idx];
    float* d = fs + fr[f].dst;
    d[2 * n] = v.x * invN * han[2 * n];
    d[2 * n + 1] = v.y * invN * han[2 * n + 1];
  }
}

// ------------------------------------------------ fused frame pipeline
// Inputs of one frame, loaded into registers at the top of the frame (their HBM
// latency overlaps the other wave's work on the SIMD; loading a frame ahead
// measured neutral or slower, r03i/r03l):
//   FILTER: s[i] = sound (y[2n], y[2n+1]), n = 64 i + lane; a[i] = envelope
//           (env[k], env[M - k]) with k = 64 i + lane (k = 0: env[0], env[M-1]); xh = env[half]
//   NOISE:  a[i] = uniforms (u[k], u[M - k]), b[i] = filter (f[k], f[M - k]) (k = 0: M - 1); xh, xh2 at half
// NOISE's filter pairs share the FILTER sound registers (b[i] = s[i]): the mode is
// wave-uniform but not a compile-time constant, so separate arrays would both be allocated
static_assert(SG_PF_PAIR <= SG_PF_SRC, "noise filter pairs alias the sound pairs");
struct FramePf {
  float2 s[SG_PF_SRC];
  float2 a[SG_PF_PAIR];
  float xh, xh2;
  __device__ __forceinline__ float2& b(int i) { return s[i]; }
  __device__ __forceinline__ const float2& b(int i) const { return s[i]; }
};

// FUSED (M = 1102 filter frames, r2_untangle_1102): envelope pairs by unit, lane's
// unit u = 1 + lane + 64 q (q < 5, u <= 275): a[2q] = (env[u], env[M - u]),
// a[2q + 1] = (env[551 - u], env[551 + u]); xh = env[551], xh2 = env[0]
template <bool FUSED = false>
__device__ __forceinline__ void frame_prefetch(FramePf& P, const SgFrame& F, int mode, int M,
                                               const float* __restrict__ fl, const float* __restrict__ fs, int lane) {
  const int half = M / 2;
  if (mode == SG_FRAME_FILTER) {
    const float* src = fs + F.src;
    const float* env = fl + F.env;
#pragma unroll
    for (int i = 0; i < SG_PF_SRC; ++i) {
      const int n = 64 * i + lane;
      if (n < M) P.s[i] = make_float2(src[2 * n], src[2 * n + 1]);
    }
    if constexpr (FUSED) {
      static_assert(2 * 5 <= SG_PF_PAIR, "fused untangle: 5 units of two envelope pairs per lane");
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        const int u = 1 + lane + 64 * q;
        if (u <= 275) {
          P.a[2 * q] = make_float2(env[u], env[1102 - u]);
          P.a[2 * q + 1] = make_float2(env[551 - u], env[551 + u]);
        }
      }
      P.xh = env[551];
      P.xh2 = env[0];
      return;
    }
#pragma unroll
    for (int i = 0; i < SG_PF_PAIR; ++i) {
      const int k = 64 * i + lane;
      if (k <= half) P.a[i] = make_float2(env[k], env[k == 0 ? M - 1 : M - k]);
    }
    P.xh = env[half];
  } else {
    const float* u = fl + F.src;
    const float* flt = fl + F.env;
#pragma unroll
    for (int i = 0; i < SG_PF_PAIR; ++i) {
      const int k = 64 * i + lane;
      if (k <= half) {
        const int km = k == 0 ? M - 1 : M - k;
        P.a[i] = make_float2(u[k], u[km]);
        P.b(i) = make_float2(flt[k], flt[km]);
      }
    }
    P.xh = u[half];
    P.xh2 = flt[half];
  }
}

// The forward M = 1102 filter transform's last stage (radix 2, Ns = 551: butterfly j
// maps Z[j], Z[j + 551] from X[j], X[j + 551] W^j) fused with the real-FFT untangle
// (frame_front's pair k reads Z[k] and Z[M - k]). Butterflies u and 551 - u hold both
// pairs (u, M - u) and (551 - u, 551 + u), so unit u (1 <= u <= 275; lane 1 + 64 q)
// reads four slots, transforms and untangles in registers and writes the same four
// slots: one LDS write and one read per point fewer than the separate passes. Units
// touch disjoint slots; lane 0 also takes butterfly 0 and the pair k = 0 (slots 0
// and 551) with its unit's Z[1] and Z[M - 1]. Same operations as stage_w<2> and the
// untangle, in the same order.
__device__ __forceinline__ void r2_untangle_1102(float2* A, const FramePf& P, const float2* twS, const float2* twN,
                                                 int lane) {
  constexpr int M = 1102, H = 551;
  const float invN = 1.f / (float)(2 * M);
  // one untangled pair (k, M - k) from Z_k = za, Z_{M-k} = zb (frame_front's packed form)
  auto pair = [&](int kk, float2 za, float2 zb, float ek, float em) {
    const v2 a = V(za), b = V(zb);
    const v2 s = add_conjb(a, b), d = sub_conjb(a, b);
    const v2 wk = V(twN[kk]);
    const v2 p = vmul(d, wk);
    const v2 yk = add_miq(s, p) * splat(0.5f * ek);
    const v2 um = add_piq(s, p) * splat(0.5f * em);
    const v2 q = vmulc(yk - um, wk);
    const v2 e = yk + um;
    const v2 zk = add_piq(e, q), zm = add_miq(e, q);
    A[kk] = F(zk);
    A[M - kk] = make_float2(zm.x, -zm.y);
  };
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const int u = 1 + lane + 64 * q;
    if (u > 275) continue;
    const int v = H - u;
    const float2 au = A[u], cu = A[u + H], av = A[v], cv = A[v + H];
    const float2 tu = cmul(cu, twS[H - 1 + u]), tv = cmul(cv, twS[H - 1 + v]);
    const float2 zu = cadd(au, tu), zuh = csub(au, tu);  // Z[u], Z[u + 551]
    const float2 zv = cadd(av, tv), zvh = csub(av, tv);  // Z[v], Z[v + 551] = Z[M - u]
    if (q == 0 && lane == 0) {  // butterfly 0 and the pair k = 0: Z[1] = zu, Z[M - 1] = zvh (u = 1)
      const float2 a0 = A[0], c0 = A[H];
      const float2 t0 = cmul(c0, twS[H - 1]);
      const float2 z0 = cadd(a0, t0), zh = csub(a0, t0);
      auto X_at = [&](float2 a, float2 b, int t) -> float2 {
        const float2 e = make_float2(0.5f * (a.x + b.x), 0.5f * (a.y - b.y));
        const float2 dd = make_float2(a.x - b.x, a.y + b.y);
        const float2 o = make_float2(0.5f * dd.y, -0.5f * dd.x);
        return cadd(e, cmul(o, twN[t]));
      };
      const float ek = P.xh2 * invN, em = P.a[0].y * invN;  // env[0], env[M - 1]
      const float2 x0 = X_at(z0, z0, 0), xl = X_at(zvh, zu, M - 1);
      const float y0 = x0.x * ek;
      const float nyq = xl.x * em;
      A[0] = make_float2(y0 + nyq, y0 - nyq);
      const float2 xk = X_at(zh, zh, H);
      const float eh = P.xh * invN;
      const float2 yk = make_float2(xk.x * eh, xk.y * eh);
      float2 a, b;
      pack_pair(yk, yk, twN[H], a, b);
      A[H] = a;
    }
    pair(u, zu, zvh, P.a[2 * q].x * invN, P.a[2 * q].y * invN);
    pair(v, zv, zuh, P.a[2 * q + 1].x * invN, P.a[2 * q + 1].y * invN);
  }
  sg_wave_fence();
}

// Consume P: the frame's packed inverse-FFT input lands in A (FILTER: sound x
// hamming -> forward FFT -> untangle, /wl x envelope, seewave's Hermitian
// mirror; NOISE: uniforms x filter). Tables in LDS: ham (wl floats), twN (M pairs).
template <int CM, int R0, int R1, int R2>
__device__ __forceinline__ void frame_front(float2* A, const FramePf& P, int mode, const SgFftGeom& g,
                                            const float2* twS, const float2* twN, const float* ham,
                                            const float4* A29, int lane SG_ST_PARAMS) {
  int M = CM ? CM : g.M, N = CM ? 2 * CM : g.wl;
  if (!CM) __asm__ __volatile__("" : "+s"(M), "+s"(N));  // opaque: no hoisting across the caller's frame loop
  const float invN = 1.f / (float)N;
  const int half = M / 2;
  if (mode == SG_FRAME_FILTER) {
#pragma unroll
    for (int i = 0; i < SG_PF_SRC; ++i) {
      const int n = 64 * i + lane;
      if (n < M) A[n] = F(V(P.s[i]) * V(reinterpret_cast<const float2*>(ham)[n]));
    }
    sg_wave_fence();
    SG_ST(0);
    if constexpr (CM == 1102 && R0 == 29 && R1 == 19 && R2 == 2) {  // the last stage fused with the untangle
      fft_wc<false, CM, R0, R1, R2, true, false>(A, twS, A29, lane SG_ST_ARGS);
      r2_untangle_1102(A, P, twS, twN, lane);
      return;
    }
    if constexpr (CM != 0) fft_wc<false, CM, R0, R1, R2>(A, twS, A29, lane SG_ST_ARGS);  // filter frames only
    else fft_w<false>(A, g, twS, lane SG_ST_ARGS);
    // untangle X[k] = E + W_N^k O (E, O from Z_k, conj Z_{M-k}), Y = X / wl x env,
    // pack for the inverse; pair k owns slots k and M - k, the k = 0 lane also
    // reads slots 1, M - 1 and half; every read of an iteration precedes its writes
#pragma unroll
    for (int i = 0; i < SG_PF_PAIR; ++i) {
      const int k0 = 64 * i;
      if (k0 > half) break;
      const int k = k0 + lane;
      const bool act = k <= half && (k == 0 || k < M - k);
      const int kk = act ? k : 0;
      const int km = kk == 0 ? 0 : M - kk;
      const float2 za = A[kk], zb = A[km];
      float2 z1 = za, zM1 = za, zh = za;
      if (i == 0) {
        z1 = A[1];
        zM1 = A[M - 1];
        zh = A[half];
      }
      // lane 0's reads of slots 1 and M - 1 must precede lane 1's writes: per
      // thread the compiler may sink them into the k = 0 branch, which the
      // SIMT code runs after the other branch
      sg_wave_fence();
      if (!act) continue;
      auto X_at = [&](float2 a, float2 b, int t) -> float2 {
        const float2 e = make_float2(0.5f * (a.x + b.x), 0.5f * (a.y - b.y));
        const float2 dd = make_float2(a.x - b.x, a.y + b.y);
        const float2 o = make_float2(0.5f * dd.y, -0.5f * dd.x);
        return cadd(e, cmul(o, twN[t]));
      };
      const float ek = P.a[i].x * invN, em = P.a[i].y * invN;  // k = 0: env[0], env[M - 1]
      if (kk == 0) {
        const float2 x0 = X_at(za, za, 0), xl = X_at(zM1, z1, M - 1);
        const float y0 = x0.x * ek;
        const float nyq = xl.x * em;
        A[0] = make_float2(y0 + nyq, y0 - nyq);
        if (M % 2 == 0) {
          const float2 xk = X_at(zh, zh, half);
          const float eh = P.xh * invN;
          const float2 yk = make_float2(xk.x * eh, xk.y * eh);
          float2 a, b;
          pack_pair(yk, yk, twN[half], a, b);
          A[half] = a;
        }
      } else {
        // packed form (v_pk_* on (re, im)): with s = Z_k + conj Z_{M-k}, d = Z_k - conj Z_{M-k},
        // p = d W_N^k: 2 X_k = s - i p and 2 X_{M-k} = conj(s + i p) (W_N^{M-k} = -conj W_N^k:
        // no second twiddle read); the inverse packing Z'_k = e + i q, Z'_{M-k} = conj(e - i q)
        // with e = Y_k + conj Y_{M-k}, q = (Y_k - conj Y_{M-k}) conj W_N^k (pack_pair)
        const v2 a = V(za), b = V(zb);
        const v2 s = add_conjb(a, b), d = sub_conjb(a, b);
        const v2 wk = V(twN[kk]);
        const v2 p = vmul(d, wk);
        const v2 yk = add_miq(s, p) * splat(0.5f * ek);
        const v2 um = add_piq(s, p) * splat(0.5f * em);  // conj Y_{M-k}
        const v2 q = vmulc(yk - um, wk);
        const v2 e = yk + um;
        const v2 zk = add_piq(e, q), zm = add_miq(e, q);
        A[kk] = F(zk);
        A[km] = make_float2(zm.x, -zm.y);
      }
    }
  } else {  // SG_FRAME_NOISE: real spectrum u x filter, packed
#pragma unroll
    for (int i = 0; i < SG_PF_PAIR; ++i) {
      const int k = 64 * i + lane;
      if (k > half) continue;
      if (k == 0) {
        const float y0 = P.a[i].x * P.b(i).x, nyq = P.a[i].y * P.b(i).y;
        A[0] = make_float2(y0 + nyq, y0 - nyq);
        if (M % 2 == 0) {
          const float2 yk = make_float2(P.xh * P.xh2, 0.f);
          float2 a, b;
          pack_pair(yk, yk, twN[half], a, b);
          A[half] = a;
        }
      } else if (k < M - k) {
        // pack_pair of the real Y_k = a, Y_{M-k} = b: with e = a + b, r = a - b,
        // Z'_k = (e + r Im W, r Re W), Z'_{M-k} = (e - r Im W, r Re W)
        const float a = P.a[i].x * P.b(i).x, b = P.a[i].y * P.b(i).y;
        const float2 w = twN[k];
        const float e = a + b, r = a - b, im = r * w.x;
        A[k] = make_float2(fmaf(r, w.y, e), im);
        A[M - k] = make_float2(fmaf(-r, w.y, e), im);
      }
    }
  }
  sg_wave_fence();
}

#ifndef SG_CARRY64
#define SG_CARRY64 0
#endif
#ifndef SG_NOISE_MFMA
#define SG_NOISE_MFMA 0
#endif
// Fused STFT x envelope -> ISTFT -> overlap-add (seewave istft,
// seewave.r:3462-3484) -> matchLengths trim. Each wavefront owns one segment
// (a run of consecutive frames of one OLA) and walks it frame by frame with
// no workgroup barrier: the frame is transformed in its LDS slice, windowed
// (/wl x hanning) and added to the carried partial sums of earlier frames,
// which live in registers (pair layout: lane l, register r <-> samples
// 2(64r + l), +1 of the frame). The samples before the next frame's start are
// final (scaled, trimmed, written, max-reduced); the rest, shifted by the
// hop, is the next carry. Frames never leave LDS; summation is in frame
// order, so results are deterministic.
// LDS: twS (M pairs), twN (M pairs), ham + han (M pairs each), SG_FFT_WAVES slices (M pairs each).
// One segment of sg_stft_ola (CM > 0: the M = CM geometry with radices R0 x R1 x R2, sizes folded)
template <int CM, int R0, int R1, int R2, int MODE, int CP = SG_CARRY_PAIRS>
__device__ __forceinline__ void stft_segment(const SgSegment& S, const SgOla* __restrict__ olas,
                                             const SgFrame* __restrict__ frames, const SgFftGeom& g,
                                             const float* __restrict__ fl, float* __restrict__ fs,
                                             float* __restrict__ slotmax, float2* twS, const float2* twN,
                                             const float* ham, const float* han, int w, int lane) {
  const int M = CM ? CM : g.M, N = CM ? 2 * CM : g.wl;
  const int mode = MODE;  // the launch's phase fixes it (noise: phase 0, filter: phase 1)
  const SgOla& O = olas[S.ola];
  float2* A = twS + M * (4 + w);
  const float* Af = reinterpret_cast<const float*>(A);
  const int hi = O.hi;
  const double h = O.h;
  auto bstart = [&](int f) -> int { return hi > 0 ? f * hi : (int)floor((double)f * h); };
  const int first = (int)O.first, len = (int)O.len;
  const float scale = O.scale;
  float* out = fs + O.out;
  float m = -INFINITY;
  // M = 1102 filter frames: the inverse transform's last stage (radix 2, Ns = 551)
  // fused with the window and the carry, which then lives in the butterflies' layout
  // (lane l, q: elements j = l + 64 q and j + 551)
  constexpr bool FUSED = CM == 1102 && R0 == 29 && R1 == 19 && R2 == 2;
  constexpr int CR = FUSED ? 9 : CP;  // carry registers per half
  float2 C[CR], C2[FUSED ? 9 : 1];
#pragma unroll
  for (int r = 0; r < CR; ++r) C[r] = make_float2(0.f, 0.f);
#pragma unroll
  for (int r = 0; r < (FUSED ? 9 : 1); ++r) C2[r] = make_float2(0.f, 0.f);
  FramePf P;
  constexpr int W = MODE == SG_FRAME_NOISE ? SG_FFT_WAVES_NOISE : SG_FFT_WAVES;
  const float4* A29 = reinterpret_cast<const float4*>(twS + M * (4 + W));  // radix-29 fragments (M = 1102)
#ifdef SG_STFT_STAMPS
  uint64_t st_accv[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t st_lastv = __builtin_amdgcn_s_memtime();
  uint64_t* st_acc = st_accv;
  uint64_t* st_last = &st_lastv;
#endif
  int bf = bstart(S.f0);
  for (int k = 0; k < S.nf; ++k) {
    {
      int Mk = M;
      if (!CM) __asm__ __volatile__("" : "+s"(Mk));
      frame_prefetch<FUSED && MODE == SG_FRAME_FILTER>(P, frames[S.fdev + k], mode, Mk, fl, fs, lane);
    }
    frame_front<CM, R0, R1, R2>(A, P, mode, g, twS, twN, ham, A29, lane SG_ST_ARGS);
    SG_ST(4);
    const float2* han2 = reinterpret_cast<const float2*>(han);
    const bool lastf = k == S.nf - 1;
    const int bn = lastf ? S.pb : bstart(S.f0 + k + 1);
    const int D = bn - bf;  // samples [bf, bn) are final
    // FUSED noise frames: an interior frame whose final samples all lie in the first
    // 1102 (elements j < 551) writes them from registers; only the elements the next
    // carry reads (those holding a sample >= D) go to LDS (wave-uniform). Measured:
    // noise 2.35 -> 2.30 ms per launch, filter 8.14 -> 8.47 ms (its stores then issue
    // inside the LDS-bound loop at 2 waves per SIMD), so the filter keeps the LDS pass.
    const bool direct = FUSED && MODE == SG_FRAME_NOISE && bf >= S.pa && bf - first >= 0 && bn - first <= len && D <= 1102;
    if constexpr (FUSED) {
      fft_wc<true, CM, R0, R1, R2, MODE == SG_FRAME_FILTER || SG_NOISE_MFMA, false>(A, twS, A29, lane SG_ST_ARGS);
      // butterfly j: Z[j], Z[j + 551] from X[j], X[j + 551] conj(W^j) (stage_w<2>'s
      // operations), each windowed (han holds hanning / wl) and added to its carry
      float* __restrict__ o = out + (bf - first);
      const bool o2 = ((O.out + bf - first) & 1) == 0;  // float2 stores (8-B aligned pairs)
#pragma unroll
      for (int q = 0; q < 9; ++q) {
        const int j = 64 * q + lane;
        if (j >= 551) continue;
        const float2 a = A[j], c = A[j + 551];
        const float2 t = cmulc(c, twS[550 + j]);
        const float2 y0 = F(pfma(V(cadd(a, t)), V(han2[j]), V(C[q])));
        A[j + 551] = F(pfma(V(csub(a, t)), V(han2[j + 551]), V(C2[q])));
        if (direct && 2 * j < D) {
          const float v0 = y0.x * scale, v1 = y0.y * scale;
          if (2 * j + 1 < D) {
            if (o2) *reinterpret_cast<float2*>(o + 2 * j) = make_float2(v0, v1);
            else {
              o[2 * j] = v0;
              o[2 * j + 1] = v1;
            }
            m = fmaxf(m, fmaxf(v0, v1));
          } else {
            o[2 * j] = v0;
            m = fmaxf(m, v0);
            A[j] = y0;  // sample D: the next carry
          }
        } else {
          A[j] = y0;
        }
      }
    } else {
      if constexpr (CM != 0) fft_wc<true, CM, R0, R1, R2, MODE == SG_FRAME_FILTER>(A, twS, A29, lane SG_ST_ARGS);
      else fft_w<true>(A, g, twS, lane SG_ST_ARGS);
      int Mk = M;
      if (!CM) __asm__ __volatile__("" : "+s"(Mk));
      // window (han holds hanning / wl: one packed FMA per pair) and add the carry
      // (pairs n = 64 r + lane)
#pragma unroll
      for (int r = 0; r < CP; ++r) {
        const int n = 64 * r + lane;
        if (n < Mk) A[n] = F(pfma(V(A[n]), V(han2[n]), V(C[r])));
      }
      for (int n = 64 * CP + lane; n < Mk; n += 64) A[n] = F(V(A[n]) * V(han2[n]));
    }
    int Nk = N;
    if (!CM) __asm__ __volatile__("" : "+s"(Nk));
    sg_wave_fence();
    SG_ST(8);
    if (direct) {
      // written above
    } else if (bf >= S.pa && bf - first >= 0 && bn - first <= len && D <= Nk) {
      // interior frame (wave-uniform): every final sample is owned, inside the trim and the frame
      float* __restrict__ o = out + (bf - first);
      int i = lane;
      for (; i + 192 < D; i += 256) {  // four LDS reads in flight per lane before the stores
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = Af[i + 64 * e] * scale;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o[i + 64 * e] = v[e];
          m = fmaxf(m, v[e]);
        }
      }
      for (; i < D; i += 64) {
        const float v = Af[i] * scale;
        o[i] = v;
        m = fmaxf(m, v);
      }
    } else {
      for (int i = lane; i < D; i += 64) {
        const int p = bf + i;
        const int q = p - first;
        if (p >= S.pa && q >= 0 && q < len) {
          const float v = (i < Nk ? Af[i] : 0.f) * scale;
          out[q] = v;
          m = fmaxf(m, v);
        }
      }
    }
    if (!lastf) {
      // the next carry: pair n holds samples 2n + D, 2n + D + 1 of this frame (zero
      // past its end); every read unconditional (index clamped into the slice), all
      // in flight at once. SG_CARRY64: pair reads (ds_read_b64, consecutive lanes on
      // consecutive pairs: no bank conflicts) -- D even: pair n + D/2; D odd (the
      // usual hop, wl/4 = 551): the odd half of pair p = n + (D-1)/2 and the even
      // half of p + 1. (Two float reads 2 words apart per lane were 2-way conflicts.)
#if SG_CARRY64 == 2
      // odd D: one pair read per lane; the even half of pair p + 1 is the next lane's
      // (DPP wave_shl:1), lane 63 takes lane 0 of the next block
      const float2* __restrict__ A2 = A;
      const int ph = D >> 1;
      auto carry_even = [&](int n) {
        const int p = n + ph;
        const float2 a = A2[min(p, M - 1)];
        return p < M ? a : make_float2(0.f, 0.f);
      };
      auto shl1 = [](float v) {
        return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xf, 0xf, false));
      };
      constexpr int NQ = FUSED ? 9 : CP;
      auto carry_odd_set = [&](int n0, float2 (&Cs)[NQ]) {
        float2 a[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) a[q] = A2[min(n0 + 64 * q + lane + ph, M - 1)];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const int p = n0 + 64 * q + lane + ph;
          float nx = shl1(a[q].x);
          if (q + 1 < NQ) nx = lane == 63 ? __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, a[q + 1].x), 0)) : nx;
          Cs[q] = make_float2(p < M ? a[q].y : 0.f, p + 1 < M ? nx : 0.f);
        }
      };
      if (D & 1) {
        if constexpr (FUSED) {
          carry_odd_set(0, C);
          carry_odd_set(551, C2);
        } else {
          carry_odd_set(0, C);
        }
      } else {
        if constexpr (FUSED) {
#pragma unroll
          for (int q = 0; q < 9; ++q) {
            const int j = 64 * q + lane;
            C[q] = carry_even(j);
            C2[q] = carry_even(j + 551);
          }
        } else {
#pragma unroll
          for (int r = 0; r < CP; ++r) C[r] = carry_even(64 * r + lane);
        }
      }
#elif SG_CARRY64
      const float2* __restrict__ A2 = A;
      const int ph = D >> 1;
      auto carry_even = [&](int n) {
        const int p = n + ph;
        const float2 a = A2[min(p, M - 1)];
        return p < M ? a : make_float2(0.f, 0.f);
      };
      auto carry_odd = [&](int n) {
        const int p = n + ph;
        const float2 a = A2[min(p, M - 1)], b = A2[min(p + 1, M - 1)];
        return make_float2(p < M ? a.y : 0.f, p + 1 < M ? b.x : 0.f);
      };
#define SG_CARRY_LOOP(carry)                      \
  if constexpr (FUSED) {                          \
    _Pragma("unroll") for (int q = 0; q < 9; ++q) { \
      const int j = 64 * q + lane;                \
      C[q] = carry(j);                            \
      C2[q] = carry(j + 551);                     \
    }                                             \
  } else {                                        \
    _Pragma("unroll") for (int r = 0; r < CP; ++r) C[r] = carry(64 * r + lane); \
  }
      if (D & 1) {
        SG_CARRY_LOOP(carry_odd)
      } else {
        SG_CARRY_LOOP(carry_even)
      }
#undef SG_CARRY_LOOP
#else
      auto carry = [&](int n) {
        const int i0 = 2 * n + D;
        const float a = Af[min(i0, Nk - 1)], b = Af[min(i0 + 1, Nk - 1)];
        return make_float2(i0 < Nk ? a : 0.f, i0 + 1 < Nk ? b : 0.f);
      };
      if constexpr (FUSED) {
#pragma unroll
        for (int q = 0; q < 9; ++q) {
          const int j = 64 * q + lane;
          C[q] = carry(j);
          C2[q] = carry(j + 551);
        }
      } else {
#pragma unroll
        for (int r = 0; r < CP; ++r) C[r] = carry(64 * r + lane);
      }
#endif
    }
    sg_wave_fence();  // the next frame overwrites the slice
    bf = bn;
    SG_ST(9);
  }
#ifdef SG_STFT_STAMPS
  if (lane == 0) {
    unsigned long long* st = sg_stft_st + (MODE == SG_FRAME_NOISE ? 16 : 0);
    for (int i = 0; i < 10; ++i) atomicAdd(&st[i], (unsigned long long)st_acc[i]);
    atomicAdd(&st[10], (unsigned long long)S.nf);
    atomicAdd(&st[11], 1ull);
  }
#endif
  // matchLengths padding (zeros) outside the istft output
  if (S.flags & SG_SEG_FIRST)
    for (int q = lane; q < min(len, -first); q += 64) {
      out[q] = 0.f;
      m = fmaxf(m, 0.f);
    }
  if (S.flags & SG_SEG_LAST)
    for (int p = max((int)O.xlen, first) + lane; p < first + len; p += 64) {
      out[p - first] = 0.f;
      m = fmaxf(m, 0.f);
    }
  m = sgd::wave_max(m);
  if (lane == 0) slotmax[S.slot] = m;
}

// the specialised geometry: M = 1102 in the planner's stage order 29, 19, 2
__device__ __forceinline__ bool geom_1102(const SgFftGeom& g) {
  return g.M == 1102 && g.nstages == 3 && g.radix[0] == 29 && g.radix[1] == 19 && g.radix[2] == 2;
}

template <int MODE>
__device__ __forceinline__ void stft_ola_body(
    const SgSegment* __restrict__ segs, const SgOla* __restrict__ olas, const SgFrame* __restrict__ frames,
    const SgFftGeom* __restrict__ geoms, const float* __restrict__ fl, float* __restrict__ fs,
    float* __restrict__ slotmax) {
  constexpr int W = MODE == SG_FRAME_NOISE ? SG_FFT_WAVES_NOISE : SG_FFT_WAVES, NT = W * 64;
  extern __shared__ float4 lds4[];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;  // w wave-uniform
  const SgFftGeom& g = geoms[segs[blockIdx.x * W].geom];  // the planner groups segments by geometry
  const int M = g.M, N = g.wl;
  float2* twS = reinterpret_cast<float2*>(lds4);
  float2* twN = twS + M;
  float* ham = reinterpret_cast<float*>(twN + M);
  float* han = ham + N;
  {
    const float2* tsg = reinterpret_cast<const float2*>(fl + g.tws);
    const float2* tng = reinterpret_cast<const float2*>(fl + g.tw) + M;
    const float* wg = fl + g.win;
    for (int t = threadIdx.x; t < M; t += NT) {
      if (t < M - 1) twS[t] = tsg[t];
      twN[t] = tng[t];
    }
    // hamming, then hanning times 1 / wl (the inverse transform's scale)
    const float hs = 1.f / (float)N;
    for (int t = threadIdx.x; t < 2 * N; t += NT) ham[t] = t < N ? wg[t] : wg[t] * hs;
    if ((MODE == SG_FRAME_FILTER || SG_NOISE_MFMA) && geom_1102(g)) mat29_fill(reinterpret_cast<float4*>(twS + M * (4 + W)), tng, threadIdx.x);
  }
  __syncthreads();
  const SgSegment S = segs[blockIdx.x * W + w];
  if (S.nf <= 0) return;  // padding segment
  if (geom_1102(g))
    stft_segment<1102, 29, 19, 2, MODE>(S, olas, frames, g, fl, fs, slotmax, twS, twN, ham, han, w, lane);
  else
    stft_segment<0, 0, 0, 0, MODE>(S, olas, frames, g, fl, fs, slotmax, twS, twN, ham, han, w, lane);
}

constexpr int SG_FFT_WPE = 2;  // waves per SIMD of sg_stft_ola (241 VGPRs)
constexpr int SG_FFT_WPE_NOISE = SG_FFT_WAVES_NOISE > 8 ? 3 : 2;
extern "C" __global__ __launch_bounds__(SG_FFT_WAVES * 64) __attribute__((amdgpu_waves_per_eu(SG_FFT_WPE))) void sg_stft_ola(
    const SgSegment* __restrict__ segs, const SgOla* __restrict__ olas, const SgFrame* __restrict__ frames,
    const SgFftGeom* __restrict__ geoms, const float* __restrict__ fl, float* __restrict__ fs,
    float* __restrict__ slotmax) {
  stft_ola_body<SG_FRAME_FILTER>(segs, olas, frames, geoms, fl, fs, slotmax);
}
// generateNoise()'s istft (phase 0): the noise mode only
extern "C" __global__ __launch_bounds__(SG_FFT_WAVES_NOISE * 64) __attribute__((amdgpu_waves_per_eu(SG_FFT_WPE_NOISE))) void sg_stft_ola_noise(
    const SgSegment* __restrict__ segs, const SgOla* __restrict__ olas, const SgFrame* __restrict__ frames,
    const SgFftGeom* __restrict__ geoms, const float* __restrict__ fl, float* __restrict__ fs,
    float* __restrict__ slotmax) {
  stft_ola_body<SG_FRAME_NOISE>(segs, olas, frames, geoms, fl, fs, slotmax);
}

// Test probe: wavefront w transforms frame w (M complex points, in place) with
// the stage kernels of sg_stft_ola (the specialised M = 1102 path, radix-29 stage
// on the matrix pipe, when the geometry is that one); inverse = conjugate
// twiddles, no scaling. LDS: twS, twN (M pairs each), the frame, the radix-29 table.
extern "C" __global__ __launch_bounds__(64) void sg_fft_probe(const SgFftGeom* __restrict__ geom,
                                                              const float* __restrict__ fl, float2* __restrict__ data,
                                                              int inverse) {
  extern __shared__ float4 lds4[];
  const SgFftGeom& g = geom[0];
  const int M = g.M, lane = threadIdx.x;
  float2* twS = reinterpret_cast<float2*>(lds4);
  float2* twN = twS + M;
  float2* A = twN + M;
  float4* A29 = reinterpret_cast<float4*>(A + M);
  const float2* tsg = reinterpret_cast<const float2*>(fl + g.tws);
  const float2* tng = reinterpret_cast<const float2*>(fl + g.tw) + M;
  float2* d = data + (int64_t)blockIdx.x * M;
  for (int t = lane; t < M; t += 64) {
    if (t < M - 1) twS[t] = tsg[t];
    twN[t] = tng[t];
    A[t] = d[t];
  }
  if (geom_1102(g)) mat29_fill(A29, tng, lane);
  sg_wave_fence();
  if (geom_1102(g)) {  // inverse bit 1: the VALU radix-29 stage (sg_stft_ola_noise's)
    if (inverse == 1) fft_wc<true, 1102, 29, 19, 2>(A, twS, A29, lane);
    else if (inverse == 3) fft_wc<true, 1102, 29, 19, 2, false>(A, twS, A29, lane);
    else if (inverse == 2) fft_wc<false, 1102, 29, 19, 2, false>(A, twS, A29, lane);
    else fft_wc<false, 1102, 29, 19, 2>(A, twS, A29, lane);
  } else if (inverse & 1) {
    fft_w<true>(A, g, twS, lane);
  } else {
    fft_w<false>(A, g, twS, lane);
  }
  for (int t = lane; t < M; t += 64) d[t] = A[t];
}

using sgd::contour_at;
__device__ __forceinline__ float wave_max_f(float v) { return sgd::wave_max(v); }

#ifndef SG_OLA_PF
#define SG_OLA_PF 4  // frames per sample read together (wl / hop = 4 at seewave's 75 % overlap)
#endif
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
    if (p >= 0 && p < O.xlen && O.hi > 0) {
      // whole-sample hop: frames f with f hi <= p < f hi + wl
      const int pi = (int)p;
      int f = pi / O.hi;
      if (f > O.nframes - 1) f = O.nframes - 1;
      int i = pi - f * O.hi;
      const float* fr0 = fs + O.frames;
      // the first SG_OLA_PF frames' reads issued together (clamped to frame f, sample i),
      // then added in frame order as the loop below adds them
      constexpr int PF = SG_OLA_PF;
      float v[PF];
#pragma unroll
      for (int t = 0; t < PF; ++t) {
        const bool ok = f - t >= 0 && i + t * O.hi < O.wl;
        v[t] = fr0[ok ? (int64_t)(f - t) * O.wl + i + t * O.hi : (int64_t)f * O.wl + i];
      }
#pragma unroll
      for (int t = 0; t < PF; ++t)
        if (f - t >= 0 && i + t * O.hi < O.wl) acc += v[t];
      for (f -= PF, i += PF * O.hi; f >= 0 && i < O.wl; --f, i += O.hi) acc += fr0[(int64_t)f * O.wl + i];
      acc *= O.scale;
    } else if (p >= 0 && p < O.xlen) {
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
  const int nt = O.nslot;
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

[[maybe_unused]] constexpr int SG_MIX_KMAX = 32;  // knots of an LDS-staged contour
__device__ __forceinline__ float fade_in_out(int lf, int64_t L, int64_t k) {  // fadeInOut(), R/utilities_soundgen.R:440-459
  float f = 1.f;
  if (lf < 2) return f;
  const float by = 1.f / (float)(lf - 1);
  if (k < lf) f *= (k == lf - 1) ? 1.f : (float)k * by;
  const int64_t kb = L - 1 - k;
  if (kb < lf) f *= (kb == lf - 1) ? 1.f : (float)kb * by;
  return f;
}

// ------------------------------------------------ fp64 filter frames
// Frames of an ill-conditioned formant-filter call (SgFrame64; planner:
// filter_conditioning): seewave's stft x env -> istft in fp64, one frame of an
// even window length N = 2M per 256-thread workgroup (M <= 2048):
//   forward: the M-point complex DFT of z_n = x_2n + i x_2n+1 (x = hamming x
//            fp64 sound), untangled to X_k = E_k + W_N^k O_k;  Y_k = X_k / N env_k
//   inverse: seewave's Hermitian extension X' (X'_M = Re Y_{M-1}, seewave.r:3474)
//            packed as Z_k = (X'_k + X'_{k+M}) + i W_N^-k (X'_k - X'_{k+M}); its
//            M-point inverse DFT gives x_2n + i x_2n+1; / N x hann, stored fp32 for
//            the overlap-add (sg_ola; that round-off is relative to the filtered
//            output, ~1e-8 RMS)
// Stockham autosort, out of place between two M-point LDS buffers (35 KB for
// wl = 2204: 4 workgroups per CU). Per stage of radix R: (a) every input times
// its twiddle, in place; (b) odd R: one work item per (butterfly, output pair k,
// R - k) from the symmetric sums x_m +- x_{R-m} (all threads busy for R = 19,
// 29), R = 2, 4: one item per butterfly. (Grouping several outputs per item so each
// input pair is read once measured no better: r04d, +2 % at 3, +21 % at 2 per item.) Roots of unity W_N^t from an fp64 table
// in global memory, one per window length (sg_roots64), L2-resident.
constexpr int SG_F64_THREADS = 256;  // threads per fp64 frame (r04: 128 / 512 / 1,024 slower)
namespace {
__device__ __forceinline__ double2 cmul64(double2 a, double2 b) {
  return make_double2(fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ double2 conj_if(double2 w, bool c) { return c ? make_double2(w.x, -w.y) : w; }
// one radix-R stage of an M-point frame, src -> dst; TN = W_N^t, t < N = 2M; rt = W_R^t.
// CM, CNS > 0: frame size and stage stride as compile-time constants (the dominant
// geometry, M = 1102 = 2 x 19 x 29): every division and modulo folds to shifts and
// multiplies, the odd butterflies' root index steps by k instead of (m k) mod R.
template <int R, int CM = 0, int CNS = 0>
__device__ void stage64(double2* __restrict__ src, double2* __restrict__ dst, int M_, int Ns_,
                        const double2* __restrict__ TN, const double2* __restrict__ rt, bool inv) {
  const int M = CM ? CM : M_, Ns = CNS ? CNS : Ns_;
  const int nR = M / R, tstep2 = 2 * (M / (Ns * R));  // W_{Ns R}^e = W_N^(2 e M / (Ns R))
  if (Ns > 1) {  // (a) input j + r nR of butterfly j times W_{Ns R}^(r (j mod Ns)), in place
    for (int q = threadIdx.x; q < M; q += SG_F64_THREADS) {
      const int r = q / nR, jm = (q - r * nR) % Ns;
      if (r != 0 && jm != 0) src[q] = cmul64(src[q], conj_if(TN[r * jm * tstep2], inv));
    }
    __syncthreads();
  }
  if constexpr (R == 2 || R == 4) {
    for (int j = threadIdx.x; j < nR; j += SG_F64_THREADS) {
      const int jm = j % Ns;
      const double2* x = src + j;
      double2* y = dst + (j - jm) * R + jm;
      if constexpr (R == 2) {
        const double2 u = x[0], v = x[nR];
        y[0] = make_double2(u.x + v.x, u.y + v.y);
        y[Ns] = make_double2(u.x - v.x, u.y - v.y);
      } else {
        const double2 a = x[0], b = x[nR], c = x[2 * nR], d = x[3 * nR];
        const double2 s0 = make_double2(a.x + c.x, a.y + c.y), d0 = make_double2(a.x - c.x, a.y - c.y);
        const double2 s1 = make_double2(b.x + d.x, b.y + d.y), d1 = make_double2(b.x - d.x, b.y - d.y);
        // forward: y1 = d0 - i d1, y3 = d0 + i d1 (inverse: swapped)
        const double2 mm = make_double2(d0.x + d1.y, d0.y - d1.x), mp = make_double2(d0.x - d1.y, d0.y + d1.x);
        y[0] = make_double2(s0.x + s1.x, s0.y + s1.y);
        y[Ns] = inv ? mp : mm;
        y[2 * Ns] = make_double2(s0.x - s1.x, s0.y - s1.y);
        y[3 * Ns] = inv ? mm : mp;
      }
    }
  } else {
    // y_k = x_0 + sum_m A_m c_mk -/+ i sum_m B_m s_mk (forward -, inverse +), y_{R-k} the
    // other sign; A_m = x_m + x_{R-m}, B_m = x_m - x_{R-m}; item k = 0: y_0 = x_0 + sum A_m
    constexpr int H = (R - 1) / 2;
    for (int i = threadIdx.x; i < nR * (H + 1); i += SG_F64_THREADS) {
      const int k = i % (H + 1), j = i / (H + 1), jm = j % Ns;
      const double2* x = src + j;
      double2* y = dst + (j - jm) * R + jm;
      const double2 x0 = x[0];
      double2 P = make_double2(0.0, 0.0), Q = make_double2(0.0, 0.0);
      int t = 0;  // (m k) mod R
#pragma unroll 2
      for (int m = 1; m <= H; ++m) {
        t += k;
        if (t >= R) t -= R;
        const double2 u = x[m * nR], v = x[(R - m) * nR];
        const double2 w = k == 0 ? make_double2(1.0, 0.0) : rt[t];  // (cos, -sin) of 2 pi m k / R
        P.x = fma(u.x + v.x, w.x, P.x);
        P.y = fma(u.y + v.y, w.x, P.y);
        Q.x = fma(u.x - v.x, -w.y, Q.x);
        Q.y = fma(u.y - v.y, -w.y, Q.y);
      }
      const double2 ya = make_double2(x0.x + P.x + Q.y, x0.y + P.y - Q.x);
      const double2 yb = make_double2(x0.x + P.x - Q.y, x0.y + P.y + Q.x);
      if (k == 0) {
        y[0] = ya;
      } else {
        y[k * Ns] = inv ? yb : ya;
        y[(R - k) * Ns] = inv ? ya : yb;
      }
    }
  }
  __syncthreads();
}
// M-point complex DFT of *a (result in *a, *b scratch); TN: W_N^t (t < 2M), global; rt: LDS (32)
__device__ void fft64(double2*& a, double2*& b, int M, const double2* __restrict__ TN,
                                   double2* __restrict__ rt, bool inv) {
  if (M == 1102) {  // 2 x 19 x 29, the stage order of the loop below, sizes folded
    stage64<2, 1102, 1>(a, b, M, 1, TN, rt, inv);
    if (threadIdx.x < 19) rt[threadIdx.x] = TN[threadIdx.x * (2 * 1102 / 19)];
    __syncthreads();
    stage64<19, 1102, 2>(b, a, M, 2, TN, rt, inv);  // ends with a barrier: its root reads are done
    if (threadIdx.x < 29) rt[threadIdx.x] = TN[threadIdx.x * (2 * 1102 / 29)];
    __syncthreads();
    stage64<29, 1102, 38>(a, b, M, 38, TN, rt, inv);
    double2* t = a; a = b; b = t;  // three stages: the result is in b -> swap as the loop does
    return;
  }
  int rest = M, Ns = 1;
  while (rest > 1) {
    int R = rest % 4 == 0 ? 4 : rest % 2 == 0 ? 2 : 0;
    if (!R)
      for (int p : {3, 5, 7, 11, 13, 17, 19, 23, 29, 31})
        if (rest % p == 0) { R = p; break; }
    if (R != 2 && R != 4) {  // odd radix: W_R^t = W_N^(t 2M / R), t < R
      if (threadIdx.x < R) rt[threadIdx.x] = TN[threadIdx.x * (2 * M / R)];
      __syncthreads();
    }
    switch (R) {
#define SG_S64(RR) case RR: stage64<RR>(a, b, M, Ns, TN, rt, inv); break;
      SG_S64(2) SG_S64(3) SG_S64(4) SG_S64(5) SG_S64(7) SG_S64(11) SG_S64(13) SG_S64(17) SG_S64(19) SG_S64(23)
      SG_S64(29) SG_S64(31)
#undef SG_S64
      default: return;  // the planner only sends 31-smooth M
    }
    double2* t = a; a = b; b = t;
    Ns *= R;
    rest /= R;
  }
}
}  // namespace

// Per window length N = 2M of the plan's fp64 frames: W_N^t = exp(-2 pi i t / N), t < N,
// then seewave's hamming and hanning (ftwindow) as pairs (w[2n], w[2n + 1]), n < M
extern "C" __global__ __launch_bounds__(256) void sg_roots64(const int32_t* __restrict__ wls,
                                                             const int64_t* __restrict__ offs,
                                                             double2* __restrict__ tabs) {
  const int N = wls[blockIdx.y], M = N / 2;
  double2* T = tabs + offs[blockIdx.y];
  const double wd = (double)(N - 1);
  for (int t = blockIdx.x * 256 + threadIdx.x; t < N; t += gridDim.x * 256) {
    double sn, cs;
    sincospi(-2.0 * (double)t / (double)N, &sn, &cs);
    T[t] = make_double2(cs, sn);
  }
  for (int n = blockIdx.x * 256 + threadIdx.x; n < M; n += gridDim.x * 256) {
    const double c0 = cospi(2.0 * (double)(2 * n) / wd), c1 = cospi(2.0 * (double)(2 * n + 1) / wd);
    T[N + n] = make_double2(0.54 - 0.46 * c0, 0.54 - 0.46 * c1);
    T[N + M + n] = make_double2(0.5 - 0.5 * c0, 0.5 - 0.5 * c1);
  }
}

extern "C" __global__ __launch_bounds__(SG_F64_THREADS) void sg_fft_frames64(
    const SgFrame64* __restrict__ frames, const int64_t* __restrict__ frame_tab, const double2* __restrict__ tabs,
    const float* __restrict__ fl, const double* __restrict__ fh, float* __restrict__ fs) {
  extern __shared__ double2 lds64[];
  const SgFrame64 F = frames[blockIdx.x];
  const int N = F.wl, M = N / 2;
  const double2* __restrict__ TN = tabs + frame_tab[blockIdx.x];
  double2* a = lds64;        // M points
  double2* b = a + M;        // M points
  double2* rt = b + M;       // radix roots (<= 31)
  const double2* __restrict__ ham = TN + N;  // window pairs (sg_roots64)
  const double2* __restrict__ han = ham + M;
  const bool noise = F.mode == SG_F64_NOISE;
  if (!noise) {
    const double* x = fh + F.src;
    for (int n = threadIdx.x; n < M; n += SG_F64_THREADS) {  // hamming (seewave ftwindow), packed pairs
      const double2 h = ham[n];
      a[n] = make_double2(x[2 * n] * h.x, x[2 * n + 1] * h.y);
    }
    __syncthreads();
    fft64(a, b, M, TN, rt, false);
  }
  // FILTER: untangle, / N, x env; NOISE: uniforms x filter (real); Y_k, k < M; then
  // seewave's Hermitian extension, packed for the inverse (-> b)
  const double invN = 1.0 / (double)N;
  const float* env = fl + F.env;
  const float* uni = fl + F.src;
  auto Yat = [&](int kk) -> double2 {  // Y_kk, 0 <= kk < M
    if (noise) return make_double2((double)uni[kk] * (double)env[kk], 0.0);
    const double2 p = a[kk], q = a[kk == 0 ? 0 : M - kk], w = TN[kk];
    const double2 e = make_double2(0.5 * (p.x + q.x), 0.5 * (p.y - q.y));
    const double2 o = make_double2(0.5 * (p.y + q.y), -0.5 * (p.x - q.x));
    const double2 xk = make_double2(e.x + (o.x * w.x - o.y * w.y), e.y + (o.x * w.y + o.y * w.x));
    const double sc = invN * (double)env[kk];
    return make_double2(xk.x * sc, xk.y * sc);
  };
  for (int k = threadIdx.x; k < M; k += SG_F64_THREADS) {
    const double2 yk = Yat(k);
    double2 yh;  // X'_{k+M}: Re Y_{M-1} for k = 0, else conj(Y_{M-k})
    if (k == 0) { const double2 t = Yat(M - 1); yh = make_double2(t.x, 0.0); }
    else { const double2 t = Yat(M - k); yh = make_double2(t.x, -t.y); }
    const double2 sm = make_double2(yk.x + yh.x, yk.y + yh.y), df = make_double2(yk.x - yh.x, yk.y - yh.y);
    const double2 t = cmul64(df, conj_if(TN[k], true));  // W_N^-k (X'_k - X'_{k+M})
    b[k] = make_double2(sm.x - t.y, sm.y + t.x);
  }
  __syncthreads();
  double2* c = b;
  double2* d = a;
  fft64(c, d, M, TN, rt, true);
  float* out = fs + F.dst;
  for (int n = threadIdx.x; n < M; n += SG_F64_THREADS) {
    const double2 h = han[n];
    out[2 * n] = (float)(c[n].x * invN * h.x);
    out[2 * n + 1] = (float)(c[n].y * invN * h.y);
  }
}

// ---- fp64 frames of the dominant geometry (wl = 2204, M = 1102 = 29 x 19 x 2), one frame
// per wavefront (round 5). sg_fft_frames64 spreads a frame over a 256-thread workgroup
// with a barrier per stage and one work item per odd-prime output pair, which reads all
// R inputs of its butterfly from LDS (O(R^2) LDS reads per butterfly): LDS-bound at
// ~17k CU-cycles per frame. Here a lane holds its butterfly's inputs in registers (R
// reads, R writes), the stages are wave-synchronous (no barrier), and the work is the
// fp64 FMAs. The arithmetic is sg_fft_frames64's (the same symmetric odd-prime form,
// roots and twiddles from the sg_roots64 table); the stage order is 29, 19, 2 so that
// the heaviest stage needs no twiddles and the radix-2 stage works in place.
constexpr int SG_F64W_WAVES = 8;  // frames per workgroup: 8 x 17.6 KB of LDS, 2 waves per SIMD
constexpr int SG_F64W_M = SG_F64W_M_HOST;
namespace {
// radix-R (odd) butterfly of the R inputs x[] -> y_k at dst[k * ys] (in registers until
// written); c[t], s[t] = cos, sin (2 pi t / R), t <= H: wave-uniform (scalar registers),
// the index (m k) mod R folds at compile time (a root t > H is t' = R - t with the sine
// negated); inv: inverse (outputs k and R - k swapped)
template <int R>
__device__ __forceinline__ void bfly64_store(double2 (&x)[R], double2* dst, int ys, const double (&c)[(R - 1) / 2 + 1],
                                             const double (&s)[(R - 1) / 2 + 1], bool inv) {
  constexpr int H = (R - 1) / 2;
  double2 y0 = x[0];
#pragma unroll
  for (int m = 1; m <= H; ++m) {  // A_m = x_m + x_{R-m} in x[m], B_m = x_m - x_{R-m} in x[R - m]
    const double2 u = x[m], v = x[R - m];
    x[m] = make_double2(u.x + v.x, u.y + v.y);
    x[R - m] = make_double2(u.x - v.x, u.y - v.y);
    y0.x += x[m].x;
    y0.y += x[m].y;
  }
  dst[0] = y0;
#pragma unroll
  for (int k = 1; k <= H; ++k) {
    double2 P = make_double2(0.0, 0.0), Q = make_double2(0.0, 0.0);
#pragma unroll
    for (int m = 1; m <= H; ++m) {
      const int t = (m * k) % R;
      const double wc = t <= H ? c[t] : c[R - t];
      const double ws = t <= H ? s[t] : -s[R - t];  // sin (2 pi t / R)
      P.x = fma(x[m].x, wc, P.x);
      P.y = fma(x[m].y, wc, P.y);
      Q.x = fma(x[R - m].x, ws, Q.x);
      Q.y = fma(x[R - m].y, ws, Q.y);
    }
    const double2 x0 = x[0];
    const double2 ya = make_double2(x0.x + P.x + Q.y, x0.y + P.y - Q.x);
    const double2 yb = make_double2(x0.x + P.x - Q.y, x0.y + P.y + Q.x);
    dst[k * ys] = inv ? yb : ya;
    dst[(R - k) * ys] = inv ? ya : yb;
  }
}
// the roots of a radix-R stage from the frame's W_N table (wave-uniform loads): W_R^t = W_N^(t N / R) = (cos, -sin)
template <int R>
__device__ __forceinline__ void roots64(const double2* __restrict__ TN, int N, double (&c)[(R - 1) / 2 + 1],
                                        double (&s)[(R - 1) / 2 + 1]) {
#pragma unroll
  for (int t = 0; t <= (R - 1) / 2; ++t) {
    const double2 w = TN[t * (N / R)];
    c[t] = w.x;
    s[t] = -w.y;
  }
}

// the M = 1102 transform of frame A (in place, LDS), forward or inverse; TN = W_N^t, t < N.
// Each stage's twiddles are loaded one stage ahead (their latency under the previous
// stage's arithmetic).
// The caller owns tw2 (radix 2's twiddles, loaded here one stage ahead); the radix-2
// stage itself runs only without SKIP2 (the callers fuse it with the untangle or the output)
// xs (forward filter frames): the first stage reads the frame straight from the fp64
// sound times hamming (hm) instead of from A (no LDS pass for the window)
template <bool SKIP2 = false>
__device__ __forceinline__ void fft64w_1102(double2* A, const double2* __restrict__ TN, bool inv, int lane,
                                            double2 (&tw2)[9], const double* __restrict__ xs = nullptr,
                                            const double2* __restrict__ hm = nullptr) {
  constexpr int N = 2 * SG_F64W_M;
  // radix 19's twiddles W_551^(r jm) = W_2204^(4 r jm), jm = j mod 29 (j = lane < 58)
  const int j19 = lane < 58 ? lane : 0, jm19 = j19 < 29 ? j19 : j19 - 29;
  double2 tw19[19];
#pragma unroll
  for (int r = 1; r < 19; ++r) tw19[r] = TN[4 * r * jm19];
  // radix 29 (Ns = 1, 38 butterflies): inputs j + 38 r, outputs 29 j + k
  {
    double c[15], sn[15];
    roots64<29>(TN, N, c, sn);
    double2 x[29];
    const int j = lane < 38 ? lane : 0;
    if (xs) {
#pragma unroll
      for (int r = 0; r < 29; ++r) {
        const int n = j + 38 * r;
        const double2 h = hm[n];
        x[r] = make_double2(xs[2 * n] * h.x, xs[2 * n + 1] * h.y);
      }
    } else {
#pragma unroll
      for (int r = 0; r < 29; ++r) x[r] = A[j + 38 * r];
    }
    sg_wave_fence();  // every read of the stage before the first write
    if (lane < 38) bfly64_store<29>(x, A + 29 * j, 1, c, sn, inv);
    sg_wave_fence();
  }
  // radix 2's twiddles W_1102^j = W_2204^(2 j), j = 64 i + lane
#pragma unroll
  for (int i = 0; i < 9; ++i) tw2[i] = TN[2 * min(64 * i + lane, 550)];
  // radix 19 (Ns = 29, 58 butterflies): inputs j + 58 r times W_551^(r jm), outputs
  // 19 (j - jm) + jm + 29 k
  {
    double c[10], sn[10];
    roots64<19>(TN, N, c, sn);
    double2 x[19];
#pragma unroll
    for (int r = 0; r < 19; ++r) {
      const double2 v = A[j19 + 58 * r];
      x[r] = r == 0 || jm19 == 0 ? v : cmul64(v, conj_if(tw19[r], inv));
    }
    sg_wave_fence();
    if (lane < 58) bfly64_store<19>(x, A + 19 * (j19 - jm19) + jm19, 29, c, sn, inv);
    sg_wave_fence();
  }
  if constexpr (SKIP2) return;
  // radix 2 (Ns = 551, 551 butterflies): j and j + 551, the second times W_1102^j; in place
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int j = 64 * i + lane;
    if (j < 551) {
      const double2 u = A[j], v = cmul64(A[j + 551], conj_if(tw2[i], inv));
      A[j] = make_double2(u.x + v.x, u.y + v.y);
      A[j + 551] = make_double2(u.x - v.x, u.y - v.y);
    }
  }
  sg_wave_fence();
}
}  // namespace

extern "C" __global__ __launch_bounds__(SG_F64W_WAVES * 64) void sg_fft_frames64w(
    const SgFrame64* __restrict__ frames, int64_t nframes, const int64_t* __restrict__ frame_tab,
    const double2* __restrict__ tabs, const float* __restrict__ fl, const double* __restrict__ fh,
    float* __restrict__ fs) {
  constexpr int M = SG_F64W_M, N = 2 * M, half = M / 2;
  extern __shared__ double2 lds64w[];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  double2* A = lds64w + (int64_t)w * M;
  const int64_t f = (int64_t)blockIdx.x * SG_F64W_WAVES + w;
  if (f >= nframes) return;  // no workgroup barrier below
  const SgFrame64 F = frames[f];
  const double2* __restrict__ TN = tabs + frame_tab[f];
  const double2* __restrict__ ham = TN + N;
  const double2* __restrict__ han = ham + M;
  const bool noise = F.mode == SG_F64_NOISE;
  const double invN = 1.0 / (double)N;
  const float* env = fl + F.env;
  double2 tw2[9];
  // FILTER: untangle, / N, x env; NOISE: uniforms x filter (real). Then seewave's
  // Hermitian extension packed for the inverse: slot k <- Y_k and conj Y_{M-k} (k = 0:
  // Re Y_{M-1}). Lane pair k owns slots k and M - k; the k = 0 lane also reads slots 1
  // and M - 1 (pair 1's), before any write of the round.
  const float* uni = fl + F.src;
  auto Yat = [&](int kk, double2 p, double2 q) -> double2 {  // Y_kk from Z_kk = p, Z_{M-kk} = q
    if (noise) return make_double2((double)uni[kk] * (double)env[kk], 0.0);
    const double2 wk = TN[kk];
    const double2 e = make_double2(0.5 * (p.x + q.x), 0.5 * (p.y - q.y));
    const double2 o = make_double2(0.5 * (p.y + q.y), -0.5 * (p.x - q.x));
    const double2 xk = make_double2(e.x + (o.x * wk.x - o.y * wk.y), e.y + (o.x * wk.y + o.y * wk.x));
    const double sc = invN * (double)env[kk];
    return make_double2(xk.x * sc, xk.y * sc);
  };
  auto pack = [&](int k, double2 yk, double2 yh) -> double2 {  // yh = X'_{k+M}
    const double2 sm = make_double2(yk.x + yh.x, yk.y + yh.y), df = make_double2(yk.x - yh.x, yk.y - yh.y);
    const double2 t = cmul64(df, conj_if(TN[k], true));  // W_N^-k (X'_k - X'_{k+M})
    return make_double2(sm.x - t.y, sm.y + t.x);
  };
  if (!noise) {
    // the forward transform's radix-2 stage fused with the untangle (as the fp32
    // r2_untangle_1102): butterflies u and 551 - u give Z[u], Z[M - u], Z[551 - u],
    // Z[551 + u], i.e. the pairs (u, M - u) and (551 - u, 551 + u); lane 0 also takes
    // butterfly 0 and the pairs k = 0 and k = 551 (self-paired)
    fft64w_1102<true>(A, TN, false, lane, tw2, fh + F.src, ham);  // hamming (seewave ftwindow) in the first stage's loads
    auto bfly = [&](int j, double2& z0, double2& z1) {  // stage 2's operations, forward
      const double2 u = A[j], v = cmul64(A[j + half], TN[2 * j]);
      z0 = make_double2(u.x + v.x, u.y + v.y);
      z1 = make_double2(u.x - v.x, u.y - v.y);
    };
    auto pair = [&](int kk, double2 p, double2 q) {  // Z_kk = p, Z_{M-kk} = q
      const double2 yk = Yat(kk, p, q), ym = Yat(M - kk, q, p);
      A[kk] = pack(kk, yk, make_double2(ym.x, -ym.y));
      A[M - kk] = pack(M - kk, ym, make_double2(yk.x, -yk.y));
    };
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      const int u = 1 + lane + 64 * q;
      if (u > 275) continue;
      const int v = half - u;
      double2 zu, zuh, zv, zvh;  // Z[u], Z[u + 551], Z[v], Z[v + 551] = Z[M - u]
      bfly(u, zu, zuh);
      bfly(v, zv, zvh);
      if (q == 0 && lane == 0) {  // u = 1: Z[1] = zu, Z[M - 1] = zvh
        double2 z0, zh;
        bfly(0, z0, zh);
        const double2 y0 = Yat(0, z0, z0), yl = Yat(M - 1, zvh, zu);
        A[0] = pack(0, y0, make_double2(yl.x, 0.0));
        const double2 yh = Yat(half, zh, zh);
        A[half] = pack(half, yh, make_double2(yh.x, -yh.y));
      }
      pair(u, zu, zvh);
      pair(v, zv, zuh);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int k = 64 * i + lane;
      if (k > half) continue;
      const int km = k == 0 ? 0 : M - k;
      const double2 z = make_double2(0.0, 0.0);  // noise: Y from the uniforms alone
      if (k == 0) {
        const double2 y0 = Yat(0, z, z), yl = Yat(M - 1, z, z);
        A[0] = pack(0, y0, make_double2(yl.x, 0.0));
      } else {
        const double2 yk = Yat(k, z, z), ym = Yat(km, z, z);
        A[k] = pack(k, yk, make_double2(ym.x, -ym.y));
        if (km != k) A[km] = pack(km, ym, make_double2(yk.x, -yk.y));
      }
    }
  }
  sg_wave_fence();
  // the inverse transform's radix-2 stage fused with the output: butterfly j's two points
  // are the frame's samples 2j, 2j + 1 and 2j + 1102, 2j + 1103 (/ N x hann), stored
  // without a pass through LDS
  fft64w_1102<true>(A, TN, true, lane, tw2);
  float* out = fs + F.dst;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int j = 64 * i + lane;
    if (j < half) {
      const double2 u = A[j], v = cmul64(A[j + half], conj_if(tw2[i], true));
      const double2 c0 = make_double2(u.x + v.x, u.y + v.y), c1 = make_double2(u.x - v.x, u.y - v.y);
      const double2 h0 = han[j], h1 = han[j + half];
      out[2 * j] = (float)(c0.x * invN * h0.x);
      out[2 * j + 1] = (float)(c0.y * invN * h0.y);
      out[2 * (j + half)] = (float)(c1.x * invN * h1.x);
      out[2 * (j + half) + 1] = (float)(c1.y * invN * h1.y);
    }
  }
}

// Gathered noise uniforms (upload time): one workgroup per noise item copies its
// draws from the union of the injected ranges into the uniform area, zero-padded
extern "C" __global__ __launch_bounds__(256) void sg_ugather(const SgUJob* __restrict__ jobs,
                                                             const float* __restrict__ us, float* __restrict__ fl) {
  const SgUJob J = jobs[blockIdx.x];
  for (int64_t j = threadIdx.x; j < J.ntot; j += 256) fl[J.dst + j] = j < J.n ? us[J.src + j] : 0.f;
}

#ifndef SG_MIX_E
#define SG_MIX_E 4  // samples per thread and chunk
#endif
#ifndef SG_MIX_WAVES
#define SG_MIX_WAVES 8
#endif
// HP: the pre-filter sound of an fp64 bout: fp64 sum into fh (X.to_fs == 2), voiced
// items (SG_ITEM_F64) read from fh, noise items from fs
template <bool HP>
__device__ __forceinline__ void mix_body(const SgMixTile* __restrict__ tiles, const SgMix* __restrict__ mixes,
                                         const SgNoiseItem* __restrict__ items, const float* __restrict__ olamax,
                                         const double* __restrict__ cknots, const float* __restrict__ fl,
                                         float* __restrict__ fs, float* __restrict__ out, double* __restrict__ fh) {
  using V = typename std::conditional<HP, double, float>::type;
  const SgMixTile T = tiles[blockIdx.x];
  const SgMix& X = mixes[T.mix];
  V* __restrict__ dst;
  if constexpr (HP) dst = fh;
  else dst = X.to_fs ? fs : out;
  // samples per thread and chunk (r04: 4 at 8 waves per SIMD, 1.83 -> 1.74 ms per C5 launch over 8 at 5)
  constexpr int E = SG_MIX_E;
  const int64_t kend = T.k0 + SG_MIX_TILE < X.len ? T.k0 + SG_MIX_TILE : X.len;
  // per-tile constants, hoisted out of the sample loops (one scalar-load burst)
  const float base_scale = X.base_kind == SG_BASE_NORM ? 1.f / olamax[X.base_ola] : 1.f;
  const bool has_base = X.base_kind != SG_BASE_NONE;
  // contour interval cursors (sgd::contour_at_cursor): a thread's samples of an
  // item only move forward, so after one bisection each lookup is a step
  constexpr int NC = 8;  // items with an LDS-held cursor per thread
  __shared__ int curs[NC][256];
  for (int i = 0; i < NC && i < X.nitems; ++i) curs[i][threadIdx.x] = -1;
  int mcur = -1;
  // spline contours (kind 3, <= SG_MIX_KMAX knots) of the mult envelope (slot NC) and
  // the first NC items staged in LDS: the per-sample interval walk and the five
  // coefficient loads then hit LDS instead of a dependent chain of global loads
  __shared__ double cks[NC + 1][5 * SG_MIX_KMAX];
  auto lds_ok = [&](const SgContour& c) { return c.kind == 3 && c.nk <= SG_MIX_KMAX; };
  for (int i = 0; i <= NC; ++i) {
    if (i < NC && i >= X.nitems) continue;
    const SgContour& c = i == NC ? X.mult : items[X.item0 + i].strength;
    if (!lds_ok(c)) continue;
    const double* src = cknots + c.k_off;
    for (int j = threadIdx.x; j < 5 * c.nk; j += 256) cks[i][j] = src[j];
  }
  __syncthreads();
#pragma unroll 1
  for (int64_t kc = T.k0; kc < kend; kc += E * 256) {
    V v[E];
    // loads are unconditional (clamped addresses), selects afterwards: a load
    // under a branch is followed by its own vmcnt(0) wait, serialising the chunk
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t k = kc + e * 256 + threadIdx.x;
      const bool in = has_base && k < kend && k < X.base_len;
      const float x = fs[X.base + (in ? k : 0)];
      v[e] = in ? (V)(x * base_scale) : (V)0;
    }
    // noise items: descriptor once per chunk, then its samples (addVectors)
    for (int i = 0; i < X.nitems; ++i) {
      const SgNoiseItem& it = items[X.item0 + i];
      const int64_t j0 = kc + threadIdx.x - it.off;
      if (j0 + (E - 1) * 256 < 0 || j0 >= it.len) continue;  // no sample of this thread in the item
      const float nscale = it.ola >= 0 ? 1.f / olamax[it.ola] : 1.f;
      const bool flat = it.strength.kind == 1;
      // the chunk's samples of the item all inside its fade ramps' complement: factor 1
      // exactly (wave-uniform test on the chunk's item range [jc, jc + E 256))
      const int64_t jc = kc - it.off;
      const bool ramp = it.fade >= 2 && (jc < it.fade || jc + E * 256 > it.len - it.fade);
      const float sflat = flat ? (float)contour_at(it.strength, cknots, it.len, 0) : 1.f;
      V raw[E];
      const bool f64 = HP && (it.flags & SG_ITEM_F64);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int64_t j = j0 + e * 256;
        const int64_t jj = it.raw + (j < 0 ? 0 : (j >= it.len ? it.len - 1 : j));
        if constexpr (HP) raw[e] = f64 ? fh[jj] : (V)fs[jj];
        else raw[e] = fs[jj];
      }
      int cur = i < NC ? curs[i][threadIdx.x] : -1;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int64_t k = kc + e * 256 + threadIdx.x, j = j0 + e * 256;
        if (k >= kend || j < 0 || j >= it.len) continue;
        V nv = raw[e] * (V)nscale;
        if (flat) nv *= (V)sflat;
        else if (it.strength.kind != 0) {
          if (i < NC && lds_ok(it.strength)) {
            SgContour cl = it.strength;
            cl.k_off = 0;
            nv = (V)((double)nv * sgd::contour_at_cursor(cl, &cks[i][0], it.len, j, cur));
          } else
            nv = (V)((double)nv * sgd::contour_at_cursor(it.strength, cknots, it.len, j, cur));
        }
        if (ramp) nv *= (V)fade_in_out(it.fade, it.len, j);
        v[e] += nv;
      }
      if (i < NC) curs[i][threadIdx.x] = cur;
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t k = kc + e * 256 + threadIdx.x;
      if (X.mult.kind != 0 && k < kend) {
        if (lds_ok(X.mult)) {
          SgContour cl = X.mult;
          cl.k_off = 0;
          v[e] = (V)((double)v[e] * sgd::contour_at_cursor(cl, &cks[NC][0], X.len, k, mcur));
        } else
          v[e] = (V)((double)v[e] * sgd::contour_at_cursor(X.mult, cknots, X.len, k, mcur));
      }
      if (X.am_lo > 0) v[e] *= (V)(1.f - sigmoid_at(fl + X.am_tab, X.am_lo, k) * X.am_dep / 100.f);
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t k = kc + e * 256 + threadIdx.x;
      if (k < kend) dst[X.dst + k] = v[e];
    }
  }
}

// sg_mix's registers capped for 8 waves per SIMD (r04: 94 VGPRs = 5 waves uncapped)
#define SG_MIX_ATTR __attribute__((amdgpu_waves_per_eu(SG_MIX_WAVES)))
extern "C" __global__ __launch_bounds__(256) SG_MIX_ATTR void sg_mix(const SgMixTile* __restrict__ tiles,
                                                         const SgMix* __restrict__ mixes,
                                                         const SgNoiseItem* __restrict__ items,
                                                         const float* __restrict__ olamax,
                                                         const double* __restrict__ cknots,
                                                         const float* __restrict__ fl, float* __restrict__ fs,
                                                         float* __restrict__ out) {
  mix_body<false>(tiles, mixes, items, olamax, cknots, fl, fs, out, nullptr);
}
extern "C" __global__ __launch_bounds__(256) void sg_mix_hp(const SgMixTile* __restrict__ tiles,
                                                            const SgMix* __restrict__ mixes,
                                                            const SgNoiseItem* __restrict__ items,
                                                            const float* __restrict__ olamax,
                                                            const double* __restrict__ cknots,
                                                            const float* __restrict__ fl, float* __restrict__ fs,
                                                            double* __restrict__ fh) {
  mix_body<true>(tiles, mixes, items, olamax, cknots, fl, fs, nullptr, fh);
}

// ---------------------------------------------------------------- launchers
#include "sg_exec.h"

#include <map>
#include <mutex>
namespace sg {
// launch failures (bad configuration, LDS over the opted-in size) are loud
#define SG_LAUNCHED(name)                                                                       \
  do {                                                                                          \
    const hipError_t _e = hipGetLastError();                                                    \
    if (_e != hipSuccess) throw SgError(SG_E_DEVICE, std::string("launch " name ": ") + hipGetErrorString(_e)); \
  } while (0)

// Dynamic LDS above 64 KB must be opted into (160 KB per CU on gfx950). The
// attribute is per device: remember the opted-in size per (kernel, device).
static void lds_opt_in(const void* fn, int lds_bytes, const char* name) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int> done;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) throw SgError(SG_E_DEVICE, std::string(name) + ": hipGetDevice failed");
  std::lock_guard<std::mutex> lk(mu);
  int& have = done[{fn, dev}];
  if (lds_bytes <= have) return;
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes) != hipSuccess)
    throw SgError(SG_E_DEVICE, std::string(name) + ": dynamic LDS " + std::to_string(lds_bytes) + " B refused");
  have = lds_bytes;
}

void launch_fft_frames(const DevicePlan& D, int64_t g0, int64_t n_groups, int lds_bytes, hipStream_t s) {
  if (n_groups <= 0) return;
  lds_opt_in(reinterpret_cast<const void*>(&sg_fft_frames), lds_bytes, "sg_fft_frames");
  hipLaunchKernelGGL(sg_fft_frames, dim3((unsigned)n_groups), dim3(SG_FFT_THREADS), lds_bytes, s, D.fgroups + g0,
                     D.frames,
                     D.geoms, D.fl, D.fs);
  SG_LAUNCHED("sg_fft_frames");
}
void launch_stft_ola(const DevicePlan& D, int phase, int64_t s0, int64_t n_segs, int lds_bytes, hipStream_t s) {
  if (n_segs <= 0) return;
  auto* k = phase == 0 ? &sg_stft_ola_noise : &sg_stft_ola;
  lds_opt_in(reinterpret_cast<const void*>(k), lds_bytes, phase == 0 ? "sg_stft_ola_noise" : "sg_stft_ola");
  const int W = sg_fft_waves(phase);
  if (n_segs % W) throw SgError(SG_E_DEVICE, "sg_stft_ola: segment count not a multiple of the workgroup's waves");
  hipLaunchKernelGGL(k, dim3((unsigned)(n_segs / W)), dim3(W * 64), lds_bytes, s,
                     D.olasegs + s0,
                     D.olas, D.frames, D.geoms, D.fl, D.fs, D.olatilemax);
  SG_LAUNCHED("sg_stft_ola");
}
void launch_fft_probe(const SgFftGeom* geom, const float* fl, float* data, int M, int nframes, int inverse,
                      hipStream_t s) {
  hipLaunchKernelGGL(sg_fft_probe, dim3((unsigned)nframes), dim3(64), 3 * M * 8 + SG_MAT29_BYTES, s, geom, fl,
                     reinterpret_cast<float2*>(data), inverse);
  SG_LAUNCHED("sg_fft_probe");
}
// phase 0: the noise frames [0, frames64_noise); phase 1: the filter frames after them.
// The root tables are built before the first of the two launches that has frames.
void launch_fft_frames64(const DevicePlan& D, const Batch& B, int ph, hipStream_t s) {
  const int64_t n0 = B.frames64_noise, n = (int64_t)B.frames64.size();
  const int64_t f0 = ph == 0 ? 0 : n0, nf = ph == 0 ? n0 : n - n0;
  if (nf <= 0) return;
  if (ph == 0 || n0 == 0) {
    hipLaunchKernelGGL(sg_roots64, dim3(16, (unsigned)B.roots64_wl.size()), dim3(256), 0, s, D.roots64_wl,
                       D.roots64_off, reinterpret_cast<double2*>(D.roots64));
    SG_LAUNCHED("sg_roots64");
  }
  // the leading wl = 2204 frames of the phase: one per wavefront
  const int64_t nw = B.frames64_w[ph];
  if (nw > 0) {
    const int lds = SG_F64W_WAVES * SG_F64W_M * (int)sizeof(double2);  // a frame per wave
    lds_opt_in(reinterpret_cast<const void*>(&sg_fft_frames64w), lds, "sg_fft_frames64w");
    hipLaunchKernelGGL(sg_fft_frames64w, dim3((unsigned)((nw + SG_F64W_WAVES - 1) / SG_F64W_WAVES)),
                       dim3(SG_F64W_WAVES * 64), lds, s, D.frames64 + f0, nw, D.frames64_tab + f0,
                       reinterpret_cast<const double2*>(D.roots64), D.fl, D.fh, D.fs);
    SG_LAUNCHED("sg_fft_frames64w");
  }
  if (nf - nw <= 0) return;
  const int lds = (B.frames64_maxwl + 32) * (int)sizeof(double2);  // two M-point buffers + radix roots
  lds_opt_in(reinterpret_cast<const void*>(&sg_fft_frames64), lds, "sg_fft_frames64");
  hipLaunchKernelGGL(sg_fft_frames64, dim3((unsigned)(nf - nw)), dim3(SG_F64_THREADS), lds, s, D.frames64 + f0 + nw,
                     D.frames64_tab + f0 + nw, reinterpret_cast<const double2*>(D.roots64), D.fl, D.fh, D.fs);
  SG_LAUNCHED("sg_fft_frames64");
}
void launch_mix_hp(const DevicePlan& D, int64_t t0, int64_t n_tiles, hipStream_t s) {
  if (n_tiles <= 0) return;
  hipLaunchKernelGGL(sg_mix_hp, dim3((unsigned)n_tiles), dim3(256), 0, s, D.mixtiles + t0, D.mixes, D.items, D.olamax,
                     D.cknots, D.fl, D.fs, D.fh);
  SG_LAUNCHED("sg_mix_hp");
}
void launch_ola(const DevicePlan& D, int64_t t0, int64_t n_tiles, hipStream_t s) {
  if (n_tiles <= 0) return;
  hipLaunchKernelGGL(sg_ola, dim3((unsigned)n_tiles), dim3(256), 0, s, D.olatiles + t0, D.olas, D.fs,
                     D.olatilemax + t0);
  SG_LAUNCHED("sg_ola");
}
void launch_ola_max(const DevicePlan& D, int64_t o0, int64_t n_olas, hipStream_t s) {
  if (n_olas <= 0) return;
  hipLaunchKernelGGL(sg_ola_max, dim3((unsigned)n_olas), dim3(64), 0, s, D.olas + o0, (int)n_olas, D.olatilemax,
                     D.olamax + o0);
  SG_LAUNCHED("sg_ola_max");
}
void launch_mix(const DevicePlan& D, int64_t t0, int64_t n_tiles, float* out, hipStream_t s) {
  if (n_tiles <= 0) return;
  hipLaunchKernelGGL(sg_mix, dim3((unsigned)n_tiles), dim3(256), 0, s, D.mixtiles + t0, D.mixes, D.items, D.olamax,
                     D.cknots, D.fl, D.fs, out);
  SG_LAUNCHED("sg_mix");
}
void launch_ugather(const SgUJob* jobs, int64_t n_jobs, const float* us, float* fl, hipStream_t s) {
  for (int64_t j0 = 0; j0 < n_jobs; j0 += 1 << 30) {
    const int64_t n = std::min<int64_t>(n_jobs - j0, 1 << 30);
    hipLaunchKernelGGL(sg_ugather, dim3((unsigned)n), dim3(256), 0, s, jobs + j0, us, fl);
    SG_LAUNCHED("sg_ugather");
  }
}
}  // namespace sg

#ifdef SG_STFT_STAMPS
extern "C" int sg_debug_stft_stamps(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(sg_stft_st), sizeof(unsigned long long) * 32) != hipSuccess) return -1;
  unsigned long long z[32] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(sg_stft_st), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
