// sg_harm.hip — gfx950 kernels of the additive harmonic source
// (generateHarmonics(), R/source.R:377-467).
//
// sg_sine_bank: one wave task = up to SG_TASK_MAX (1024) consecutive samples of one epoch
// inside ONE amplitude interval (the approx() knots x_i, x_{i+1}, R/source.R:403-405),
// so both amplitude columns A[i][.], dA[i][.] = A[i+1][.] - A[i][.] are wave-uniform
// (staged in the wave's LDS slice, read back as broadcasts):
//   integr(u)  closed-form quartic prefix sum of the FMM pitch spline (fp64, Horner)
//   theta      = 2*pi*frac(integr / D)   (1/D folded into the coefficients by the planner)
//   W(j)       = sum_r (A_r + t_j dA_r) sin(r theta)             (R/source.R:396-419)
//              = (b_1 + t_j e_1) sin(theta)  by Clenshaw's recurrence
//                b_r = A_r + 2cos(theta) b_{r+1} - b_{r+2}  (2 VALU ops per row and chain)
//   a task whose two columns are equal runs the A chain only.
// Each task also writes the signed max of its samples that land 1:1 in the
// assembled syllable (R's waveform / max(waveform), R/source.R:449); a small
// kernel reduces those per syllable — no atomics, deterministic.
#include <hip/hip_runtime.h>

#include "sg_dev.h"

#include "sg_amp.h"
#include "sg_devfn.h"

using sgd::contour_at;
using sgd::linear_at;
using sgd::wave_max;

// Amplitude rows of the wave's task are staged in the wave's LDS slice (A
// rows, then dA rows); every Clenshaw step reads 4 rows with one broadcast
// ds_read_b128 (all lanes, same address) into VGPRs, so each row costs exactly
// the two VALU ops of the recurrence. (A DPP row broadcast folded into the
// v_sub measured 4.5 lane-instructions per (sample, row) on gfx950, VGPR/SGPR
// operands 2.7 — tools/ubench/clenshaw_ubench.hip.)
constexpr int SG_LDS_ROWS = 256;

// Interpolated amplitudes (the dA rows): ONE chain over the per-sample amplitude
// a_r(t) = A_r + t dA_r (fma, then the recurrence: 3 VALU ops per row instead of
// 2 x 2 for separate A and dA chains; Reinsch 4 instead of 6), so
// W = (sum_r a_r(t) sin r theta) by linearity (r04: the sine-bank classes -13 %).


// A: the task's column A[i], A1: the next column A[i + 1]; ld gets dA = A1 - A
// (fp32, as the column differences were stored before round 5: bit for bit)
template <bool TWO>
__device__ __forceinline__ void stage_rows(float* __restrict__ la, float* __restrict__ ld, const float* __restrict__ A,
                                           const float* __restrict__ A1, int r0, int n, int lane) {
  for (int r = lane; r < n; r += 64) {
    const float a = A[r0 + r];
    la[r] = a;
    if (TWO) ld[r] = A1[r0 + r] - a;
  }
}

typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float vfma(float a, float b, float c) { return fmaf(a, b, c); }
__device__ __forceinline__ double vfma(double a, double b, double c) { return fma(a, b, c); }
__device__ __forceinline__ f2 vfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// Clenshaw over staged rows n-1 .. 0 (n a multiple of 4), continuing b
#define SG_ROW(a, d)                                                  \
  {                                                                   \
    _Pragma("unroll") for (int s = 0; s < NS; ++s) {                  \
      const Acc av = TWO ? vfma(tt[s], (Acc)(d), (Acc)(a)) : (Acc)(a); \
      const Acc b = vfma(al[s], b1[s], av - b2[s]);                   \
      b2[s] = b1[s];                                                  \
      b1[s] = b;                                                      \
    }                                                                 \
  }
constexpr int SG_ROWS_IT = 8;  // rows per loop iteration (r01: 8 over 4)
template <int NS, bool TWO, typename Acc>
__device__ __forceinline__ void clenshaw_lds(const float* __restrict__ la, const float* __restrict__ ld, int n,
                                             const Acc (&al)[NS], const Acc (&tt)[NS], Acc (&b1)[NS], Acc (&b2)[NS]) {
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (n & 4) {  // odd group of 4 on top
    const float4 A4 = *reinterpret_cast<const float4*>(la + n - 4);
    const float4 D4 = TWO ? *reinterpret_cast<const float4*>(ld + n - 4) : z4;
    SG_ROW(A4.w, D4.w)
    SG_ROW(A4.z, D4.z)
    SG_ROW(A4.y, D4.y)
    SG_ROW(A4.x, D4.x)
    n -= 4;
  }
#pragma unroll 1
  for (int r = n - SG_ROWS_IT; r >= 0; r -= SG_ROWS_IT) {
    const float4 A4 = *reinterpret_cast<const float4*>(la + r + 4);
    const float4 D4 = TWO ? *reinterpret_cast<const float4*>(ld + r + 4) : z4;
    const float4 A0 = *reinterpret_cast<const float4*>(la + r);
    const float4 D0 = TWO ? *reinterpret_cast<const float4*>(ld + r) : z4;
    SG_ROW(A4.w, D4.w)
    SG_ROW(A4.z, D4.z)
    SG_ROW(A4.y, D4.y)
    SG_ROW(A4.x, D4.x)
    SG_ROW(A0.w, D0.w)
    SG_ROW(A0.z, D0.z)
    SG_ROW(A0.y, D0.y)
    SG_ROW(A0.x, D0.x)
  }
}

// Per-sample set-up for task sample l: approx() weight t, 2cos(theta), sin(theta).
// LIN: the phase segment is linear (wave-uniform, chosen per task), one fp64 FMA.
// theta = 2 pi x with x the fractional cycle in [-1/2, 1/2]; v_sin_f32 / v_cos_f32
// take revolutions (measured max abs error 1.24e-7 on gfx950, the fp32 rounding level).
template <bool TWO, bool LIN>
__device__ __forceinline__ void sample_setup(const SgWTask& T, int l, float& t, float& al, float& sn) {
  t = TWO ? fmaf((float)l, T.xby, T.tc0) * T.rdx : 0.f;
  const double m = (double)(T.mbase + l);
  const double P = LIN ? fma(m, T.c1, T.c0) : fma(m, fma(m, fma(m, fma(m, T.c4, T.c3), T.c2), T.c1), T.c0);
  const double v = P;  // cycles of 1/D (planner folds 1/D into the coefficients)
  const float x = (float)(v - rint(v));
  sn = __builtin_amdgcn_sinf(x);
  al = 2.f * __builtin_amdgcn_cosf(x);
}

// fp32 slots in pairs: each row is one v_pk_add_f32 + one v_pk_fma_f32 per two samples
template <int NS, bool TWO>
__device__ __forceinline__ void clenshaw_pk(const float* __restrict__ la, const float* __restrict__ ld, int n,
                                            const float (&al)[NS], const float (&tt)[NS], float (&b1)[NS],
                                            float (&b2)[NS]) {
  constexpr int NP = NS / 2;
  f2 al2[NP], t2[NP], p1[NP], p2[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    al2[i] = f2{al[2 * i], al[2 * i + 1]};
    t2[i] = f2{tt[2 * i], tt[2 * i + 1]};
    p1[i] = f2{b1[2 * i], b1[2 * i + 1]};
    p2[i] = f2{b2[2 * i], b2[2 * i + 1]};
  }
  clenshaw_lds<NP, TWO, f2>(la, ld, n, al2, t2, p1, p2);
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    b1[2 * i] = p1[i].x; b1[2 * i + 1] = p1[i].y;
    b2[2 * i] = p2[i].x; b2[2 * i + 1] = p2[i].y;
  }
}
template <int NS, bool TWO, typename Acc>
__device__ __forceinline__ void clenshaw_any(const float* __restrict__ la, const float* __restrict__ ld, int n,
                                             const Acc (&al)[NS], const Acc (&tt)[NS], Acc (&b1)[NS], Acc (&b2)[NS]) {
  if constexpr (sizeof(Acc) == 4 && NS % 2 == 0)  // fp32 slot pairs as packed fp32 (v_pk_fma_f32 / v_pk_add_f32)
    clenshaw_pk<NS, TWO>(la, ld, n, al, tt, b1, b2);
  else
    clenshaw_lds<NS, TWO, Acc>(la, ld, n, al, tt, b1, b2);
}

// fp64 variant for tall tasks (T.R > SG_ROWS_F32, subharmonic sidebands): the
// fp32 recurrence loses ~R^2 eps near theta = 0 and fp32 cos(theta) misplaces
// the angle by ~eps/theta, which row R multiplies by R.
template <bool TWO, bool LIN>
__device__ __forceinline__ void sample_setup(const SgWTask& T, int l, float& t, double& al, double& sn) {
  t = TWO ? fmaf((float)l, T.xby, T.tc0) * T.rdx : 0.f;
  const double m = (double)(T.mbase + l);
  const double P = LIN ? fma(m, T.c1, T.c0) : fma(m, fma(m, fma(m, fma(m, T.c4, T.c3), T.c2), T.c1), T.c0);
  double cs;
  sincospi(2.0 * (P - rint(P)), &sn, &cs);
  al = 2.0 * cs;
}

template <int NS, bool TWO, bool ENV, bool LIN, typename Acc, typename WT = float>
__device__ __forceinline__ void run_slots(const SgWTask& T, bool staged, float* __restrict__ la, float* __restrict__ ld,
                                          const float* __restrict__ amps, const SgSyllable* __restrict__ syls,
                                          const double* __restrict__ cknots, WT* __restrict__ W, int l0, int lane,
                                          float& tmax, const float (&rc)[8], const float (&rs)[8]) {
  // linear-phase slots 1..7 by rotation of slot 0 (no per-slot fp64 / v_sin / v_cos)
  constexpr bool ROT = LIN && sizeof(Acc) == 4 && NS > 1;
  float t[NS];
  Acc al[NS], sn[NS], b1[NS], b2[NS];
  int l[NS];
  bool valid[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    l[s] = l0 + 64 * s + lane;
    valid[s] = l[s] < T.len;
    b1[s] = b2[s] = (Acc)0;
    if (ROT && s > 0) {  // slot s = slot 0 rotated by 64 s samples of a linear phase
      t[s] = TWO ? fmaf((float)l[s], T.xby, T.tc0) * T.rdx : 0.f;
      const float h = 0.5f * (float)al[0], s2 = 2.f * (float)sn[0];
      al[s] = fmaf((float)al[0], rc[s], -s2 * rs[s]);
      sn[s] = fmaf((float)sn[0], rc[s], h * rs[s]);
    } else {
      sample_setup<TWO, LIN>(T, valid[s] ? l[s] : 0, t[s], al[s], sn[s]);
    }
  }
  Acc tt[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) tt[s] = (Acc)t[s];
  if (staged) {
    clenshaw_any<NS, TWO, Acc>(la, ld, T.Rn, al, tt, b1, b2);
  } else {  // rare (subharmonic epochs with many rows): 256-row chunks, top first
    for (int r0 = (T.Rn - 1) / SG_LDS_ROWS * SG_LDS_ROWS; r0 >= 0; r0 -= SG_LDS_ROWS) {
      const int n = T.Rn - r0 < SG_LDS_ROWS ? T.Rn - r0 : SG_LDS_ROWS;
      stage_rows<TWO>(la, ld, amps + T.a_off, amps + T.d_off, r0, n, lane);
      clenshaw_any<NS, TWO, Acc>(la, ld, n, al, tt, b1, b2);
    }
  }
  // a pass whose samples all exist and all land 1:1 in the syllable (most of a long
  // task's passes): no per-lane range tests in the epilogue
  const int jp0 = T.j0 + l0;
  if (!ENV && l0 + 64 * NS <= T.len && jp0 >= T.dj0 && jp0 + 64 * NS <= T.dj1) {
    WT* __restrict__ wp = W + T.w_off + jp0 + lane;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const Acc yv = b1[s] * sn[s];
      wp[64 * s] = (WT)yv;
      tmax = fmaxf(tmax, (float)yv);
    }
    return;
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const Acc yv = b1[s] * sn[s];
    const float y = (float)yv;
    const int j = T.j0 + l[s];
    if (valid[s]) W[T.w_off + j] = (WT)yv;
    // fused max over the samples that land 1:1 in the syllable (branch-free)
    const bool in = valid[s] && j >= T.dj0 && j < T.dj1;
    if (!ENV) {
      tmax = in ? fmaxf(tmax, y) : tmax;
    } else if (in) {  // amplAnchors envelope (rare): R's max is taken after it
      const SgSyllable& sy = syls[T.syl];
      tmax = fmaxf(tmax, (float)((double)y * contour_at(sy.env, cknots, sy.L, T.dk0 + j)));
    }
  }
}

template <bool TWO, bool ENV, bool LIN, typename Acc = float, typename WT = float>
__device__ __forceinline__ float run_task(const SgWTask& T, float* __restrict__ la, float* __restrict__ ld,
                                          const float* __restrict__ amps, const SgSyllable* __restrict__ syls,
                                          const double* __restrict__ cknots, WT* __restrict__ W, int lane) {
  const bool staged = T.Rn <= SG_LDS_ROWS;  // rows stay in LDS for every pass of the task
  if (staged) stage_rows<TWO>(la, ld, amps + T.a_off, amps + T.d_off, 0, T.Rn, lane);
  float tmax = 0.f;
  int l0 = 0;
  // passes of 8 / 4 / 2 / 1 slots of 64 samples (8-slot passes on the A chain
  // only: with the dA chain they exceed the VGPR budget)
  constexpr bool F32 = sizeof(Acc) == 4;
  // cos / sin of the linear phase advance over 64 k samples, k = 0..7 (wave-uniform)
  float rc[8], rs[8];
  if (LIN && F32) {
    const double x = (double)(64 * (lane & 7)) * T.c1;
    const float f = (float)(x - rint(x));
    const int c = __builtin_bit_cast(int, __builtin_amdgcn_cosf(f)), sv = __builtin_bit_cast(int, __builtin_amdgcn_sinf(f));
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      rc[k] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(c, k));
      rs[k] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(sv, k));
    }
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) rc[k] = rs[k] = 0.f;
  }
  if constexpr (!F32) {  // fp64 passes of at most 2 slots (fewer VGPRs, higher occupancy; r02)
#pragma unroll 1
    for (; T.len - l0 > 64; l0 += 128)
      run_slots<2, TWO, ENV, LIN, Acc, WT>(T, staged, la, ld, amps, syls, cknots, W, l0, lane, tmax, rc, rs);
    if (l0 < T.len)
      run_slots<1, TWO, ENV, LIN, Acc, WT>(T, staged, la, ld, amps, syls, cknots, W, l0, lane, tmax, rc, rs);
    return tmax;
  }
  if (F32 && !TWO) {
#pragma unroll 1
    for (; T.len - l0 > 448; l0 += 512)
      run_slots<8, TWO, ENV, LIN, Acc, WT>(T, staged, la, ld, amps, syls, cknots, W, l0, lane, tmax, rc, rs);
  }
#pragma unroll 1
  for (; T.len - l0 > 192; l0 += 256)
    run_slots<4, TWO, ENV, LIN, Acc, WT>(T, staged, la, ld, amps, syls, cknots, W, l0, lane, tmax, rc, rs);
  if (T.len - l0 > 64) {
    run_slots<2, TWO, ENV, LIN, Acc, WT>(T, staged, la, ld, amps, syls, cknots, W, l0, lane, tmax, rc, rs);
    l0 += 128;
  }
  if (l0 < T.len)
    run_slots<1, TWO, ENV, LIN, Acc, WT>(T, staged, la, ld, amps, syls, cknots, W, l0, lane, tmax, rc, rs);
  return tmax;
}

// One task on its own wave pass (any length, envelope, linear or general phase)
__device__ __forceinline__ float run_one(const SgWTask& T, float* __restrict__ la, float* __restrict__ ld,
                                         const float* __restrict__ amps, const SgSyllable* __restrict__ syls,
                                         const double* __restrict__ cknots, float* __restrict__ W, int lane) {
  if (T.flags & SG_TASK_ENV)  // amplAnchors envelope: rare, kept out of the hot variants
    return (T.flags & SG_TASK_CONST) ? run_task<false, true, false>(T, la, ld, amps, syls, cknots, W, lane)
                                     : run_task<true, true, false>(T, la, ld, amps, syls, cknots, W, lane);
  if (T.flags & SG_TASK_LIN)  // constant pitch over the phase segment
    return (T.flags & SG_TASK_CONST) ? run_task<false, false, true>(T, la, ld, amps, syls, cknots, W, lane)
                                     : run_task<true, false, true>(T, la, ld, amps, syls, cknots, W, lane);
  return (T.flags & SG_TASK_CONST) ? run_task<false, false, false>(T, la, ld, amps, syls, cknots, W, lane)
                                   : run_task<true, false, false>(T, la, ld, amps, syls, cknots, W, lane);
}

// Two tasks of <= 64 samples (most of C5's: one glottal cycle each) in one
// wave: lane l runs sample l of task P in the low and of task Q in the high half
// of packed fp32 pairs, so each row costs the 2 packed ops per chain of ONE
// task. Their rows interleave in LDS (la[2r] = A_P[r], la[2r + 1] = A_Q[r],
// zero above a task's R; the dA rows likewise, zero for a CONST task), and one
// broadcast ds_read_b128 yields rows r, r + 1 of both.
// The last amplitude column a run step loaded (rows lane, lane + 64 of its epoch block;
// SG_ROWS_F32 <= 128): consecutive glottal cycles share a column (task t's A[i + 1] is
// task t + 1's A[i]), so a run reads each column once. Off by default (SG_RUN_CACHE=1
// enables it): the second read hits L2 and the cache's selects cost more (r06h: pairs
// 1.888 ms without, 1.965 ms with; a variant that also loaded step s + 1's columns and
// descriptors during step s's rows took 2.466 ms).
struct ColCache {
  int64_t off = -1;
  float v[2] = {0.f, 0.f};
};
static_assert(SG_ROWS_F32 <= 128, "ColCache holds two rows per lane");
#ifndef SG_RUN_CACHE
#define SG_RUN_CACHE 0
#endif

// Rows [r0, r0 + n) of a pair's columns into LDS, interleaved (la[2r] = A_P[r],
// la[2r + 1] = A_Q[r]; ld the column differences, zero for a CONST task). Each lane
// reads row min(r, Rn - 1) of all four columns unconditionally (the rows the masked
// form read, no more bytes), against wave-uniform column bases (SGPR base + 32-bit
// lane offset), and one wait covers the four reads; rows at or past a task's Rn are
// zero as before (selects). The masked, per-column form waited after each read.
template <bool TWO>
__device__ __forceinline__ void stage_pair(const SgWTask& P, const SgWTask& Q, const float* __restrict__ amps,
                                           float* __restrict__ la, float* __restrict__ ld, int r0, int n, int lane) {
  const bool pc = P.flags & SG_TASK_CONST, qc = Q.flags & SG_TASK_CONST;
  const float* __restrict__ pa = amps + P.a_off;
  const float* __restrict__ qa = amps + Q.a_off;
  const float* __restrict__ pd = amps + (pc ? P.a_off : P.d_off);
  const float* __restrict__ qd = amps + (qc ? Q.a_off : Q.d_off);
  const int lp = P.Rn > 0 ? P.Rn - 1 : 0, lq = Q.Rn > 0 ? Q.Rn - 1 : 0;  // last row read: no bytes past Rn
  // n <= 128: the pairs' R <= SG_ROWS_F32, the tall pairs' chunks SG_LDS_ROWS / 2
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (h == 1 && n <= 64) break;  // wave-uniform
    const int r = lane + 64 * h;
    if (r >= n) break;
    const int rr = r0 + r;
    // byte offsets as 32-bit values: the SGPR-base + VGPR-offset load form
    const unsigned bp = 4u * (unsigned)(rr < P.Rn ? rr : lp), bq = 4u * (unsigned)(rr < Q.Rn ? rr : lq);
    auto at = [](const float* __restrict__ c, unsigned b) {
      return *reinterpret_cast<const float*>(reinterpret_cast<const char*>(c) + b);
    };
    const float ap0 = at(pa, bp), aq0 = at(qa, bq);
    const float dp0 = TWO ? at(pd, bp) : 0.f, dq0 = TWO ? at(qd, bq) : 0.f;
    const bool inp = rr < P.Rn, inq = rr < Q.Rn;
    const float ap = inp ? ap0 : 0.f, aq = inq ? aq0 : 0.f;
    *reinterpret_cast<float2*>(la + 2 * r) = make_float2(ap, aq);
    if (TWO)
      *reinterpret_cast<float2*>(ld + 2 * r) = make_float2(inp && !pc ? dp0 - ap : 0.f, inq && !qc ? dq0 - aq : 0.f);
  }
}

static_assert(SG_ROWS_F32 <= 128 && SG_LDS_ROWS / 2 <= 128, "stage_pair stages at most 128 rows per call");

// A pair's samples to W (wave-uniform destination bases) and their masked maxima
__device__ __forceinline__ void pair_store(const SgWTask& P, const SgWTask& Q, float yp, float yq,
                                           float* __restrict__ W, int lane, float& mp, float& mq) {
  const bool vp = lane < P.len, vq = lane < Q.len;
  float* __restrict__ wp = W + (P.w_off + P.j0);
  float* __restrict__ wq = W + (Q.w_off + Q.j0);
  if (vp) wp[(unsigned)lane] = yp;
  if (vq) wq[(unsigned)lane] = yq;
  const int jp = P.j0 + lane, jq = Q.j0 + lane;
  mp = vp && jp >= P.dj0 && jp < P.dj1 ? yp : 0.f;
  mq = vq && jq >= Q.dj0 && jq < Q.dj1 ? yq : 0.f;
}

template <bool TWO>
__device__ __forceinline__ void run_pair(const SgWTask& P, const SgWTask& Q, float* __restrict__ la,
                                         float* __restrict__ ld, const float* __restrict__ amps,
                                         float* __restrict__ W, int lane, float& mp, float& mq,
                                         ColCache* cc = nullptr) {
#ifdef SG_DIAG_PAIR_NOROWS  // diagnostic build only: the pair's set-up, staging and stores without the rows
  const int R = 0;
#else
  const int R = P.Rn > Q.Rn ? P.Rn : Q.Rn;  // multiples of 16
#endif
  if (SG_RUN_CACHE && cc) {
    // Rows of a column past its task's Rn are zero (Rn covers both of the task's columns), so
    // a column read up to its epoch's R (the block's rows) is the same for every task that
    // shares it: reuse by offset is exact. The old form's masks (r < Rn) select the same values.
    const bool pc = P.flags & SG_TASK_CONST, qc = Q.flags & SG_TASK_CONST;
    ColCache nc;
    const int hn = (P.R > 64 || Q.R > 64) ? 2 : 1;  // whole columns (R <= SG_ROWS_F32 < 128), so the cache is
#pragma unroll
    for (int h = 0; h < 2; ++h) {                   // valid for any later R
      if (h >= hn) break;
      const int r = lane + 64 * h;
      auto load = [&](int64_t off, int rows) { return r < rows ? amps[off + r] : 0.f; };
      const float pa = P.a_off == cc->off ? cc->v[h] : load(P.a_off, P.R);
      const float pd = TWO && !pc ? (P.d_off == cc->off ? cc->v[h] : load(P.d_off, P.R)) : pa;
      const float qa = Q.a_off == P.a_off ? pa
                       : Q.a_off == P.d_off && TWO && !pc ? pd
                       : Q.a_off == cc->off ? cc->v[h] : load(Q.a_off, Q.R);
      const float qd = TWO && !qc ? (Q.d_off == P.d_off && !pc ? pd : load(Q.d_off, Q.R)) : qa;
      if (r < R) {
        *reinterpret_cast<float2*>(la + 2 * r) = make_float2(pa, qa);
        if (TWO) *reinterpret_cast<float2*>(ld + 2 * r) = make_float2(pc ? 0.f : pd - pa, qc ? 0.f : qd - qa);
      }
      nc.v[h] = TWO && !qc ? qd : qa;
    }
    nc.off = TWO && !qc ? Q.d_off : Q.a_off;
    *cc = nc;
  } else {
    stage_pair<TWO>(P, Q, amps, la, ld, 0, R, lane);
  }
  const bool vp = lane < P.len, vq = lane < Q.len;
  float tp, alp, snp, tq, alq, snq;
  sample_setup<TWO, false>(P, vp ? lane : 0, tp, alp, snp);
  sample_setup<TWO, false>(Q, vq ? lane : 0, tq, alq, snq);
  const f2 al{alp, alq}, tpq{tp, tq};
  f2 b1{0.f, 0.f}, b2{0.f, 0.f};
#define SG_PROW(a, d)                                   \
  {                                                     \
    const f2 av = TWO ? vfma(tpq, (d), (a)) : (a);      \
    const f2 b = vfma(al, b1, av - b2);                 \
    b2 = b1;                                            \
    b1 = b;                                             \
  }
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 1
  for (int r = R - 4; r >= 0; r -= 4) {  // rows r + 3 .. r
    const float4 A1 = *reinterpret_cast<const float4*>(la + 2 * r + 4);
    const float4 A0 = *reinterpret_cast<const float4*>(la + 2 * r);
    const float4 D1 = TWO ? *reinterpret_cast<const float4*>(ld + 2 * r + 4) : z4;
    const float4 D0 = TWO ? *reinterpret_cast<const float4*>(ld + 2 * r) : z4;
    SG_PROW((f2{A1.z, A1.w}), (f2{D1.z, D1.w}))
    SG_PROW((f2{A1.x, A1.y}), (f2{D1.x, D1.y}))
    SG_PROW((f2{A0.z, A0.w}), (f2{D0.z, D0.w}))
    SG_PROW((f2{A0.x, A0.y}), (f2{D0.x, D0.y}))
  }
#undef SG_PROW
  pair_store(P, Q, b1.x * snp, b1.y * snq, W, lane, mp, mq);
}

// Tasks of the fp32 class (listed in idx), one per wave. (A grid of resident waves
// walking the list measured slower: r04f, C2 +14 %, C5 +22 %.)
// Registers capped for 8 waves per SIMD (70 -> 63 VGPRs, no spill; r04occ C5 1.964 -> 1.798 ms per launch).
extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void sg_sine_bank(
    const int32_t* __restrict__ idx, int64_t n, const SgWTask* __restrict__ tasks, const float* __restrict__ amps,
    const SgSyllable* __restrict__ syls, const double* __restrict__ cknots, float* __restrict__ W,
    float* __restrict__ taskmax) {
  __shared__ __attribute__((aligned(16))) float rows[4][2][SG_LDS_ROWS];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t k = (int64_t)sgd::xcd_swizzle(blockIdx.x, gridDim.x) * 4 + wave;
  if (k >= n) return;
  const int64_t ti = idx[k];
  const SgWTask T = tasks[ti];
  const float wm = wave_max(run_one(T, rows[wave][0], rows[wave][1], amps, syls, cknots, W, lane));
  if (lane == 0) taskmax[ti] = wm;
}

// A run of short tasks (consecutive entries of one syllable in the class list idx:
// idx[rs[r] .. rs[r + 1]), <= SG_RUN_TASKS) on one wave, two tasks per step in the
// halves of packed pairs (PAIR: run_pair or run_pair_rs; a task's arithmetic does not
// depend on its partner, the last odd one pairs with itself). The syllable max needs
// only the max over its tasks (sg_syl_max), so the run's max goes to its first task's
// slot and -inf to the others: one wave reduction per run instead of two per step
// (round 6; the per-step set-up, staging and stores stay per step).
// IDXPF: the next step's two task indices are loaded with this step's descriptors, so a
// step waits for one scalar round trip instead of two (r06l, same box: sg_sine_bank_pairs
// 1.670 -> 1.631 ms; sg_sine_bank_tall_pairs 1.686 -> 1.719 ms, so off there)
template <bool IDXPF, class PAIR>
__device__ __forceinline__ void run_of_pairs(const int32_t* __restrict__ idx, const int32_t* __restrict__ rs,
                                             int64_t nruns, const SgWTask* __restrict__ tasks,
                                             float* __restrict__ taskmax, PAIR&& pair) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t r = (int64_t)sgd::xcd_swizzle(blockIdx.x, gridDim.x) * 4 + wave;
  if (r >= nruns) return;
  const int32_t k0 = rs[r], k1 = rs[r + 1];
  float m = -INFINITY;
  int32_t ip = idx[k0], iq = idx[k0 + 1 < k1 ? k0 + 1 : k0];
  for (int32_t k = k0; k < k1; k += 2) {
    if (!IDXPF) {
      ip = idx[k];
      iq = idx[k + 1 < k1 ? k + 1 : k];
    }
    const SgWTask P = tasks[ip];
    const SgWTask Q = tasks[iq];
    if (IDXPF && k + 2 < k1) {
      ip = idx[k + 2];
      iq = idx[k + 3 < k1 ? k + 3 : k + 2];
    }
    float mp, mq;
    pair(P, Q, wave, lane, mp, mq);
    m = fmaxf(m, fmaxf(mp, mq));
    __asm__ __volatile__("" ::: "memory");  // the next step's staging follows this step's row reads
  }
  m = wave_max(m);
  for (int32_t k = k0 + lane; k < k1; k += 64) taskmax[idx[k]] = k == k0 ? m : -INFINITY;
}

// Short fp32 tasks (<= 64 samples, no envelope), runs of them (run_of_pairs).
extern "C" __global__ __launch_bounds__(256) void sg_sine_bank_pairs(
    const int32_t* __restrict__ idx, const int32_t* __restrict__ rs, int64_t nruns,
    const SgWTask* __restrict__ tasks, const float* __restrict__ amps, float* __restrict__ W,
    float* __restrict__ taskmax) {
  __shared__ __attribute__((aligned(16))) float rows[4][2][SG_LDS_ROWS];
  ColCache cc;
  run_of_pairs<true>(idx, rs, nruns, tasks, taskmax,
               [&](const SgWTask& P, const SgWTask& Q, int wave, int lane, float& mp, float& mq) {
                 if ((P.flags & Q.flags) & SG_TASK_CONST) run_pair<false>(P, Q, rows[wave][0], rows[wave][1], amps, W, lane, mp, mq, &cc);
                 else run_pair<true>(P, Q, rows[wave][0], rows[wave][1], amps, W, lane, mp, mq, &cc);
               });
}

// ---------------------------------------------- tall tasks, fp32 Reinsch
// Plain Clenshaw in fp32 loses ~R^2 eps when cos(theta) is near +-1 (a sideband
// grid's angle is small: theta = 2 pi subFreq / fs): 2 cos(theta) is then known
// only to eps absolutely, which misplaces the angle by eps / theta. Reinsch's
// modification carries d_k = b_k - sg b_{k+1} (sg = sign cos theta) and enters the
// angle through u = 2 cos(theta) - 2 sg = -4 sin^2(theta/2) (sg = 1) or
// 4 cos^2(theta/2) (sg = -1), both known to a few eps RELATIVE:
//   d_k = a_k + u b_{k+1} + sg d_{k+1},   b_k = d_k + sg b_{k+1},   S = b_1 sin(theta)
// (3 FMAs per row and chain; samples in packed pairs). sin/cos of the half angle
// come from fp32 Taylor polynomials on [-pi/2, pi/2] (relative error < 1e-9 before
// rounding), not from v_sin / v_cos, whose error is absolute.

__device__ __forceinline__ void rs_setup(const SgWTask& T, int l, bool two, float& t, float& u, float& sg, float& sn) {
  t = two ? fmaf((float)l, T.xby, T.tc0) * T.rdx : 0.f;
  const double m = (double)(T.mbase + l);
  const double P = fma(m, fma(m, fma(m, fma(m, T.c4, T.c3), T.c2), T.c1), T.c0);
  const float x = (float)(P - rint(P));  // revolutions, |x| <= 1/2
  const float h = 3.14159265358979f * x;  // theta / 2
  const float h2 = h * h;
  float s = fmaf(h2, 1.6059043836821614e-10f, -2.5052108385441720e-08f);
  s = fmaf(h2, s, 2.7557319223985893e-06f);
  s = fmaf(h2, s, -1.9841269841269841e-04f);
  s = fmaf(h2, s, 8.3333333333333333e-03f);
  s = fmaf(h2, s, -1.6666666666666667e-01f);
  s = fmaf(h2 * s, h, h);  // sin(theta / 2)
  float c = fmaf(h2, -1.1470745597729725e-11f, 2.0876756987868099e-09f);
  c = fmaf(h2, c, -2.7557319223985891e-07f);
  c = fmaf(h2, c, 2.4801587301587302e-05f);
  c = fmaf(h2, c, -1.3888888888888889e-03f);
  c = fmaf(h2, c, 4.1666666666666667e-02f);
  c = fmaf(h2, c, -0.5f);
  c = fmaf(h2, c, 1.f);  // cos(theta / 2)
  sn = 2.f * s * c;
  const bool pos = fabsf(x) <= 0.25f;  // cos(theta) >= 0
  sg = pos ? 1.f : -1.f;
  u = pos ? -4.f * s * s : 4.f * c * c;
}

// Two tall tasks of <= 64 samples in one wave (as run_pair: task P in the low,
// Q in the high half of packed pairs), Reinsch chains, rows staged interleaved
// in 128-row chunks from the top.
template <bool TWO>
__device__ __forceinline__ void run_pair_rs(const SgWTask& P, const SgWTask& Q, float* __restrict__ la,
                                            float* __restrict__ ld, const float* __restrict__ amps,
                                            float* __restrict__ W, int lane, float& mp, float& mq) {
  const int R = P.Rn > Q.Rn ? P.Rn : Q.Rn;
  const bool vp = lane < P.len, vq = lane < Q.len;
  float tp, up, sgp, snp, tq, uq, sgq, snq;
  rs_setup(P, vp ? lane : 0, TWO, tp, up, sgp, snp);
  rs_setup(Q, vq ? lane : 0, TWO, tq, uq, sgq, snq);
  const f2 u{up, uq}, sg{sgp, sgq}, tpq{tp, tq};
  f2 b{0.f, 0.f}, d{0.f, 0.f};
#define SG_RPROW(a, dd)                                  \
  {                                                      \
    const f2 av = TWO ? vfma(tpq, (dd), (a)) : (a);      \
    f2 q = vfma(sg, d, av);                              \
    q = vfma(u, b, q);                                   \
    b = vfma(sg, b, q);                                  \
    d = q;                                               \
  }
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  constexpr int CH = SG_LDS_ROWS / 2;  // rows per interleaved chunk
#pragma unroll 1
  for (int r0 = (R - 1) / CH * CH; r0 >= 0; r0 -= CH) {
    const int n = R - r0 < CH ? R - r0 : CH;  // multiple of 16
    stage_pair<TWO>(P, Q, amps, la, ld, r0, n, lane);
#pragma unroll 1
    for (int r = n - 4; r >= 0; r -= 4) {
      const float4 A1 = *reinterpret_cast<const float4*>(la + 2 * r + 4);
      const float4 A0 = *reinterpret_cast<const float4*>(la + 2 * r);
      const float4 D1 = TWO ? *reinterpret_cast<const float4*>(ld + 2 * r + 4) : z4;
      const float4 D0 = TWO ? *reinterpret_cast<const float4*>(ld + 2 * r) : z4;
      SG_RPROW((f2{A1.z, A1.w}), (f2{D1.z, D1.w}))
      SG_RPROW((f2{A1.x, A1.y}), (f2{D1.x, D1.y}))
      SG_RPROW((f2{A0.z, A0.w}), (f2{D0.z, D0.w}))
      SG_RPROW((f2{A0.x, A0.y}), (f2{D0.x, D0.y}))
    }
  }
#undef SG_RPROW
  pair_store(P, Q, b.x * snp, b.y * snq, W, lane, mp, mq);
}

__device__ __forceinline__ float run_one_tall(const SgWTask& T, float* __restrict__ la, float* __restrict__ ld,
                                              const float* __restrict__ amps, const SgSyllable* __restrict__ syls,
                                              const double* __restrict__ cknots, float* __restrict__ W, int lane) {
  if (T.flags & SG_TASK_ENV)
    return (T.flags & SG_TASK_CONST) ? run_task<false, true, false, double>(T, la, ld, amps, syls, cknots, W, lane)
                                     : run_task<true, true, false, double>(T, la, ld, amps, syls, cknots, W, lane);
  return (T.flags & SG_TASK_CONST) ? run_task<false, false, false, double>(T, la, ld, amps, syls, cknots, W, lane)
                                   : run_task<true, false, false, double>(T, la, ld, amps, syls, cknots, W, lane);
}

// The tasks with more than SG_ROWS_F32 rows (listed in idx), one task per wave:
// fp64 sincospi and fp64 Clenshaw chains (fp32 Reinsch chains measured equal time
// on C5: the kernel is latency-bound). The short ones (<= 64 samples, no envelope)
// are listed separately for sg_sine_bank_tall_pairs.
extern "C" __global__ __launch_bounds__(256) void sg_sine_bank_tall(
    const int32_t* __restrict__ idx, int64_t n, const SgWTask* __restrict__ tasks, const float* __restrict__ amps,
    const SgSyllable* __restrict__ syls, const double* __restrict__ cknots, float* __restrict__ W,
    float* __restrict__ taskmax) {
  __shared__ __attribute__((aligned(16))) float rows[4][2][SG_LDS_ROWS];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t k = (int64_t)sgd::xcd_swizzle(blockIdx.x, gridDim.x) * 4 + wave;
  if (k >= n) return;
  const int64_t ti = idx[k];
  const SgWTask T = tasks[ti];
  const float wm = wave_max(run_one_tall(T, rows[wave][0], rows[wave][1], amps, syls, cknots, W, lane));
  if (lane == 0) taskmax[ti] = wm;
}

// Short tall tasks, runs of them, fp32 Reinsch (run_pair_rs).
extern "C" __global__ __launch_bounds__(256) void sg_sine_bank_tall_pairs(
    const int32_t* __restrict__ idx, const int32_t* __restrict__ rs, int64_t nruns,
    const SgWTask* __restrict__ tasks, const float* __restrict__ amps, float* __restrict__ W,
    float* __restrict__ taskmax) {
  __shared__ __attribute__((aligned(16))) float rows[4][2][SG_LDS_ROWS];
  run_of_pairs<false>(idx, rs, nruns, tasks, taskmax,
               [&](const SgWTask& P, const SgWTask& Q, int wave, int lane, float& mp, float& mq) {
                 if ((P.flags & Q.flags) & SG_TASK_CONST) run_pair_rs<false>(P, Q, rows[wave][0], rows[wave][1], amps, W, lane, mp, mq);
                 else run_pair_rs<true>(P, Q, rows[wave][0], rows[wave][1], amps, W, lane, mp, mq);
               });
}

// ------------------------------------------- fp64 path (SG_TASK_HP tasks)
// Tasks of an ill-conditioned formant-filter bout (planner: filter_conditioning):
// fp64 angle (sincospi) and fp64 Clenshaw chains, the epoch waveform kept in
// fp64 (W64). Amplitudes stay fp32: their rounding scales each harmonic by
// (1 + 6e-8), an error at the harmonic's own frequency, which the envelope
// weighs like the harmonic itself (only white round-off is amplified).
__device__ __forceinline__ float run_one_hp(const SgWTask& T, float* __restrict__ la, float* __restrict__ ld,
                                            const float* __restrict__ amps, const SgSyllable* __restrict__ syls,
                                            const double* __restrict__ cknots, double* __restrict__ W, int lane) {
  const bool c = T.flags & SG_TASK_CONST;
  if (T.flags & SG_TASK_ENV)
    return c ? run_task<false, true, false, double, double>(T, la, ld, amps, syls, cknots, W, lane)
             : run_task<true, true, false, double, double>(T, la, ld, amps, syls, cknots, W, lane);
  if (T.flags & SG_TASK_LIN)
    return c ? run_task<false, false, true, double, double>(T, la, ld, amps, syls, cknots, W, lane)
             : run_task<true, false, true, double, double>(T, la, ld, amps, syls, cknots, W, lane);
  return c ? run_task<false, false, false, double, double>(T, la, ld, amps, syls, cknots, W, lane)
           : run_task<true, false, false, double, double>(T, la, ld, amps, syls, cknots, W, lane);
}

extern "C" __global__ __launch_bounds__(256) void sg_sine_bank_hp(
    const int32_t* __restrict__ idx, int64_t n, const SgWTask* __restrict__ tasks, const float* __restrict__ amps,
    const SgSyllable* __restrict__ syls, const double* __restrict__ cknots, double* __restrict__ W64,
    float* __restrict__ taskmax) {
  __shared__ __attribute__((aligned(16))) float rows[4][2][SG_LDS_ROWS];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t k = (int64_t)sgd::xcd_swizzle(blockIdx.x, gridDim.x) * 4 + wave;
  if (k >= n) return;
  const int64_t ti = idx[k];
  const SgWTask T = tasks[ti];
  const float wm = wave_max(run_one_hp(T, rows[wave][0], rows[wave][1], amps, syls, cknots, W64, lane));
  if (lane == 0) taskmax[ti] = wm;
}

// fade(k) of R's fade() on a syllable of L samples, lf-sample ramps (R/source.R:436-467)
template <typename V = float>
__device__ __forceinline__ V fade_at(int lf, int64_t L, int64_t k) {
  V f = 1;
  const V by = (V)1 / (V)(lf - 1);
  if (k < lf) f *= (k == lf - 1) ? (V)1 : (V)k * by;
  const int64_t kb = L - 1 - k;
  if (kb < lf) f *= (kb == lf - 1) ? (V)1 : (V)kb * by;
  return f;
}

// ------------------------------------------- wavetable path (SgTabJob, sg_dev.h)
// One workgroup per job. Table: S and h dS/dx (h = 1 / N) at the N points as the
// real and imaginary parts of ONE inverse complex DFT, x_k = sum_m Z_m e^{2 pi i m k / N}
// with Z = U + i V for the two Hermitian spectra U_{+-r} = -+i A_r / 2 (real part:
// sum_r A_r sin(2 pi r k / N) = S_k) and V_{+-r} = r A_r pi / N (imaginary part:
// (2 pi / N) sum_r r A_r cos(2 pi r k / N) = h S'(x_k)); fp32 radix-4 Stockham in LDS
// (~N / 4 log4 N butterflies instead of the 2 N Rn fp64 Clenshaw steps, rounding
// ~log2 N eps of sum |A_r|), twiddles from sincospif. Then each interval's cubic
// Hermite coefficients. LDS (bytes from 0): the float4 table [16 N), aliased by the
// FFT's two float2 buffers during the transform, and the twiddles [16 N, 18 N).
constexpr int SG_TAB_THREADS = 512;  // threads per sg_sine_bank_tab workgroup
__device__ __forceinline__ void tab_build(float4* __restrict__ lt, const float* __restrict__ la, int Rn, int logn) {
  const int N = 1 << logn;
  float2* X = reinterpret_cast<float2*>(lt);
  float2* Y = X + N;
  float2* tw = X + 2 * N;
  const float pin = 3.14159265358979f / (float)N;
  for (int t = threadIdx.x; t < N / 4; t += SG_TAB_THREADS) {  // the radix-4 stages' w^1
    float sv, cv;
    sincospif(2.f * (float)t / (float)N, &sv, &cv);
    tw[t] = make_float2(cv, sv);
  }
  for (int m = threadIdx.x; m < N; m += SG_TAB_THREADS) {
    float z = 0.f;
    if (m >= 1 && m <= Rn) z = la[m - 1] * ((float)m * pin - 0.5f);
    else if (m >= N - Rn) z = la[N - m - 1] * ((float)(N - m) * pin + 0.5f);
    X[m] = make_float2(0.f, z);
  }
  __syncthreads();
  // Stockham autosort: a radix-2 stage first when log2 N is odd, then radix-4
  // stages; stage with sub-transform size Ns: v_r = X[j + r N / R] w^r,
  // w = e^{2 pi i k / (R Ns)}, k = j mod Ns, into Y[(j - k) R + k + r Ns]
  int Ns = 1;
  if (logn & 1) {
    for (int j = threadIdx.x; j < N / 2; j += SG_TAB_THREADS) {
      const float2 a = X[j], b = X[j + N / 2];
      Y[2 * j] = make_float2(a.x + b.x, a.y + b.y);
      Y[2 * j + 1] = make_float2(a.x - b.x, a.y - b.y);
    }
    __syncthreads();
    float2* t = X;
    X = Y;
    Y = t;
    Ns = 2;
  }
  auto cmul = [](float2 a, float2 b) { return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); };
  for (; Ns < N; Ns <<= 2) {
    const int sh = logn - 2 - __builtin_ctz(Ns);  // w = tw[k N / (4 Ns)]
    for (int j = threadIdx.x; j < N / 4; j += SG_TAB_THREADS) {
      const int k = j & (Ns - 1);
      const float2 w1 = tw[k << sh], w2 = cmul(w1, w1), w3 = cmul(w2, w1);
      const float2 v0 = X[j], v1 = cmul(X[j + N / 4], w1), v2 = cmul(X[j + N / 2], w2),
                   v3 = cmul(X[j + 3 * N / 4], w3);
      const float2 s02 = make_float2(v0.x + v2.x, v0.y + v2.y), d02 = make_float2(v0.x - v2.x, v0.y - v2.y);
      const float2 s13 = make_float2(v1.x + v3.x, v1.y + v3.y), d13 = make_float2(v1.x - v3.x, v1.y - v3.y);
      const int o = (j - k) * 4 + k;
      Y[o] = make_float2(s02.x + s13.x, s02.y + s13.y);
      Y[o + Ns] = make_float2(d02.x - d13.y, d02.y + d13.x);  // v0 + i v1 - v2 - i v3
      Y[o + 2 * Ns] = make_float2(s02.x - s13.x, s02.y - s13.y);
      Y[o + 3 * Ns] = make_float2(d02.x + d13.y, d02.y - d13.x);  // v0 - i v1 - v2 + i v3
    }
    __syncthreads();
    float2* t = X;
    X = Y;
    Y = t;
  }
  // X: (S_k, h S'_k). Intervals k = tid + 512 q into registers, then the table over the buffers
  constexpr int QM = (1 << SG_TAB_LOGN_MAX) / SG_TAB_THREADS;
  float4 c[QM];
#pragma unroll
  for (int q = 0; q < QM; ++q) {
    const int k = threadIdx.x + q * SG_TAB_THREADS;
    if (k < N) {
      const float2 p0 = X[k], p1 = X[(k + 1) & (N - 1)];
      c[q] = make_float4(p0.x, p0.y, 3.f * (p1.x - p0.x) - 2.f * p0.y - p1.y, 2.f * (p0.x - p1.x) + p0.y + p1.y);
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < QM; ++q) {
    const int k = threadIdx.x + q * SG_TAB_THREADS;
    if (k < N) lt[k] = c[q];
  }
}

// Blocks of 64 samples of a task from the table at lane phases x, x + dx, ...
// (fixed point), their table reads issued together. FULL: all exist and land 1:1
// in [dj0, dj1) (no per-lane tests).
struct TabTask;
template <int NB, bool FULL, typename TT>
__device__ __forceinline__ void tab_blocks(const float4* __restrict__ lt, int logn, const TT& T,
                                           float* __restrict__ w, uint32_t x, uint32_t dx, int l, float& tmax) {
  float4 c[NB];
  uint32_t xs[NB];
#pragma unroll
  for (int s = 0; s < NB; ++s) {
    xs[s] = x + (uint32_t)s * dx;
    c[s] = lt[xs[s] >> (32 - logn)];
  }
#pragma unroll
  for (int s = 0; s < NB; ++s) {
    const float f = (float)(xs[s] << logn) * 2.3283064365386963e-10f;  // [0, 1]
    const float y = fmaf(f, fmaf(f, fmaf(f, c[s].w, c[s].z), c[s].y), c[s].x);
    if (FULL) {
      w[64 * s] = y;
      tmax = fmaxf(tmax, y);
    } else if (l + 64 * s < T.len) {
      w[64 * s] = y;
      const int j = T.j0 + l + 64 * s;
      tmax = (j >= T.dj0 && j < T.dj1) ? fmaxf(tmax, y) : tmax;
    }
  }
}

// The fields of a task the table path reads (48 B in LDS instead of 128)
struct TabTask {
  double c0, c1;
  int64_t off;    // W offset of epoch sample 0; direct jobs: output offset of epoch sample 0
  int32_t mbase, j0, len, dj0, dj1, dk0;
};
// A direct job's samples of one task in its window [dj0, dj1): pass 1 (STORE false)
// the max, pass 2 out[off + j] = y / max * fade(dk0 + j) (sg_harm_copy's arithmetic).
// Blocks of 4 x 64 samples on the W path's grid; a block inside the window and
// clear of the fades takes no per-lane tests.
template <bool STORE, bool CHECK>
__device__ __forceinline__ void tab_dblocks(const float4* __restrict__ lt, int logn, float* __restrict__ w,
                                            uint32_t x, uint32_t dx, int l, int ls, int le, float inv, int lf,
                                            int64_t L, int64_t k, float& tmax) {
  float4 c[4];
  uint32_t xs[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    xs[s] = x + (uint32_t)s * dx;
    c[s] = lt[xs[s] >> (32 - logn)];
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const float f = (float)(xs[s] << logn) * 2.3283064365386963e-10f;
    const float y = fmaf(f, fmaf(f, fmaf(f, c[s].w, c[s].z), c[s].y), c[s].x);
    const bool ok = !CHECK || (l + 64 * s >= ls && l + 64 * s < le);
    if (STORE) {
      float v = y * inv;
      if (CHECK && lf >= 2) v *= fade_at(lf, L, k + 64 * s);
      if (ok) w[64 * s] = v;
    } else {
      tmax = ok ? fmaxf(tmax, y) : tmax;
    }
  }
}
template <bool STORE>
__device__ __forceinline__ void tab_direct(const float4* __restrict__ lt, int logn, const TabTask& T,
                                           float* __restrict__ base, int lane, float inv, int lf, int64_t L,
                                           float& tmax) {
  const int ls = max(0, T.dj0 - T.j0), le = min(T.len, T.dj1 - T.j0);  // task samples in the window
  if (le <= ls) return;
  // the lane phases of the W path (x at sample lane, + dx per 64 samples, mod 2^32):
  // the same samples bit for bit
  constexpr double TWO32 = 4294967296.0;
  const double P = fma((double)(T.mbase + lane), T.c1, T.c0);
  const double d64 = 64.0 * T.c1;
  const uint32_t dx = (uint32_t)(uint64_t)((d64 - floor(d64)) * TWO32 + 0.5);
  const int lb = ls & ~63;
  uint32_t x = (uint32_t)(uint64_t)((P - floor(P)) * TWO32) + (uint32_t)(lb >> 6) * dx;
  float* __restrict__ wp = base + T.off + T.j0 + lane;
  const int64_t kt = (int64_t)T.dk0 + T.j0;  // syllable sample of task sample 0
#pragma unroll 1
  for (int l0 = lb; l0 < le; l0 += 256, x += 4u * dx) {
    const bool ramp = lf >= 2 && (kt + l0 < lf || kt + l0 + 256 > L - lf);
    if (l0 >= ls && l0 + 256 <= le && !ramp)
      tab_dblocks<STORE, false>(lt, logn, wp + l0, x, dx, l0 + lane, ls, le, inv, lf, L, kt + l0 + lane, tmax);
    else
      tab_dblocks<STORE, true>(lt, logn, wp + l0, x, dx, l0 + lane, ls, le, inv, lf, L, kt + l0 + lane, tmax);
  }
}

// One workgroup per SgTabJob (dynamic LDS: the table and twiddles, 18 N bytes).
// The job's task fields are staged in LDS with the amplitude column, before any
// store: loads and stores share vmcnt, so a descriptor load after a task's stores
// would wait for all of them to complete. At N = 2048, 4 workgroups fit per CU.
// SG_TAB_DIRECT jobs hold a whole syllable without crossfades, envelope or drift:
// the workgroup takes its max itself (pass 1, every task's in-window samples)
// and writes the final samples to the output (pass 2) instead of W, where
// sg_harm_copy would have read them back.
extern "C" __global__ __launch_bounds__(SG_TAB_THREADS) __attribute__((amdgpu_waves_per_eu(8))) void sg_sine_bank_tab(
    const SgTabJob* __restrict__ jobs, const SgWTask* __restrict__ tasks, const float* __restrict__ amps,
    const SgSyllable* __restrict__ syls, float* __restrict__ W, float* __restrict__ out_buf,
    float* __restrict__ fs, float* __restrict__ taskmax) {
  extern __shared__ float4 lt[];
  __shared__ float la[SG_ROWS_F32 + 4];
  __shared__ TabTask ts[SG_TAB_TASKS];
  __shared__ float red[SG_TAB_THREADS / 64];
  const SgTabJob J = jobs[blockIdx.x];
  const int logn = J.logn;
  const bool direct = J.flags & SG_TAB_DIRECT;
  int64_t out0 = 0, L = 0;
  int lf = 0;
  float* obase = W;
  if (direct) {
    const SgSyllable& sy = syls[J.syl];
    out0 = sy.out_off;
    L = sy.L;
    lf = sy.fade;
    obase = sy.dst_fs ? fs : out_buf;
  }
  for (int r = threadIdx.x; r < J.Rn; r += SG_TAB_THREADS) la[r] = amps[J.a_off + r];
  for (int q = threadIdx.x; q < J.n; q += SG_TAB_THREADS) {
    const SgWTask& T = tasks[J.t0 + q];
    ts[q] = TabTask{T.c0, T.c1, direct ? out0 + T.dk0 : T.w_off, T.mbase, T.j0, T.len, T.dj0, T.dj1, (int32_t)T.dk0};
  }
  __syncthreads();
  tab_build(lt, la, J.Rn, logn);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr double TWO32 = 4294967296.0;
  if (direct) {
    float wm = 0.f;
    for (int q = wave; q < J.n; q += SG_TAB_THREADS / 64) {
      float tmax = 0.f;
      tab_direct<false>(lt, logn, ts[q], obase, lane, 0.f, lf, L, tmax);
      wm = fmaxf(wm, wave_max(tmax));
    }
    if (lane == 0) red[wave] = wm;
    __syncthreads();
    float m = red[0];
#pragma unroll
    for (int w = 1; w < SG_TAB_THREADS / 64; ++w) m = fmaxf(m, red[w]);
    // every task slot of the syllable holds the syllable max: sg_syl_max takes the same value
    for (int q = threadIdx.x; q < J.n; q += SG_TAB_THREADS) taskmax[(int64_t)J.t0 + q] = m;
    const float inv = 1.f / m;
    float unused = 0.f;
    for (int q = wave; q < J.n; q += SG_TAB_THREADS / 64) tab_direct<true>(lt, logn, ts[q], obase, lane, inv, lf, L, unused);
    return;
  }
  for (int q = wave; q < J.n; q += SG_TAB_THREADS / 64) {
    const int64_t ti = (int64_t)J.t0 + q;
    const TabTask T = ts[q];
    // the lane's phase at its first sample and the advance over 64 samples, in
    // 2^-32 cycles (the fp64 phase of sample_setup, reduced mod 1)
    const double P = fma((double)(T.mbase + lane), T.c1, T.c0);
    uint32_t x = (uint32_t)(uint64_t)((P - floor(P)) * TWO32);
    const double d64 = 64.0 * T.c1;
    const uint32_t dx = (uint32_t)(uint64_t)((d64 - floor(d64)) * TWO32 + 0.5);
    float* __restrict__ wp = W + T.off + T.j0 + lane;
    float tmax = 0.f;
    int l0 = 0;
#pragma unroll 1
    for (; l0 + 256 <= T.len; l0 += 256, x += 4u * dx) {
      const int jp = T.j0 + l0;
      if (jp >= T.dj0 && jp + 256 <= T.dj1)
        tab_blocks<4, true>(lt, logn, T, wp + l0, x, dx, 0, tmax);
      else
        tab_blocks<4, false>(lt, logn, T, wp + l0, x, dx, l0 + lane, tmax);
    }
#pragma unroll 1
    for (; l0 < T.len; l0 += 64, x += dx) tab_blocks<1, false>(lt, logn, T, wp + l0, x, dx, l0 + lane, tmax);
    const float wm = wave_max(tmax);
    if (lane == 0) taskmax[ti] = wm;
  }
}

// per-syllable max over its task slots and crossfade-piece slots
extern "C" __global__ __launch_bounds__(256) void sg_syl_max(const SgSyllable* __restrict__ syls,
                                                             const float* __restrict__ taskmax,
                                                             const float* __restrict__ ptilemax,
                                                             float* __restrict__ maxes) {
  const SgSyllable& sy = syls[blockIdx.x];
  float m = 0.f;
  for (int64_t i = threadIdx.x; i < sy.ntask; i += 256) m = fmaxf(m, taskmax[sy.task0 + i]);
  for (int i = threadIdx.x; i < sy.nptile; i += 256) m = fmaxf(m, ptilemax[sy.ptile0 + i]);
  __shared__ float red[4];
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) maxes[sy.max_slot] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

namespace {
template <typename V>
__device__ __forceinline__ V piece_value(const SgPiece& p, const V* __restrict__ W, int64_t q) {
  if (p.nterms < 0) return W[p.t[0].src + q];
  V v = 0;
  const V qf = (V)q;
  for (int t = 0; t < p.nterms; ++t)
    v = vfma(vfma(qf, vfma(qf, (V)p.t[t].w2, (V)p.t[t].w1), (V)p.t[t].w0), W[p.t[t].src + q], v);
  return v;
}

// max over crossfade pieces (multi-term); tiles list (syl, piece, q0)
template <typename V>
__device__ __forceinline__ void piece_max_body(const SgSylTile* __restrict__ ptiles, const SgPiece* __restrict__ pieces,
                                               const SgSyllable* __restrict__ syls, const double* __restrict__ cknots,
                                               const V* __restrict__ W, float* __restrict__ ptilemax) {
  const SgSylTile tl = ptiles[blockIdx.x];
  const SgPiece& p = pieces[tl.piece];
  const SgSyllable& sy = syls[tl.syl];
  const int64_t q = tl.k0 + threadIdx.x;
  float cand = 0.f;
  if (q < p.len) {
    const V v = piece_value(p, W, q);
    cand = (float)v;
    if (sy.env.kind != 0) cand = (float)((double)v * contour_at(sy.env, cknots, sy.L, p.start + q));
  }
  __shared__ float red[4];
  const float wm = wave_max(cand);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = wm;
  __syncthreads();
  if (threadIdx.x == 0) {
    ptilemax[blockIdx.x] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  }
}
}  // namespace

extern "C" __global__ __launch_bounds__(256) void sg_piece_max(
    const SgSylTile* __restrict__ ptiles, const SgPiece* __restrict__ pieces, const SgSyllable* __restrict__ syls,
    const double* __restrict__ cknots, const float* __restrict__ W, float* __restrict__ ptilemax) {
  piece_max_body<float>(ptiles, pieces, syls, cknots, W, ptilemax);
}
extern "C" __global__ __launch_bounds__(256) void sg_piece_max_hp(
    const SgSylTile* __restrict__ ptiles, const SgPiece* __restrict__ pieces, const SgSyllable* __restrict__ syls,
    const double* __restrict__ cknots, const double* __restrict__ W64, float* __restrict__ ptilemax) {
  piece_max_body<double>(ptiles, pieces, syls, cknots, W64, ptilemax);
}

// out[k] = assembled[k] * env[k] / max * fade[k] * drift[k]   (R/source.R:436-467)
// A tile lying inside one direct piece whose source and destination share their
// 16-B residue moves float4s (4 consecutive samples per thread); otherwise each
// thread takes samples k0 + 256 e + tid.

// Fast path of the finalize (tiles from the planner's split, SgCopyTile):
// one wavefront per tile of <= SG_COPY_TILE_MAX samples; aligned tiles keep up to
// sixteen float4 loads per lane in flight before any store; one dependent descriptor level
// (tile -> data + max).
extern "C" __global__ __launch_bounds__(256) void sg_harm_copy(const SgCopyTile* __restrict__ tiles, int64_t ntiles,
                                                               const float* __restrict__ W,
                                                               const float* __restrict__ maxes,
                                                               float* __restrict__ out_buf, float* __restrict__ fs) {
  const int lane = threadIdx.x & 63;
  const int64_t ti = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (ti >= ntiles) return;
  const SgCopyTile T = tiles[ti];
  const float* __restrict__ src = W + T.src;
  float* __restrict__ dst = ((T.flags & SG_COPY_FS) ? fs : out_buf) + T.dst;
  const float inv_max = 1.f / maxes[T.max_slot];
  constexpr int E = SG_COPY_TILE_MAX / 256;
  if (T.flags & SG_COPY_VEC) {
    // source and destination share their 16-B residue: a scalar head up to the
    // destination's alignment, float4s, a scalar tail (h, nt < 4; wave-uniform)
    const int h = min((4 - (int)(T.dst & 3)) & 3, T.n);
    const int nb = (T.n - h) & ~3, nt = T.n - h - nb;
    if (lane < h || (lane >= 4 && lane < 4 + nt)) {
      const int q = lane < h ? lane : h + nb + lane - 4;
      float v = src[q] * inv_max;
      if (T.fade >= 2) v *= fade_at(T.fade, T.L, T.k0 + q);
      dst[q] = v;
    }
    const float* __restrict__ s4 = src + h;
    float* __restrict__ d4 = dst + h;
    const int64_t k4 = T.k0 + h;
    float4 v[E];
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (256 * e + 4 * lane < nb) v[e] = *reinterpret_cast<const float4*>(s4 + 256 * e + 4 * lane);
    const bool ramp = T.fade >= 2 && (k4 < T.fade || k4 + nb > T.L - T.fade);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (256 * e + 4 * lane >= nb) break;
      v[e].x *= inv_max; v[e].y *= inv_max; v[e].z *= inv_max; v[e].w *= inv_max;
      if (ramp) {
        const int64_t k = k4 + 256 * e + 4 * lane;
        v[e].x *= fade_at(T.fade, T.L, k); v[e].y *= fade_at(T.fade, T.L, k + 1);
        v[e].z *= fade_at(T.fade, T.L, k + 2); v[e].w *= fade_at(T.fade, T.L, k + 3);
      }
      *reinterpret_cast<float4*>(d4 + 256 * e + 4 * lane) = v[e];
    }
  } else {  // misaligned or short runs, zero pieces
    const bool zero = T.flags & SG_COPY_ZERO;
    for (int q = lane; q < T.n; q += 64) {
      float v = zero ? 0.f : src[q] * inv_max;
      if (T.fade >= 2) v *= fade_at(T.fade, T.L, T.k0 + q);
      dst[q] = v;
    }
  }
}

#ifndef SG_FIN_PRELOAD
#define SG_FIN_PRELOAD 1
#endif
// General path: the tiles the planner did not give to sg_harm_copy (crossfade
// pieces, amplitude envelope, drift, misaligned slots).
// V = double: an fp64 syllable (W64 -> fh; out_buf is fh, fs unused)
template <typename V = float>
__device__ __forceinline__ void finalize_tile(const SgSylTile& tl, const SgPiece* __restrict__ pieces,
                                              const SgSyllable* __restrict__ syls, const double* __restrict__ cknots,
                                              const V* __restrict__ W, const float* __restrict__ maxes,
                                              V* __restrict__ out_buf, V* __restrict__ fs,
                                              int wv, double* lkw) {
  const SgSyllable& sy = syls[tl.syl];
  int ecur = -1;  // a lane's samples increase: the envelope interval is found by stepping
  int gcur = -1;  // the same for the bout's global envelope (placed syllables)
  constexpr bool F64 = sizeof(V) == 8;
  V* __restrict__ out = (!F64 && sy.dst_fs) ? fs : out_buf;
  const V inv_max = (V)1 / (V)maxes[sy.max_slot];
  const int pend = sy.piece0 + sy.npiece;
  const int64_t tile_end = tl.k0 + 1024 < sy.L ? tl.k0 + 1024 : sy.L;
  // general path: wave w owns samples [k0 + 256 w, +256), lane l takes
  // c0 + 64 e + l (coalesced). The planner gives each wave the piece and the
  // drift-knot interval of its first sample; up to 8 knots from there are
  // held as wave-uniform values and each lane picks its interval by compares
  // (no dependent loads); chunks spanning more knots or pieces step per lane.
  const int lane = threadIdx.x & 63;
  const int64_t c0 = tl.k0 + 256 * wv;
  if (c0 >= tile_end) return;
  const int64_t c1 = c0 + 256 < tile_end ? c0 + 256 : tile_end;
  const int pu = tl.wpiece[wv];
  const bool one_piece = pu + 1 >= pend || pieces[pu + 1].start >= c1;
  const SgLinear dr = sy.drift;
  const bool drift = dr.nk > 1;
  const int d0 = tl.wdrift[wv];
  constexpr int KW = 8;
  double xs[KW], ys[KW];
  bool local_knots = false;
  const double dby = drift ? (dr.x1 - dr.x0) / (double)(sy.L - 1) : 0.0;
  auto u_at = [&](int64_t k) -> double {
    if (k == 0) return dr.x0;
    if (k == sy.L - 1) return dr.x1;
    return (k < sy.L / 2) ? dr.x0 + (double)k * dby : dr.x1 - (double)(sy.L - 1 - k) * dby;
  };
  // fp32 drift (V = float): the planner's per-interval lines (kb_t, a_t, b_t) after the
  // drift knots (sg_plan_harm.cpp); a chunk inside intervals d0 .. d0 + 6 picks its
  // interval by integer compares against the wave-uniform kb_t and takes one FMA, with
  // no per-chunk fp64 set-up. The fp64 evaluation per sample (interval compares, approx
  // arithmetic, the product) was 38 % of this kernel (r05r: 3.36 -> 2.07 ms per C5
  // launch without drift); a sample next to a knot may take the neighbouring line, equal
  // there to within one sample's step.
  // (lane q < 8 loads line d0 + q into the wave's LDS slot, a view of lkw: kb relative to
  // c0 as int [0, 8), then (a, b) float pairs; the uniform values stay out of SGPRs,
  // which this kernel spills)
  bool fast32 = false;
  int* const lkb = reinterpret_cast<int*>(lkw);
  float* const lab = reinterpret_cast<float*>(lkw) + KW;
  int kbr[KW - 2];
  if (!F64 && drift) {
    const double* lt = cknots + dr.k_off + 2 * (int64_t)dr.nk;
    const int last = dr.nk - 2;  // intervals 0 .. nk - 2
    if (lane < KW) {
      const int t = d0 + lane <= last ? d0 + lane : last;
      const uint64_t bits = __builtin_bit_cast(uint64_t, lt[2 * t + 1]);
      const int64_t rel = (int64_t)lt[2 * t] - c0;
      lkb[lane] = d0 + lane <= last ? (int)(rel < (1 << 30) ? rel : (1 << 30)) : 1 << 30;
      lab[2 * lane] = __builtin_bit_cast(float, (uint32_t)bits);
      lab[2 * lane + 1] = __builtin_bit_cast(float, (uint32_t)(bits >> 32));
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    fast32 = (int)(c1 - 1 - c0) < lkb[KW - 1];  // every sample inside intervals d0 .. d0 + 6
#pragma unroll
    for (int q = 0; q < KW - 2; ++q) kbr[q] = lkb[q + 1];
    __builtin_amdgcn_wave_barrier();  // the slow path's set-up below rewrites the slot
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (drift && !fast32) {
    const double* x = cknots + dr.k_off;
#pragma unroll
    for (int t = 0; t < KW; ++t) {
      const int idx = d0 + t < dr.nk ? d0 + t : dr.nk - 1;
      xs[t] = x[idx];
      ys[t] = x[dr.nk + idx];
    }
    // every sample of the chunk lies in intervals d0 .. d0 + KW - 2
    local_knots = d0 + KW - 1 >= dr.nk - 1 || u_at(c1 - 1) < xs[KW - 1];
    // per interval (x_t, y_t, slope_t) in the wave's LDS slot: a lane then reads its
    // interval by index instead of selecting four doubles through KW - 2 compares,
    // and multiplies by the slope instead of dividing (a few fp64 ulps from approx()'s
    // (y_j - y_i) * ((u - x_i) / (x_j - x_i)), far below the fp32 output)
    if (lane < KW - 1) {
      double xv = xs[0], yv = ys[0], x1 = xs[1], y1 = ys[1];
#pragma unroll
      for (int t = 1; t < KW - 1; ++t)
        if (lane == t) { xv = xs[t]; yv = ys[t]; x1 = xs[t + 1]; y1 = ys[t + 1]; }
      lkw[3 * lane] = xv;
      lkw[3 * lane + 1] = yv;
      lkw[3 * lane + 2] = x1 > xv ? (y1 - yv) / (x1 - xv) : 0.0;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }

  int p = pu, di = d0;
  // a chunk clear of both fade ramps multiplies by exactly 1: skip it (wave-uniform)
  const bool ramp = sy.fade >= 2 && (c0 < sy.fade || c1 > sy.L - sy.fade);
  // a chunk inside one direct piece (most of them): its four epoch-waveform reads are
  // issued together, unconditionally (a lane past c1 rereads sample c1 - 1), before
  // the per-sample work; in the loop below each read sat behind its own branch and
  // waited alone (one read in flight per lane)
  V pre[4];
  bool direct1 = false;
  if (SG_FIN_PRELOAD && one_piece) {
    const SgPiece& pc = pieces[pu];
    if (pc.nterms < 0) {
      direct1 = true;
      const V* __restrict__ src = W + (pc.t[0].src - pc.start);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t k = c0 + 64 * e + lane;
        pre[e] = src[k < c1 ? k : c1 - 1];
      }
    }
  }
  V res[4];  // every load of the chunk before its stores
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int64_t k = c0 + 64 * e + lane;
    res[e] = 0;
    if (k >= c1) break;
    V x;
    if (direct1) {
      x = pre[e];
    } else if (one_piece) {
      const SgPiece& pc = pieces[pu];
      x = pc.nterms == 0 ? (V)0 : piece_value(pc, W, k - pc.start);
    } else {
      while (p + 1 < pend && pieces[p + 1].start <= k) ++p;
      const SgPiece& pc = pieces[p];
      x = pc.nterms == 0 ? (V)0 : piece_value(pc, W, k - pc.start);
    }
    if (sy.env.kind != 0) {
      x = (V)((double)x * sgd::contour_at_cursor(sy.env, cknots, sy.L, k, ecur));
    }
    x *= inv_max;
    if (ramp) x *= fade_at<V>(sy.fade, sy.L, k);
    if (fast32) {
      const int r = (int)(k - c0);
      int t = 0;
#pragma unroll
      for (int q = 0; q < KW - 2; ++q) t += r >= kbr[q] ? 1 : 0;
      const float2 ab = reinterpret_cast<const float2*>(lab)[t];
      x *= (V)fmaf(ab.y, (float)(r - lkb[t]), ab.x);
    } else if (drift) {
      double dm;
      if (local_knots) {  // linear_at's interval and arithmetic, knots from registers
        const double u = u_at(k);
        int t = 0;  // the conditions hold for a prefix of t: their count is the interval
#pragma unroll
        for (int q = 1; q < KW - 1; ++q) t += (d0 + q <= dr.nk - 2 && xs[q] <= u) ? 1 : 0;
        const double xi = lkw[3 * t], yi = lkw[3 * t + 1], sl = lkw[3 * t + 2];
        dm = u == xi ? yi : fma(sl, u - xi, yi);
      } else {
        dm = sgd::linear_at_cursor(dr, cknots, sy.L, k, di);
      }
      x = (V)((double)x * dm);
    } else if (dr.nk == 1) {
      x = (V)((double)x * cknots[dr.k_off + 1]);
    }
    if (sy.genv.kind != 0)  // placed under the bout's global envelope (the pre-filter mix's product)
      x = (V)((double)x * sgd::contour_at_cursor(sy.genv, cknots, sy.genv_len, sy.genv_off + k, gcur));
    res[e] = x;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int64_t k = c0 + 64 * e + lane;
    if (k < c1) out[sy.out_off + k] = res[e];
  }
}

// SG_FIN_TILES consecutive 1024-sample tiles per workgroup: the descriptor
// chain (tile -> syllable -> piece, drift knots) of a syllable's next tile hits cache
constexpr int SG_FIN_TILES = 4;  // r02: 2 / 8 neutral; r04: 1 / 2 neutral
// Registers capped for 8 waves per SIMD (SGPRs 106 -> 78, 7 -> 8 waves; r04: 3.75 -> 3.40 ms per C5 launch).
// (A whole-tile path for tiles inside one direct piece measured 5.93 -> 7.82 ms on C5;
// one wave per tile, LDS-staged envelope knots: no better.)
extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void sg_harm_finalize(
    const SgSylTile* __restrict__ stiles, int64_t ntiles, const SgPiece* __restrict__ pieces,
    const SgSyllable* __restrict__ syls, const double* __restrict__ cknots, const float* __restrict__ W,
    const float* __restrict__ maxes, float* __restrict__ out_buf, float* __restrict__ fs) {
  __shared__ double lk[4][3 * 8];  // per wave: drift intervals (x, y, slope)
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  double* lkw = lk[wv];
#pragma unroll 1
  for (int i = 0; i < SG_FIN_TILES; ++i) {
    const int64_t t = (int64_t)blockIdx.x * SG_FIN_TILES + i;
    if (t >= ntiles) break;
    finalize_tile(stiles[t], pieces, syls, cknots, W, maxes, out_buf, fs, wv, lkw);
  }
}

// fp64 syllables (SgSyllable::hp): W64 -> fh, the general path in fp64
extern "C" __global__ __launch_bounds__(256) void sg_harm_finalize_hp(
    const SgSylTile* __restrict__ stiles, int64_t ntiles, const SgPiece* __restrict__ pieces,
    const SgSyllable* __restrict__ syls, const double* __restrict__ cknots, const double* __restrict__ W64,
    const float* __restrict__ maxes, double* __restrict__ fh) {
  __shared__ double lk[4][3 * 8];
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t t = blockIdx.x;
  if (t >= ntiles) return;
  finalize_tile<double>(stiles[t], pieces, syls, cknots, W64, maxes, fh, fh, wv, lk[wv]);
}

// ---------------------------------------------------------------- launchers
// ------------------------------------------------- amplitude blocks (K3)
// One workgroup per epoch job (run once, at upload): thread r owns row r of
// every glottal cycle and writes A[g][r] in fp32 (the sine banks form the column
// differences dA[g] = A[g + 1] - A[g] in fp32 where they stage the rows).
// The values come from the shared formula (sg_amp.h) or, for the host-built
// fallback, from the uploaded blocks.
__global__ __launch_bounds__(256) void sg_amp_build(const SgAmpJob* __restrict__ jobs,
                                                    const SgAmpCol* __restrict__ cols, const float* __restrict__ src,
                                                    const double* __restrict__ lg, float* __restrict__ amps) {
  const SgAmpJob J = jobs[blockIdx.x];
  for (int r = threadIdx.x; r < J.Rp; r += blockDim.x)
    for (int g = 0; g < J.G; ++g) {
      float a;
      if (r >= J.R) a = 0.f;
      else if (J.src_off >= 0) a = src[J.src_off + (int64_t)g * J.Rp + r];
      else a = (float)sg::amp_value(cols + J.col0, J, lg, g, r);
      amps[J.amp_off + (int64_t)g * J.Rp + r] = a;
    }
}

#include "sg_exec.h"
namespace sg {
#define SG_LAUNCHED(name)                                                                       \
  do {                                                                                          \
    const hipError_t _e = hipGetLastError();                                                    \
    if (_e != hipSuccess) throw SgError(SG_E_DEVICE, std::string("launch " name ": ") + hipGetErrorString(_e)); \
  } while (0)

void launch_amp_build(const DevicePlan& D, int64_t n_jobs, hipStream_t s) {
  if (n_jobs <= 0) return;
  hipLaunchKernelGGL(sg_amp_build, dim3((unsigned)n_jobs), dim3(256), 0, s, D.ampjobs, D.ampcols, D.ampsrc, D.elog2,
                     D.amps);
  SG_LAUNCHED("sg_amp_build");
}
void launch_sine_bank(const DevicePlan& D, int64_t k0, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  const int64_t nb = (n + 3) / 4;
  hipLaunchKernelGGL(sg_sine_bank, dim3((unsigned)nb), dim3(256), 0, s, D.tlong + k0, n, D.tasks, D.amps,
                     D.syls, D.cknots, D.W, D.taskmax);
  SG_LAUNCHED("sg_sine_bank");
}
// r0, n: the runs (D.srun) of the slice
void launch_sine_bank_pairs(const DevicePlan& D, int64_t r0, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(sg_sine_bank_pairs, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, D.tshort, D.srun + r0, n,
                     D.tasks, D.amps, D.W, D.taskmax);
  SG_LAUNCHED("sg_sine_bank_pairs");
}
void launch_sine_bank_tall(const DevicePlan& D, int64_t k0, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(sg_sine_bank_tall, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, D.tall + k0, n, D.tasks,
                     D.amps, D.syls, D.cknots, D.W, D.taskmax);
  SG_LAUNCHED("sg_sine_bank_tall");
}
// r0, n: the runs (D.trun) of the slice
void launch_sine_bank_tall_pairs(const DevicePlan& D, int64_t r0, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(sg_sine_bank_tall_pairs, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, D.tallp,
                     D.trun + r0, n, D.tasks, D.amps, D.W, D.taskmax);
  SG_LAUNCHED("sg_sine_bank_tall_pairs");
}
void launch_sine_bank_tab(const DevicePlan& D, int logn, int64_t j0, int64_t n, float* out, hipStream_t s) {
  if (n <= 0) return;
  // the table (16 N bytes, the FFT buffers during the build) and the twiddles (2 N)
  hipLaunchKernelGGL(sg_sine_bank_tab, dim3((unsigned)n), dim3(SG_TAB_THREADS), (size_t)18 << logn, s,
                     D.tabjobs + j0, D.tasks, D.amps, D.syls, D.W, out, D.fs, D.taskmax);
  SG_LAUNCHED("sg_sine_bank_tab");
}
void launch_piece_max(const DevicePlan& D, int64_t p0, int64_t n_ptiles, hipStream_t s) {
  if (n_ptiles <= 0) return;
  hipLaunchKernelGGL(sg_piece_max, dim3((unsigned)n_ptiles), dim3(256), 0, s, D.ptiles + p0, D.pieces, D.syls,
                     D.cknots, D.W, D.ptilemax + p0);
  SG_LAUNCHED("sg_piece_max");
}
void launch_syl_max(const DevicePlan& D, int64_t s0, int64_t n_syls, hipStream_t s) {
  if (n_syls <= 0) return;
  hipLaunchKernelGGL(sg_syl_max, dim3((unsigned)n_syls), dim3(256), 0, s, D.syls + s0, D.taskmax, D.ptilemax,
                     D.maxes);
  SG_LAUNCHED("sg_syl_max");
}
void launch_harm_copy(const DevicePlan& D, int64_t c0, int64_t n_ctiles, float* out, hipStream_t s) {
  if (n_ctiles <= 0) return;
  hipLaunchKernelGGL(sg_harm_copy, dim3((unsigned)((n_ctiles + 3) / 4)), dim3(256), 0, s, D.copy_tiles + c0, n_ctiles, D.W,
                     D.maxes, out, D.fs);
  SG_LAUNCHED("sg_harm_copy");
}
void launch_sine_bank_hp(const DevicePlan& D, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(sg_sine_bank_hp, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, D.thp, n, D.tasks, D.amps, D.syls,
                     D.cknots, D.W64, D.taskmax);
  SG_LAUNCHED("sg_sine_bank_hp");
}
void launch_piece_max_hp(const DevicePlan& D, int64_t p0, int64_t n_ptiles, hipStream_t s) {
  if (n_ptiles <= 0) return;
  hipLaunchKernelGGL(sg_piece_max_hp, dim3((unsigned)n_ptiles), dim3(256), 0, s, D.ptiles + p0, D.pieces, D.syls,
                     D.cknots, D.W64, D.ptilemax + p0);
  SG_LAUNCHED("sg_piece_max_hp");
}
void launch_harm_finalize_hp(const DevicePlan& D, int64_t n_stiles, hipStream_t s) {
  if (n_stiles <= 0) return;
  hipLaunchKernelGGL(sg_harm_finalize_hp, dim3((unsigned)n_stiles), dim3(256), 0, s, D.fin_tiles_hp, n_stiles, D.pieces,
                     D.syls, D.cknots, D.W64, D.maxes, D.fh);
  SG_LAUNCHED("sg_harm_finalize_hp");
}
void launch_harm_finalize(const DevicePlan& D, int64_t f0, int64_t n_stiles, float* out, hipStream_t s) {
  if (n_stiles <= 0) return;
  const int64_t per_block = SG_FIN_TILES;
  hipLaunchKernelGGL(sg_harm_finalize, dim3((unsigned)((n_stiles + per_block - 1) / per_block)), dim3(256), 0, s,
                     D.syl_tiles + f0, n_stiles, D.pieces, D.syls,
                     D.cknots, D.W, D.maxes, out, D.fs);
  SG_LAUNCHED("sg_harm_finalize");
}
}  // namespace sg
