// sg_dev.h — plain-old-data descriptors shared by the host planner and the
// gfx950 kernels. Everything here lives in HBM after sg_plan_upload().
#pragma once
#include <stdint.h>

// Cumulative-pitch segment: pitch_up[u] for u in (t0, t1] is the cubic
// y + dx*(b + dx*(c + dx*d)), dx = u - t0 (R's spline_eval keeps the left
// segment at an exact knot, R/utilities_soundgen.R:410 via stats splines.c).
// prefix = sum_{u' <= t0} pitch_up[u'] (long-double accumulated on host).
struct SgSeg {
  double t0;
  double prefix;
  double y, b, c, d;
};

// One subharmonic epoch of one syllable (R/source.R:389-427).
//   samples u = u0 + j, j in [0, n): W[j] = sum_r A_r(xo_j) * sin(2*pi*r*integr(u)/D)
//   xo_j = seq.int(x1, xG, length.out = n)[j]  (approx() compressed mapping)
//   A_r(x) = linear interpolation over knots[0..G) of column-major amps[G][R]
struct SgEpoch {
  int64_t w_off;     // scratch offset of W[0]
  int64_t amp_off;   // float offset of the [G][R] amplitude block
  int64_t knot_off;  // double offset of the G knots
  int32_t seg_off;   // first SgSeg of the syllable
  int32_t nseg;
  int32_t n;         // N_e samples
  int32_t G;         // knots / amplitude columns (>= 2)
  int32_t R;         // rows (multiple of 8, zero padded)
  int32_t u0;        // first sample, 1-based within the syllable
  double x1, xG;     // xout range
  double xby;        // (xG - x1) / (n - 1), as R's seq.int computes it
  double inv_srD;    // 1 / (samplingRate * D), D = nSubharm + 1
  // direct-copy window used for the fused max: W[j] lands at syllable
  // sample k = dk0 + j for j in [dj0, dj1) with weight 1.
  int32_t dj0, dj1;
  int64_t dk0;
  int32_t syl;       // syllable index
  int32_t pad;
};

constexpr int SG_SINE_TILE = 2048;  // samples per sine-bank workgroup (256 threads x 8)

struct SgTile {
  int32_t epoch;
  int32_t j0;  // first sample of the tile
  int32_t i0;  // amplitude interval of sample j0
  int32_t k0;  // pitch segment of sample j0
};

// A piece of an assembled syllable (crossFade() chain, R/utilities_soundgen.R:328-375):
// value(k) = sum_t (w0 + w1*q + w2*q^2) * W[src_t + q], q = k - start.
constexpr int SG_MAX_TERMS = 4;
struct SgTerm {
  int64_t src;
  float w0, w1, w2, pad;
};
struct SgPiece {
  int64_t start;  // syllable-local sample
  int32_t len;
  int32_t nterms;
  SgTerm t[SG_MAX_TERMS];
};

// Smooth contour over L samples (getSmoothContour(), R/smoothContours.R):
// kind 0 none(=1 after conversion), 1 flat, 2 seq(from,to), 3 fmm spline on
// xout = seq.int(x0, x1, L); then clamp, then optional 2^(v/10).
struct SgContour {
  int32_t kind;
  int32_t nk;        // spline knots
  int64_t k_off;     // offset (doubles) of x[nk], y, b, c, d arrays (5*nk)
  double a, b;       // flat value / seq from,to ; spline x0,x1
  double lo, hi;     // clamp (use -inf/inf when absent)
  int32_t db;        // 1: apply 2^(v/10)
  int32_t pad;
};

// Piecewise-linear approx() over knots (drift multiplier, R/source.R:459-467).
struct SgLinear {
  int32_t nk;        // 0 = none (multiplier 1)
  int32_t pad;
  int64_t k_off;     // x[nk], y[nk]
  double x0, x1;     // xout = seq.int(x0, x1, L)
};

struct SgSyllable {
  int64_t L;         // assembled length
  int64_t out_off;   // destination offset (final buffer or voiced scratch)
  int32_t piece0, npiece;
  int32_t fade;      // fade length (0/1 = none)
  int32_t max_slot;  // index into the per-syllable max array
  SgContour env;     // amplEnvelope (kind 0 = none)
  SgLinear drift;
};

// assemble/finalize tiles over syllable samples
struct SgSylTile {
  int32_t syl;
  int32_t piece;     // piece containing k0
  int64_t k0;
};
