// sg_amp.h — one element of a harmonic amplitude matrix, shared by the device
// build (sg_amp_build, sg_harm.hip) and the planner's host columns (crossfade
// zero crossings, filter-conditioning probes). The fp64 operations follow
// R's order exactly and are never contracted, so host and device agree bit
// for bit up to the pow / exp of each platform's math library.
#pragma once
#include <cmath>

#include "sg_dev.h"

#if defined(__HIP__)
#define SG_HD __host__ __device__ inline
#else
#define SG_HD inline
#endif

namespace sg {

// getRolloff() element (kept row h, 0-based; the planner sends only calls whose
// kept rows are 0..H-1) times the shimmer factor: 0 above Nyquist or below the
// throwaway, else 2^((dB - column max) / 10)   R/sourceSpectrum.R:118-186
// the element's dB before normalisation; false: -Inf (above Nyquist or under the throwaway)
SG_HD bool roll_db(const SgAmpCol& P, const SgAmpJob& J, const double* lg, int h, double* out) {
#pragma clang fp contract(off)
  const double hh = (double)(h + 1);
  if (hh * P.pitch >= J.nyq) return false;
  const double delta = (J.any_oct && h >= 1) ? P.oct * (P.pitch * hh - J.baseline) / 1000 : 0.0;
  double v = (P.slope * lg[h]) + delta;
  if (J.parab != 0) {
    if (P.rph < 3) {
      if (P.rph < 2 && h == 0) v = v + J.parab;
    } else if (hh <= P.rph) {
      v = v + P.pa * hh * hh + P.pb * hh + P.pc;
    }
  }
  if (v < J.thr) return false;
  *out = v;
  return true;
}

SG_HD double roll_value(const SgAmpCol& P, const SgAmpJob& J, const double* lg, int h) {
#pragma clang fp contract(off)
  double v;
  if (!roll_db(P, J, lg, h, &v)) return 0.0;
  return pow(2.0, (v - P.mx) / 10) * P.sh;
}

// getVocalFry_per_epoch()'s sideband weight for subharmonic s of cycle P
//   R/subharmonics.R:60-66
SG_HD double fry_ml(const SgAmpCol& P, const SgAmpJob& J, int s) {
#pragma clang fp contract(off)
  const double d = P.pitch * (double)s / (double)(J.nsub + 1), sd = P.sbw;
  if (sd == 0) return d == 0 ? NAN : 0.0;
  return exp(-0.5 * (d / sd) * (d / sd));
}

// A[g][r] of epoch J (g relative to the epoch, rank r = row r + 1 of R's
// rolloff_new): harmonic rows copy the rolloff; the sidebands between them
// interpolate the epoch's FIRST cycle's harmonics (R indexes the matrix
// linearly there) with per-cycle Gaussian weights; values under 2^(thr / 10)
// are zeroed   R/subharmonics.R:40-86
SG_HD double amp_value(const SgAmpCol* cols, const SgAmpJob& J, const double* lg, int g, int r) {
#pragma clang fp contract(off)
  const SgAmpCol& P = cols[J.g0 + g];
  if (J.nsub == 0) return roll_value(P, J, lg, r);
  const int D = J.nsub + 1, i = r + 1;
  double v;
  if (i % D == 0) {
    const int h = i / D - 1;
    v = h < J.H ? roll_value(P, J, lg, h) : 0.0;
  } else {
    const int block = i / D + 1, gg = i % D;
    const SgAmpCol& P0 = cols[J.g0];
    const double a = block >= 2 ? roll_value(P0, J, lg, block - 2) : 0.0;
    const double b = block - 1 < J.H ? roll_value(P0, J, lg, block - 1) : 0.0;
    v = a * fry_ml(P, J, gg) + b * fry_ml(P, J, J.nsub + 1 - gg);
  }
  return v < J.t01 ? 0.0 : v;
}

}  // namespace sg
