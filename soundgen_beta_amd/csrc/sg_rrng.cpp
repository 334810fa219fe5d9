// sg_rrng.cpp — R's default random number generation, restated so that a
// seeded call planned here draws exactly what `set.seed(seed); soundgen(...)`
// draws in R 3.4.0 (RNGkind "Mersenne-Twister", normal.kind "Inversion";
// SURVEY.md §8f rank 1). R is not vendored in the reference (it is the
// packrat R 3.4.0 runtime, packrat/packrat.lock:3); the algorithms restated:
//   src/main/RNG.c      RNG_Init (set.seed scrambling), MT_genrand, fixup
//   src/nmath/snorm.c   norm_rand, INVERSION: u = (int)(2^27 U1) + U2; qnorm5(u / 2^27)
//   src/nmath/qnorm.c   qnorm5 (Wichura 1988, AS 241 PPND16)
//   src/nmath/sexp.c    exp_rand (Ahrens & Dieter 1972, algorithm SA)
//   src/nmath/rgamma.c  rgamma (Ahrens & Dieter 1974 GS for a < 1, 1982 GD for a >= 1)
// The planner already restates rbinom(1, 1, p) and pre-3.6 sample() on top of
// unif_rand (sg_plan_soundgen.cpp), so binding these three draws to an
// sg_random reproduces R's whole stream. Pinned by R's published outputs
// (tests/test_rrng.py); rgamma's acceptance branches are parity-unpinned.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <new>

#include "soundgen_hip.h"

struct sg_rrng {
  uint32_t dummy[625];  // RNG.c layout: dummy[0] = mti, mt = dummy + 1
};

namespace {
constexpr int N = 624, M = 397;
constexpr uint32_t MATRIX_A = 0x9908b0dfU, UPPER_MASK = 0x80000000U, LOWER_MASK = 0x7fffffffU;
constexpr uint32_t TEMPERING_MASK_B = 0x9d2c5680U, TEMPERING_MASK_C = 0xefc60000U;
constexpr double i2_32m1 = 2.328306437080797e-10;  // 1 / (2^32 - 1)

void mt_sgenrand(uint32_t* mt, uint32_t seed) {  // only reached when mti == N + 1
  for (int i = 0; i < N; i++) {
    mt[i] = seed & 0xffff0000U;
    seed = 69069 * seed + 1;
    mt[i] |= (seed & 0xffff0000U) >> 16;
    seed = 69069 * seed + 1;
  }
}

double mt_genrand(sg_rrng* g) {
  static const uint32_t mag01[2] = {0x0U, MATRIX_A};
  uint32_t* mt = g->dummy + 1;
  int mti = (int)g->dummy[0];
  uint32_t y;
  if (mti >= N) {  // generate N words at one time
    if (mti == N + 1) mt_sgenrand(mt, 4357);
    int kk;
    for (kk = 0; kk < N - M; kk++) {
      y = (mt[kk] & UPPER_MASK) | (mt[kk + 1] & LOWER_MASK);
      mt[kk] = mt[kk + M] ^ (y >> 1) ^ mag01[y & 0x1];
    }
    for (; kk < N - 1; kk++) {
      y = (mt[kk] & UPPER_MASK) | (mt[kk + 1] & LOWER_MASK);
      mt[kk] = mt[kk + (M - N)] ^ (y >> 1) ^ mag01[y & 0x1];
    }
    y = (mt[N - 1] & UPPER_MASK) | (mt[0] & LOWER_MASK);
    mt[N - 1] = mt[M - 1] ^ (y >> 1) ^ mag01[y & 0x1];
    mti = 0;
  }
  y = mt[mti++];
  y ^= (y >> 11);
  y ^= (y << 7) & TEMPERING_MASK_B;
  y ^= (y << 15) & TEMPERING_MASK_C;
  y ^= (y >> 18);
  g->dummy[0] = (uint32_t)mti;
  return (double)y * 2.3283064365386963e-10;  // reals: [0, 1)
}

double fixup(double x) {  // RNG.c: keep unif_rand in (0, 1)
  if (x <= 0.0) return 0.5 * i2_32m1;
  if ((1.0 - x) <= 0.0) return 1.0 - 0.5 * i2_32m1;
  return x;
}

// qnorm(p, 0, 1, lower_tail = TRUE, log_p = FALSE) for p in (0, 1)
double qnorm_std(double p) {
  const double q = p - 0.5;
  double r, val;
  if (std::fabs(q) <= .425) {  // 0.075 <= p <= 0.925
    r = .180625 - q * q;
    val = q *
          (((((((r * 2509.0809287301226727 + 33430.575583588128105) * r + 67265.770927008700853) * r +
               45921.953931549871457) * r + 13731.693765509461125) * r + 1971.5909503065514427) * r +
            133.14166789178437745) * r + 3.387132872796366608) /
          (((((((r * 5226.495278852545925 + 28729.085735721942674) * r + 39307.89580009271061) * r +
               21213.794301586595867) * r + 5394.1960214247511077) * r + 687.1870074920579083) * r +
            42.313330701600911252) * r + 1.);
    return val;
  }
  r = q > 0 ? 1.0 - p : p;  // min(p, 1 - p) < 0.075
  r = std::sqrt(-std::log(r));
  if (r <= 5.) {  // min(p, 1 - p) >= exp(-25)
    r += -1.6;
    val = (((((((r * 7.7454501427834140764e-4 + .0227238449892691845833) * r + .24178072517745061177) * r +
               1.27045825245236838258) * r + 3.64784832476320460504) * r + 5.7694972214606914055) * r +
            4.6303378461565452959) * r + 1.42343711074968357734) /
          (((((((r * 1.05075007164441684324e-9 + 5.475938084995344946e-4) * r + .0151986665636164571966) * r +
               .14810397642748007459) * r + .68976733498510000455) * r + 1.6763848301838038494) * r +
            2.05319162663775882187) * r + 1.);
  } else {  // very close to 0 or 1
    r += -5.;
    val = (((((((r * 2.01033439929228813265e-7 + 2.71155556874348757815e-5) * r + .0012426609473880784386) * r +
               .026532189526576123093) * r + .29656057182850489123) * r + 1.7848265399172913358) * r +
            5.4637849111641143699) * r + 6.6579046435011037772) /
          (((((((r * 2.04426310338993978564e-15 + 1.4215117583164458887e-7) * r + 1.8463183175100546818e-5) * r +
               7.868691311456132591e-4) * r + .0148753612908506148525) * r + .13692988092273580531) * r +
            .59983220655588793769) * r + 1.);
  }
  if (q < 0.0) val = -val;
  return val;
}

// q[k] = sum_{j = 1..k+1} log(2)^j / j!  (sexp.c's table; q[15] == 1 within double precision)
struct ExpTable {
  double q[16];
  ExpTable() {
    const double l2 = 0.6931471805599453;
    double term = 1.0, s = 0.0;
    for (int k = 0; k < 16; ++k) {
      term *= l2 / (double)(k + 1);
      s += term;
      q[k] = s;
    }
    q[15] = 1.0;
  }
};
const ExpTable kExp;
}  // namespace

extern "C" {

int sg_rrng_create(int32_t seed, sg_rrng** out) {
  if (!out) return SG_E_ARG;
  sg_rrng* g = new (std::nothrow) sg_rrng;
  if (!g) return SG_E_NOMEM;
  sg_rrng_set_seed(g, seed);
  *out = g;
  return SG_OK;
}

void sg_rrng_destroy(sg_rrng* g) { delete g; }

void sg_rrng_set_seed(sg_rrng* g, int32_t seed) {  // RNG_Init(MERSENNE_TWISTER, seed) + FixupSeeds
  uint32_t s = (uint32_t)seed;
  for (int j = 0; j < 50; j++) s = (69069 * s + 1);  // initial scrambling
  for (int j = 0; j < 625; j++) {
    s = (69069 * s + 1);
    g->dummy[j] = s;
  }
  g->dummy[0] = 624;  // FixupSeeds(initial): mti = N
}

double sg_rrng_unif(sg_rrng* g) { return fixup(mt_genrand(g)); }
// runif(n): the same values as n sg_rrng_unif calls. The state's words are tempered
// and scaled a block at a time (a loop the compiler vectorises); mt_genrand refills
// the state exactly as it would one word at a time.
void sg_rrng_unif_n(sg_rrng* g, double* out, int64_t n) {
  uint32_t* mt = g->dummy + 1;
  int64_t i = 0;
  while (i < n) {
    int mti = (int)g->dummy[0];
    if (mti >= N) {  // refill (and the set.seed-less first call) through the one-word path
      out[i++] = fixup(mt_genrand(g));
      continue;
    }
    const int64_t m = std::min<int64_t>(n - i, N - mti);
    for (int64_t q = 0; q < m; ++q) {
      uint32_t y = mt[mti + q];
      y ^= (y >> 11);
      y ^= (y << 7) & TEMPERING_MASK_B;
      y ^= (y << 15) & TEMPERING_MASK_C;
      y ^= (y >> 18);
      const double x = (double)y * 2.3283064365386963e-10;
      out[i + q] = x <= 0.0 ? 0.5 * i2_32m1 : ((1.0 - x) <= 0.0 ? 1.0 - 0.5 * i2_32m1 : x);
    }
    g->dummy[0] = (uint32_t)(mti + m);
    i += m;
  }
}

double sg_rrng_norm(sg_rrng* g) {
  const double BIG = 134217728;  // 2^27: unif_rand() alone is not precise enough
  double u = sg_rrng_unif(g);
  u = (int)(BIG * u) + sg_rrng_unif(g);
  return qnorm_std(u / BIG);
}

double sg_rrng_exp(sg_rrng* g) {
  const double* q = kExp.q;
  double a = 0.;
  double u = sg_rrng_unif(g);
  while (u <= 0. || u >= 1.) u = sg_rrng_unif(g);
  for (;;) {
    u += u;
    if (u > 1.) break;
    a += q[0];
  }
  u -= 1.;
  if (u <= q[0]) return a + u;
  int i = 0;
  double ustar = sg_rrng_unif(g), umin = ustar;
  do {
    ustar = sg_rrng_unif(g);
    if (umin > ustar) umin = ustar;
    i++;
  } while (u > q[i]);
  return a + umin * q[0];
}

double sg_rrng_gamma(sg_rrng* g, double a, double scale) {
  const double sqrt32 = 5.656854;
  const double exp_m1 = 0.36787944117144233;  // exp(-1)
  const double q1 = 0.04166669, q2 = 0.02083148, q3 = 0.00801191, q4 = 0.00144121, q5 = -7.388e-5,
               q6 = 2.4511e-4, q7 = 2.424e-4;
  const double a1 = 0.3333333, a2 = -0.250003, a3 = 0.2000062, a4 = -0.1662921, a5 = 0.1423657,
               a6 = -0.1367177, a7 = 0.1233795;
  if (std::isnan(a) || std::isnan(scale)) return NAN;
  if (a <= 0.0 || scale <= 0.0) {
    if (scale == 0. || a == 0.) return 0.;
    return NAN;
  }
  if (!std::isfinite(a) || !std::isfinite(scale)) return INFINITY;

  if (a < 1.) {  // GS algorithm for parameters a < 1
    const double e = 1.0 + exp_m1 * a;
    double x;
    for (;;) {
      const double p = e * sg_rrng_unif(g);
      if (p >= 1.0) {
        x = -std::log((e - p) / a);
        if (sg_rrng_exp(g) >= (1.0 - a) * std::log(x)) break;
      } else {
        x = std::exp(std::log(p) / a);
        if (sg_rrng_exp(g) >= x) break;
      }
    }
    return scale * x;
  }
  // GD algorithm (a >= 1). Step 1 (R caches these per a; recomputing is identical)
  const double s2 = a - 0.5, s = std::sqrt(s2), d = sqrt32 - s * 12.;
  // Step 2: t = standard normal deviate, x = (s, 1/2)-normal deviate; immediate acceptance
  double t = sg_rrng_norm(g);
  double x = s + 0.5 * t;
  const double ret_val = x * x;
  if (t >= 0.) return scale * ret_val;
  // Step 3: squeeze acceptance
  double u = sg_rrng_unif(g);
  if (d * u <= t * t * t) return scale * ret_val;
  // Step 4: q0, b, si, c
  const double r = 1. / a;
  const double q0 = ((((((q7 * r + q6) * r + q5) * r + q4) * r + q3) * r + q2) * r + q1) * r;
  double b, si, c;
  if (a <= 3.686) {
    b = 0.463 + s + 0.178 * s2;
    si = 1.235;
    c = 0.195 / s - 0.079 + 0.16 * s;
  } else if (a <= 13.022) {
    b = 1.654 + 0.0076 * s2;
    si = 1.68 / s + 0.275;
    c = 0.062 / s + 0.024;
  } else {
    b = 1.77;
    si = 0.75;
    c = 0.1515 / s;
  }
  double q, v;
  // Step 5-7: quotient acceptance
  if (x > 0.) {
    v = t / (s + s);
    if (std::fabs(v) <= 0.25)
      q = q0 + 0.5 * t * t * ((((((a7 * v + a6) * v + a5) * v + a4) * v + a3) * v + a2) * v + a1) * v;
    else
      q = q0 - s * t + 0.25 * t * t + (s2 + s2) * std::log(1.0 + v);
    if (std::log(1.0 - u) <= q) return scale * ret_val;
  }
  for (;;) {  // Steps 8-11: double-exponential rejection
    const double e = sg_rrng_exp(g);
    u = sg_rrng_unif(g);
    u = u + u - 1.0;
    t = u < 0.0 ? b - si * e : b + si * e;
    if (t >= -0.71874483771719) {
      v = t / (s + s);
      if (std::fabs(v) <= 0.25)
        q = q0 + 0.5 * t * t * ((((((a7 * v + a6) * v + a5) * v + a4) * v + a3) * v + a2) * v + a1) * v;
      else
        q = q0 - s * t + 0.25 * t * t + (s2 + s2) * std::log(1.0 + v);
      if (q > 0.0) {
        const double w = std::expm1(q);
        if (c * std::fabs(u) <= w * std::exp(e - 0.5 * t * t)) break;
      }
    }
  }
  x = s + 0.5 * t;
  return scale * x * x;
}

static double rrng_norm_cb(void* u) { return sg_rrng_norm(static_cast<sg_rrng*>(u)); }
static double rrng_unif_cb(void* u) { return sg_rrng_unif(static_cast<sg_rrng*>(u)); }
static void rrng_unif_n_cb(void* u, double* out, int64_t n) { sg_rrng_unif_n(static_cast<sg_rrng*>(u), out, n); }
static double rrng_gamma_cb(void* u, double shape, double rate) {
  return sg_rrng_gamma(static_cast<sg_rrng*>(u), shape, 1.0 / rate);  // rgamma(n, shape, rate): scale = 1/rate
}

void sg_random_bind_rrng(sg_random* r, sg_rrng* g) {
  r->norm_cb = rrng_norm_cb;
  r->unif_cb = rrng_unif_cb;
  r->gamma_cb = rrng_gamma_cb;
  r->unif_n_cb = rrng_unif_n_cb;
  r->user = g;
}

}  // extern "C"
