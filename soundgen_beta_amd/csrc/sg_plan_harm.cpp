// sg_plan_harm.cpp — host planner for generateHarmonics() (R/source.R:173-471).
//
// The planner reproduces every data-independent step of the reference in
// fp64 (vibrato, glottal cycles, jitter/drift/random walks from injected
// draws, getRolloff, shimmer, getVocalFry, upsample) and the two
// data-dependent bookkeeping steps (zero-crossing trims of crossFade(), the
// output length) by evaluating the epoch waveform in fp64 only at the few
// samples the zero-crossing searches visit. The per-sample work — the sine
// bank, the crossfades, normalisation, fades, envelopes — runs on the GPU.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "sg_amp.h"
#include "sg_loess.h"
#include "sg_plan.h"
#include "sg_prof.h"

namespace sg {

// ------------------------------------------------------------- contours
bool smooth_contour(const sg_anchors& an, int64_t len, bool thisIsPitch, int method, bool has_floor,
                    double vfloor, bool has_ceil, double vceil, vec& out, double sr) {
  ProfScope ps(PF_CONTOUR);
  out.clear();
  if (an.n <= 0) return false;
  const int64_t n = an.n;
  if (n > 10 && method == 0) method = 1;
  vec t(an.time, an.time + n), v(an.value, an.value + n);
  if (has_floor) for (auto& x : v) if (x < vfloor) x = vfloor;
  if (has_ceil) for (auto& x : v) if (x > vceil) x = vceil;
  if (thisIsPitch) {
    for (auto& x : v) x = HzToSemitones(x);
    if (has_floor) vfloor = HzToSemitones(vfloor);
    if (has_ceil) vceil = HzToSemitones(vceil);
  }
  // len = NULL (len < 0, R/smoothContours.R:92-96): the times are durations in ms
  // and stay as they are (spline's x); len = floor(duration_ms * sr / 1000)
  const vec traw = t;
  const bool len_null = len < 0;
  double dur_ms = (double)len / sr * 1000;
  if (len_null) {
    dur_ms = r_max(t) - r_min(t);
    len = (int64_t)std::floor(dur_ms * sr / 1000);
    if (!(dur_ms != 0)) return false;
  }
  const double tmin = r_min(t);
  for (auto& x : t) x -= tmin;
  const double tmax = r_max(t);
  for (auto& x : t) x /= tmax;  // (the loess anchor points: the same bits either way)
  if (len <= 0) return false;
  if (n == 1) out.assign(len, v[0]);
  else if (n == 2) out = r_seq_len(v[0], v[1], len);
  else {
    if (method != 1) {  // loess, R/smoothContours.R:119-154 (duration_ms: len / sr * 1000, or the anchors' span)
      const LoessFit T = smooth_loess(t.data(), v.data(), n, len, dur_ms, has_floor, vfloor);
      out.resize(len);
      int leaf = -1;
      for (int64_t k = 0; k < len; ++k) {
        const double z = (double)(k + 1);
        out[k] = (z < T.xmin || z > T.xmax) ? NAN : T.eval_seq(z, leaf);
      }
    } else {
      out = r_spline(len_null ? traw : t, v, len);
    }
    for (auto& x : out) {
      if (has_floor && x < vfloor) x = vfloor;
      if (has_ceil && x > vceil) x = vceil;
    }
  }
  for (auto& x : out) if (std::isnan(x)) x = 0;
  if (thisIsPitch) for (auto& x : out) x = semitonesToHz(x);
  return true;
}

SgContour contour_desc(Batch& B, const sg_anchors& an, int64_t L, bool has_floor, double vfloor,
                       bool has_ceil, double vceil, bool db, double sr) {
  SgContour c{};
  c.lo = -INFINITY; c.hi = INFINITY; c.db = db ? 1 : 0;
  c.L = L;
  if (an.n <= 0 || L <= 0) { c.kind = 0; return c; }
  const int64_t n = an.n;
  vec t(an.time, an.time + n), v(an.value, an.value + n);
  if (has_floor) for (auto& x : v) if (x < vfloor) x = vfloor;
  if (has_ceil) for (auto& x : v) if (x > vceil) x = vceil;
  if (n == 1) { c.kind = 1; c.a = v[0]; return c; }
  if (n == 2) {
    c.kind = 2; c.a = v[0]; c.b = v[1];
    c.by = L > 1 ? (c.b - c.a) / (double)(L - 1) : 0.0;
    return c;
  }
  const double tmin = r_min(t);
  for (auto& x : t) x -= tmin;
  const double tmax = r_max(t);
  for (auto& x : t) x /= tmax;
  if (n <= 10) {
    // loess: evaluated at u = 1..L; the Hermite pieces between consecutive
    // k-d tree vertices become power-basis cubics in dx = u - vertex
    const LoessFit T = smooth_loess(t.data(), v.data(), n, L, (double)L / sr * 1000, has_floor, vfloor);
    std::vector<int> ord(T.vx.size());
    for (size_t i = 0; i < ord.size(); ++i) ord[i] = (int)i;
    std::sort(ord.begin(), ord.end(), [&](int a, int b) { return T.vx[a] < T.vx[b]; });
    const size_t nk = ord.size();
    vec kx(nk), ky(nk), kb(nk), kc(nk, 0.0), kd(nk, 0.0);
    for (size_t i = 0; i < nk; ++i) {
      kx[i] = T.vx[ord[i]];
      ky[i] = T.val[ord[i]];
      kb[i] = T.slope[ord[i]];
    }
    for (size_t i = 0; i + 1 < nk; ++i) {
      const double h = kx[i + 1] - kx[i], dy = ky[i + 1] - ky[i];
      kc[i] = (3 * dy / h - 2 * kb[i] - kb[i + 1]) / h;
      kd[i] = (-2 * dy / h + kb[i] + kb[i + 1]) / (h * h);
    }
    c.kind = 3; c.nk = (int32_t)nk; c.k_off = (int64_t)B.cknots.size();
    c.a = 1; c.b = (double)L;
    c.by = L > 1 ? (c.b - c.a) / (double)(L - 1) : 0.0;
    if (has_floor) c.lo = vfloor;
    if (has_ceil) c.hi = vceil;
    for (const vec* a : {&kx, &ky, &kb, &kc, &kd}) B.cknots.insert(B.cknots.end(), a->begin(), a->end());
    return c;
  }
  Spline s = fmm_spline(t, v);
  c.kind = 3; c.nk = (int32_t)n; c.k_off = (int64_t)B.cknots.size();
  c.a = t.front(); c.b = t.back();
  c.by = L > 1 ? (c.b - c.a) / (double)(L - 1) : 0.0;
  if (has_floor) c.lo = vfloor;
  if (has_ceil) c.hi = vceil;
  for (const vec* a : {&s.x, &s.y, &s.b, &s.c, &s.d}) B.cknots.insert(B.cknots.end(), a->begin(), a->end());
  return c;
}

// host evaluation of a device contour (used for the fused-max bookkeeping tests)
static double contour_eval(const Batch& B, const SgContour& c, int64_t L, int64_t k) {
  double v;
  switch (c.kind) {
    case 0: return 1.0;
    case 1: v = c.a; break;
    case 2: {
      if (k == 0 || c.a == c.b) v = c.a;
      else if (k == L - 1) v = c.b;
      else v = c.a + (double)k * ((c.b - c.a) / (double)(L - 1));
      break;
    }
    default: {
      const double* x = &B.cknots[c.k_off];
      const double* y = x + c.nk; const double* b = y + c.nk; const double* cc = b + c.nk; const double* d = cc + c.nk;
      const double u = r_seqint_at(c.a, c.b, L, k);
      int64_t i = 0, j = c.nk;
      do { int64_t m = (i + j) / 2; if (u < x[m]) j = m; else i = m; } while (j > i + 1);
      const double dx = u - x[i];
      v = y[i] + dx * (b[i] + dx * (cc[i] + dx * d[i]));
      if (v < c.lo) v = c.lo;
      if (v > c.hi) v = c.hi;
    }
  }
  return c.db ? std::pow(2.0, v / 10) : v;
}

// ------------------------------------------------------ random walks
static void zero_one(vec& x) {
  const double mn = r_min(x);
  for (auto& v : x) v -= mn;
  const double mx = r_max(x);
  for (auto& v : x) v /= mx;
}

// getRandomWalk(), R/utilities_math.R:289-326 (method: 0 linear, 1 spline)
vec get_random_walk(Rng& R, int64_t len, double rw_range, double rw_smoothing, int method,
                    const vec& trend_in, bool trend_lazy_rnorm, bool draws_only) {
  if (len < 2) return vec{R.rgamma(1.0 / (rw_range * rw_range), 1.0 / (rw_range * rw_range))};
  vec trend = trend_in;
  if (trend_lazy_rnorm) trend = vec{R.rnorm(0, 1)};
  const double p = std::pow(2.0, 1.0 / rw_smoothing);
  double nd = std::floor(p > 2 ? p : 2);
  vec tshort;
  if (trend.size() > 1) {
    nd = r_round(nd / 2) * 2;
    const int64_t each = (int64_t)(nd / (double)trend.size());
    for (double tv : trend) for (int64_t e = 0; e < each; ++e) tshort.push_back(tv);
  } else tshort = trend;
  if (draws_only) {  // the same draws, no walk (a planning pass that only consumes draws)
    const int64_t cnt = nd > (double)len ? len : (int64_t)nd;
    for (int64_t i = 0; i < cnt; ++i) (void)R.rnorm(tshort[i % tshort.size()], 1.0);
    return vec{};
  }
  vec rw_long;
  if (nd > (double)len) {
    vec z(len);
    for (int64_t i = 0; i < len; ++i) z[i] = R.rnorm(tshort[i % tshort.size()], 1.0);
    rw_long = r_cumsum(z);
  } else {
    const int64_t n = (int64_t)nd;
    vec z(n);
    for (int64_t i = 0; i < n; ++i) z[i] = R.rnorm(tshort[i % tshort.size()], 1.0);
    vec rs = r_cumsum(z), xs(n);
    for (int64_t i = 0; i < n; ++i) xs[i] = (double)(i + 1);
    rw_long = method == 0 ? r_approx_n(xs, rs, len) : r_spline(xs, rs, len);
  }
  const double mn = r_min(rw_long);
  for (auto& v : rw_long) v -= mn;
  double mx = 0;
  for (double v : rw_long) { double a = std::fabs(v); if (a > mx || std::isnan(a)) mx = a; }
  for (auto& v : rw_long) v = v / mx * rw_range;
  return rw_long;
}

// clumper(), R/utilities_math.R:555-600
void clumper(vec& s, const vec& minLen_in) {
  const int64_t n = (int64_t)s.size();
  if (r_max(minLen_in) < 2) return;
  vec ml(minLen_in.size());
  for (size_t i = 0; i < ml.size(); ++i) ml[i] = r_round(minLen_in[i]);
  bool uniq2 = false;
  for (int64_t i = 1; i < n && !uniq2; ++i) if (s[i] != s[0]) uniq2 = true;
  if (!uniq2 || (ml.size() == 1 && (double)n < ml[0]) || (double)n < ml[0]) {
    vec tmp = s; std::sort(tmp.begin(), tmp.end());
    const double med = (n % 2) ? tmp[n / 2] : (tmp[n / 2 - 1] + tmp[n / 2]) / 2.0;
    for (auto& v : s) v = r_round(med);
    return;
  }
  if (ml.size() == 1 || (int64_t)ml.size() != n) {
    vec m2(n);
    for (int64_t i = 0; i < n; ++i) m2[i] = ml[i % ml.size()];
    ml = m2;
  }
  double c = 0;
  for (int64_t i = 1; i < n; ++i) {
    if (s[i - 1] == s[i]) c = c + 1;
    else if (c < ml[i]) { s[i] = s[i - 1]; c = c + 1; }
    else c = 1;
  }
  const double mlast = ml[n - 1];
  int64_t lo = (int64_t)((double)n - mlast + 1);
  if (lo < 2) lo = 2;
  int64_t cnt = 0;
  for (int64_t k = lo; k <= n; ++k) if (s[k - 1] == s[n - 1]) cnt++;
  if ((double)cnt < mlast) {
    const int64_t nidx = n - lo + 1;
    std::vector<int64_t> idx(nidx);
    for (int64_t k = 0; k < nidx; ++k) idx[k] = n - k;
    double cc = 1; int64_t ii = 2;
    while (ii <= nidx && s[idx[ii - 1] - 1] == s[idx[ii - 1] - 2] && ii < nidx) { cc++; ii++; }
    if (cc < mlast) { const double v = s[lo - 1]; for (int64_t k = 0; k < nidx; ++k) s[idx[k] - 1] = v; }
  }
}

// ------------------------------------------------------------- rolloff
// rowSums() of a column-major nrow x ncol matrix with R's long double
// accumulator, each row summed in column order; four rows per pass so that a
// column's reads share cache lines and the accumulators stay in registers.
static void row_sums(const double* M, int64_t nrow, int64_t ncol, std::vector<long double>& out) {
  out.assign((size_t)nrow, 0.0L);
  int64_t i = 0;
  for (; i + 4 <= nrow; i += 4) {
    long double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    for (int64_t g = 0; g < ncol; ++g) {
      const double* c = M + g * nrow + i;
      s0 += c[0]; s1 += c[1]; s2 += c[2]; s3 += c[3];
    }
    out[i] = s0; out[i + 1] = s1; out[i + 2] = s2; out[i + 3] = s3;
  }
  for (; i < nrow; ++i) {
    long double s = 0;
    for (int64_t g = 0; g < ncol; ++g) s += M[g * nrow + i];
    out[i] = s;
  }
}

// getRolloff(), R/sourceSpectrum.R:71-186 with per-gc vector parameters.
// Returns H x nGC column-major (kept rows compacted, renumbered 1..H).
vec get_rolloff(const vec& pitch, int64_t nH, const vec& rolloff, const vec& rolloffOct, double rolloffParab,
                double rolloffParabHarm, const vec& rolloffKHz, double baseline, double throwaway, double sr,
                int64_t& H, double rolloffParabCeiling) {
  ProfScope ps(PF_ROLLOFF);
  const int64_t nGC = (int64_t)pitch.size();
  if (nH < 1) throw SgError(SG_E_DOMAIN, "getRolloff: nHarmonics < 1");
  vec r(nH * nGC);
  auto at = [&](int64_t h, int64_t g) -> double& { return r[g * nH + h]; };
  bool anyOct = false;
  for (double v : rolloffOct) if (v != 0) anyOct = true;
  vec slope(nGC);
  for (int64_t g = 0; g < nGC; ++g) slope[g] = rolloff[g] + rolloffKHz[g] * (pitch[g] - baseline) / 1000;
  vec lg(nH);  // log2(h), once per call instead of per (gc, harmonic)
  for (int64_t h = 0; h < nH; ++h) lg[h] = std::log2((double)(h + 1));
  for (int64_t g = 0; g < nGC; ++g) {
    double* col = &r[g * nH];
    for (int64_t h = 0; h < nH; ++h) {
      const double hh = (double)(h + 1);
      if (hh * pitch[g] >= sr / 2) {  // above Nyquist: -Inf for this and every higher row
        for (int64_t k = h; k < nH; ++k) col[k] = -INFINITY;
        break;
      }
      const double delta = (anyOct && h >= 1) ? rolloffOct[g] * (pitch[g] * hh - baseline) / 1000 : 0.0;
      col[h] = (slope[g] * lg[h]) + delta;
    }
  }
  if (rolloffParab != 0) {
    for (int64_t g = 0; g < nGC; ++g) {
      // harmonics affected: round(rolloffParabCeiling / pitch_per_gc) per column when
      // a ceiling is given, else round(rolloffParabHarm); 2 becomes 3 (boosts H1)
      double rph = std::isnan(rolloffParabCeiling) ? r_round(rolloffParabHarm) : r_round(rolloffParabCeiling / pitch[g]);
      if (rph == 2) rph = 3;
      const double a = -4 * rolloffParab / ((rph - 1) * (rph - 1));
      const double b = -a * (1 + rph), c = a * rph;
      if (rph < 3) { if (rph < 2) at(0, g) = at(0, g) + rolloffParab; }
      else {
        if (rph > nH) throw SgError(SG_E_DOMAIN, "getRolloff: subscript out of bounds (rolloffParabHarm > nHarmonics)");
        for (int64_t k = 1; k <= (int64_t)rph; ++k) at(k - 1, g) = at(k - 1, g) + a * k * k + b * k + c;
      }
    }
  }
  for (auto& v : r) if (v < throwaway) v = -INFINITY;
  for (int64_t g = 0; g < nGC; ++g) {
    double mx = -INFINITY;
    for (int64_t h = 0; h < nH; ++h) if (at(h, g) > mx) mx = at(h, g);
    for (int64_t h = 0; h < nH; ++h) at(h, g) = at(h, g) - mx;
  }
  for (auto& v : r) v = v == -INFINITY ? 0.0 : std::pow(2.0, v / 10);
  std::vector<int64_t> keep;
  std::vector<long double> rs;
  row_sums(r.data(), nH, nGC, rs);
  for (int64_t h = 0; h < nH; ++h)
    if ((double)rs[h] > 0) keep.push_back(h);
  H = (int64_t)keep.size();
  vec o(H * nGC);
  for (int64_t g = 0; g < nGC; ++g)
    for (int64_t k = 0; k < H; ++k) o[g * H + k] = at(keep[k], g);
  return o;
}

// ---------------------------------------------------------- vocal fry
// A syllable's amplitude parameters for the device build (sg_amp.h): one
// SgAmpCol per glottal cycle, the shared constants in a job template.
struct AmpSpec {
  std::vector<SgAmpCol> cols;
  SgAmpJob J{};
  vec lg;          // log2(h + 1), as getRolloff and the device table (elog2) hold it
  vec lsh;         // log2 of each cycle's shimmer factor (0 without shimmer)
};

struct EpochMat {
  int64_t g0, g1;     // 0-based gc range (inclusive)
  int64_t D;          // nSubharm + 1
  int64_t R;          // max rank
  vec A;              // host-built: [G][R] by rank, fp64 (zero rows for dropped ranks)
  vec mult;           // [R]: R's times_f0 for ranks present (0 if absent)
  // device-built (spec set): columns computed here only where the host needs
  // values (zero-crossing searches), by the formula sg_amp_build runs
  const AmpSpec* spec = nullptr;
  SgAmpJob job{};
  mutable std::vector<vec> cache;
  // per column: rows up to the last nonzero A (lnz); eq[g]: column g + 1 equals column g
  std::vector<int32_t> lnz;
  std::vector<char> eq;
  const double* col(int64_t g) const {
    if (!spec) return A.data() + g * R;
    if (cache.empty()) cache.resize((size_t)(g1 - g0 + 1));
    vec& c = cache[(size_t)g];
    if ((int64_t)c.size() != R) {
      c.resize((size_t)R);
      for (int64_t r = 0; r < R; ++r) c[r] = amp_value(spec->cols.data(), job, spec->lg.data(), (int)g, (int)r);
    }
    return c.data();
  }
  // lnz / eq of a host-built matrix from its fp32 values (what the device reads)
  void float_pattern() {
    const int64_t G = g1 - g0 + 1;
    lnz.assign((size_t)G, 0);
    eq.assign((size_t)G, 0);
    for (int64_t g = 0; g < G; ++g) {
      int32_t l = 0;
      for (int64_t r = 0; r < R; ++r) if ((float)A[g * R + r] != 0.0f) l = (int32_t)(r + 1);
      lnz[g] = l;
      if (g + 1 < G) {
        bool e = true;
        for (int64_t r = 0; r < R && e; ++r) e = (float)A[g * R + r] == (float)A[(g + 1) * R + r];
        eq[g] = e;
      }
    }
  }
};

static double rowname_num(double x) {
  char buf[64];
  snprintf(buf, sizeof buf, "%.15g", x);
  return strtod(buf, nullptr);
}

// getVocalFry_per_epoch(), R/subharmonics.R:25-86
static EpochMat fry_per_epoch(const double* roll, int64_t H, int64_t g0, int64_t g1, const vec& pitch, int64_t nSub,
                              const vec& sbw, double throwaway01) {
  EpochMat m;
  m.g0 = g0; m.g1 = g1;
  const int64_t ncol = g1 - g0 + 1;
  if (nSub < 1) {
    m.D = 1; m.R = H; m.A.assign(roll + g0 * H, roll + (g1 + 1) * H);
    m.mult.resize(H);
    for (int64_t h = 0; h < H; ++h) m.mult[h] = (double)(h + 1);
    return m;
  }
  vec gseq = r_seq_by(0, (double)(H + 1), 1.0 / (double)(nSub + 1));
  const int64_t nr = (int64_t)gseq.size();
  vec rn(nr * ncol, NAN);
  auto RN = [&](int64_t i, int64_t g) -> double& { return rn[g * nr + i]; };
  for (int64_t g = 0; g < ncol; ++g) { RN(0, g) = 0; RN(nr - 1, g) = 0; }
  char a[64], b[64];
  for (int64_t h = 0; h < H; ++h) {  // match(rownames(rolloff), rownames(rolloff_new))
    // rownames are 15-significant-digit strings: harmonic h + 1 can only match
    // gseq[(h + 1) (nSub + 1)] (within an ulp of h + 1; every other entry is at
    // least 1 / (nSub + 1) away). Confirm that one string, else search all.
    int64_t hit = -1;
    const int64_t i0 = (h + 1) * (nSub + 1);
    snprintf(a, sizeof a, "%.15g", (double)(h + 1));
    if (i0 < nr) {
      snprintf(b, sizeof b, "%.15g", gseq[i0]);
      if (!strcmp(a, b)) hit = i0;
    }
    for (int64_t i = 0; hit < 0 && i < nr; ++i) {
      snprintf(b, sizeof b, "%.15g", gseq[i]);
      if (!strcmp(a, b)) hit = i;
    }
    if (hit >= 0)
      for (int64_t g = 0; g < ncol; ++g) RN(hit, g) = roll[(g0 + g) * H + h];
  }
  vec ml(nSub * ncol);
  for (int64_t s = 1; s <= nSub; ++s)
    for (int64_t g = 0; g < ncol; ++g) {
      const double d = pitch[g0 + g] * (double)s / (double)(nSub + 1), sd = sbw[g0 + g];
      ml[(s - 1) * ncol + g] = (sd == 0) ? (d == 0 ? NAN : 0.0) : std::exp(-0.5 * (d / sd) * (d / sd));
    }
  for (int64_t block = 1; block <= H + 1; ++block) {
    const int64_t row_lwr = 1 + (block - 1) * (nSub + 1), row_upr = row_lwr + nSub + 1;
    const double Alin = rn[row_lwr - 1], Blin = rn[row_upr - 1];  // linear index = column 1 (quirk)
    for (int64_t g = 0; g < ncol; ++g)  // column-major writes (each element written once)
      for (int64_t gg = 1; gg <= nSub; ++gg)
        RN(row_lwr + gg - 1, g) = Alin * ml[(gg - 1) * ncol + g] + Blin * ml[(nSub - gg) * ncol + g];
  }
  for (auto& v : rn) if (v < throwaway01) v = 0;
  std::vector<int64_t> keep;
  std::vector<long double> rs;
  row_sums(rn.data(), nr, ncol, rs);
  for (int64_t i = 0; i < nr; ++i)
    if ((double)rs[i] > 0) keep.push_back(i);
  m.D = nSub + 1;
  m.R = keep.empty() ? 0 : keep.back();
  m.A.assign(ncol * std::max<int64_t>(m.R, 1), 0.0);
  m.mult.assign(std::max<int64_t>(m.R, 1), 0.0);
  // rank i (0 never survives: row 1 is all zero)
  for (int64_t i : keep) m.mult[i - 1] = rowname_num(gseq[i]);
  for (int64_t g = 0; g < ncol; ++g)
    for (int64_t i : keep) m.A[g * m.R + (i - 1)] = RN(i, g);
  return m;
}

// getVocalFry()'s epochs: runs of glottal cycles with one number of
// subharmonics (clumped to shortestEpoch), [g0, g1] inclusive
//   R/subharmonics.R:108-163
struct FryEpoch { int64_t g0, g1, nsub; };
static std::vector<FryEpoch> fry_epochs(const vec& pitch, const vec& subFreq, double shortestEpoch) {
  const int64_t nGC = (int64_t)pitch.size();
  vec nsub(nGC);
  double mx = -INFINITY;
  for (int64_t g = 0; g < nGC; ++g) {
    double v = r_round(pitch[g] / subFreq[g]) - 1;
    if (v < 0) v = 0;
    nsub[g] = v; mx = std::max(mx, v);
  }
  if (mx < 1) return {FryEpoch{0, nGC - 1, 0}};
  vec minlen(nGC);
  for (int64_t g = 0; g < nGC; ++g) minlen[g] = r_round(shortestEpoch / (1000 / pitch[g]));
  if (nGC > 1) clumper(nsub, minlen);
  std::vector<FryEpoch> out;
  int64_t s0 = 0;
  for (int64_t g = 1; g <= nGC; ++g) {
    if (g == nGC || nsub[g] != nsub[g - 1]) {
      out.push_back(FryEpoch{s0, g - 1, (int64_t)nsub[g - 1]});
      s0 = g;
    }
  }
  return out;
}

// getVocalFry(), R/subharmonics.R:108-163
static std::vector<EpochMat> get_vocal_fry(const vec& roll, int64_t H, const vec& pitch, const vec& subFreq,
                                           const vec& subDep, double throwaway, double shortestEpoch) {
  const std::vector<FryEpoch> eps = fry_epochs(pitch, subFreq, shortestEpoch);
  const double throwaway01 = eps.size() == 1 && eps[0].nsub == 0 ? 0.0 : std::pow(2.0, throwaway / 10);
  std::vector<EpochMat> out;
  for (const FryEpoch& e : eps) out.push_back(fry_per_epoch(roll.data(), H, e.g0, e.g1, pitch, e.nsub, subDep, throwaway01));
  return out;
}

// ------------------------------------------- device-built amplitude matrices
// getRolloff() without the matrix: per cycle its parameters and column max,
// the kept rows H, each column's last finite row (lf, 1-based). The device
// builds the values (sg_amp_build). false -> the host-built path: kept rows
// that are not 0..H-1 (R renumbers them), a column without a finite value, or
// a dynamic range whose powers could underflow.
//   R/sourceSpectrum.R:71-186 (rolloffParabCeiling NA, as generateHarmonics calls it)
static bool rolloff_spec(const vec& pitch, int64_t nH, const vec& rolloff, const vec& rolloffOct, double rolloffParab,
                         double rolloffParabHarm, const vec& rolloffKHz, double baseline, double throwaway, double sr,
                         AmpSpec& S, int64_t& H, std::vector<int32_t>& lf) {
  ProfScope ps(PF_ROLLOFF);
  const int64_t nGC = (int64_t)pitch.size();
  if (nH < 1) throw SgError(SG_E_DOMAIN, "getRolloff: nHarmonics < 1");
  bool anyOct = false;
  for (double v : rolloffOct) if (v != 0) anyOct = true;
  S.lg.resize((size_t)nH);
  for (int64_t h = 0; h < nH; ++h) S.lg[h] = std::log2((double)(h + 1));
  SgAmpJob& J = S.J;
  J = SgAmpJob{};
  J.thr = throwaway;
  J.nyq = sr / 2;
  J.parab = rolloffParab;
  J.t01 = std::pow(2.0, throwaway / 10);
  J.baseline = baseline;
  J.any_oct = anyOct;
  double rph = r_round(rolloffParabHarm), a = 0, b = 0, c = 0;
  if (rph == 2) rph = 3;
  if (rolloffParab != 0) {
    a = -4 * rolloffParab / ((rph - 1) * (rph - 1));
    b = -a * (1 + rph);
    c = a * rph;
    if (rph >= 3 && rph > nH && nGC > 0)
      throw SgError(SG_E_DOMAIN, "getRolloff: subscript out of bounds (rolloffParabHarm > nHarmonics)");
  }
  S.cols.resize((size_t)nGC);
  std::vector<char> kept((size_t)nH, 0);
  lf.assign((size_t)nGC, 0);
  double vmin = INFINITY;
  for (int64_t g = 0; g < nGC; ++g) {
    SgAmpCol& P = S.cols[g];
    P = SgAmpCol{};
    P.pitch = pitch[g];
    P.slope = rolloff[g] + rolloffKHz[g] * (pitch[g] - baseline) / 1000;
    P.oct = rolloffOct[g];
    P.sh = 1;
    P.rph = rph;
    P.pa = a; P.pb = b; P.pc = c;
    double mx = -INFINITY, v;
    int32_t last = 0;
    for (int64_t h = 0; h < nH; ++h) {
      if ((double)(h + 1) * P.pitch >= J.nyq) break;  // -Inf from here up
      if (!roll_db(P, J, S.lg.data(), (int)h, &v)) continue;
      kept[h] = 1;
      last = (int32_t)(h + 1);
      if (v > mx) mx = v;
      if (v < vmin) vmin = v;
    }
    if (mx == -INFINITY) return false;
    P.mx = mx;
    lf[g] = last;
    if (mx - vmin > 9000) return false;  // 2^(-900) and below: keep R's underflow decisions on the host
  }
  H = 0;
  while (H < nH && kept[H]) ++H;
  for (int64_t h = H; h < nH; ++h) if (kept[h]) return false;
  return H > 0;
}

// a plain epoch (no subharmonics): the kept rolloff rows as they are
static void plain_spec(const AmpSpec& S, int64_t H, int64_t g0, int64_t g1, const std::vector<int32_t>& lf,
                       EpochMat& m) {
  const int64_t ncol = g1 - g0 + 1;
  m.g0 = g0; m.g1 = g1; m.D = 1; m.R = H;
  m.mult.resize((size_t)H);
  for (int64_t h = 0; h < H; ++h) m.mult[h] = (double)(h + 1);
  m.spec = &S;
  m.job = S.J;
  m.job.g0 = (int32_t)g0; m.job.G = (int32_t)ncol; m.job.H = (int32_t)H; m.job.nsub = 0; m.job.R = (int32_t)H;
  m.lnz.assign(lf.begin() + g0, lf.begin() + g1 + 1);
  m.eq.assign((size_t)ncol, 0);
  for (int64_t g = 0; g + 1 < ncol; ++g)
    m.eq[g] = std::memcmp(&S.cols[g0 + g], &S.cols[g0 + g + 1], sizeof(SgAmpCol)) == 0;
}

// getVocalFry_per_epoch()'s kept ranks, multipliers and per-cycle nonzero rows
// without the matrix. Harmonic rows are decided in the log domain (exponent
// against throwaway / 10), sidebands from exact end points and weights. false
// -> host path: a value within rounding of the threshold, where the device's
// pow / exp might decide the other way.   R/subharmonics.R:25-86
static bool fry_spec(const AmpSpec& S, int64_t H, int64_t g0, int64_t g1, int64_t nSub, const std::vector<int32_t>& lf,
                     EpochMat& m) {
  const int64_t D = nSub + 1, ncol = g1 - g0 + 1;
  const vec gseq = r_seq_by(0, (double)(H + 1), 1.0 / (double)D);
  const int64_t nr = (int64_t)gseq.size();
  if (nr != (H + 1) * D + 1) return false;
  for (int64_t h = 0; h < H; ++h)  // rownames match at row (h + 1) D (15 significant digits)
    if (std::fabs(gseq[(h + 1) * D] - (double)(h + 1)) > 1e-13 * (double)(h + 1)) return false;
  SgAmpJob J = S.J;
  J.g0 = (int32_t)g0; J.G = (int32_t)ncol; J.H = (int32_t)H; J.nsub = (int32_t)nSub;
  const double* lg = S.lg.data();
  vec r0((size_t)H);
  for (int64_t h = 0; h < H; ++h) r0[h] = roll_value(S.cols[g0], J, lg, (int)h);
  vec ml((size_t)(nSub * ncol));
  for (int64_t q = 1; q <= nSub; ++q)
    for (int64_t g = 0; g < ncol; ++g) ml[(q - 1) * ncol + g] = fry_ml(S.cols[g0 + g], J, (int)q);
  const double thr10 = J.thr / 10;
  // element (i, g) nonzero? 0 / 1, or -1: too close to the threshold to decide for the device
  auto nz_at = [&](int64_t i, int64_t g) -> int {
    if (i % D == 0) {
      const int64_t h = i / D - 1;
      double v;
      if (h >= H || !roll_db(S.cols[g0 + g], J, lg, (int)h, &v)) return 0;
      const double y = (v - S.cols[g0 + g].mx) / 10 + (S.lsh.empty() ? 0.0 : S.lsh[g0 + g]);
      if (y > thr10 + 1e-9) return 1;
      if (y < thr10 - 1e-9) return 0;
      return -1;
    }
    const int64_t block = i / D + 1, gg = i % D;
    const double a = block >= 2 ? r0[block - 2] : 0.0, b = block - 1 < H ? r0[block - 1] : 0.0;
    const double val = a * ml[(gg - 1) * ncol + g] + b * ml[(nSub - gg) * ncol + g];
    if (std::isnan(val) || std::fabs(val - J.t01) <= 1e-12 * J.t01) return -1;
    return val >= J.t01 ? 1 : 0;
  };
  // bounds that decide whole rows at once: harmonic rows at or above every
  // cycle's last finite rolloff row, sideband rows whose end points times the
  // largest weights stay clearly under the threshold
  int64_t hmax = 0;
  for (int64_t g = 0; g < ncol; ++g) hmax = std::max<int64_t>(hmax, lf[g0 + g]);
  vec mlmax((size_t)nSub, 0.0);
  for (int64_t q = 0; q < nSub; ++q)
    for (int64_t g = 0; g < ncol; ++g) mlmax[q] = std::max(mlmax[q], ml[q * ncol + g]);
  auto row_zero = [&](int64_t i) -> bool {
    if (i % D == 0) return i / D - 1 >= std::min<int64_t>(H, hmax);
    const int64_t block = i / D + 1, gg = i % D;
    const double a = block >= 2 ? r0[block - 2] : 0.0, b = block - 1 < H ? r0[block - 1] : 0.0;
    return a * mlmax[gg - 1] + b * mlmax[nSub - gg] < J.t01 * (1 - 1e-9);
  };
  // per cycle: the last nonzero rank (scan down from the top possible row)
  m.lnz.assign((size_t)ncol, 0);
  const int64_t itop = std::min<int64_t>(nr - 1, (std::min<int64_t>(H, hmax) + 1) * D);
  for (int64_t g = 0; g < ncol; ++g)
    for (int64_t i = itop; i > 0; --i) {
      if (row_zero(i)) continue;
      const int z = nz_at(i, g);
      if (z < 0) return false;
      if (z) { m.lnz[g] = (int32_t)i; break; }
    }
  // kept rows (rowSums > 0): any cycle nonzero
  std::vector<char> keep((size_t)nr, 0);
  for (int64_t i = 1; i <= itop; ++i) {
    if (row_zero(i)) continue;
    for (int64_t g = 0; g < ncol; ++g) {
      const int z = nz_at(i, g);
      if (z < 0) return false;
      if (z) { keep[i] = 1; break; }
    }
  }
  int64_t R = 0;
  for (int64_t i = nr - 1; i > 0 && !R; --i) if (keep[i]) R = i;
  m.g0 = g0; m.g1 = g1; m.D = D; m.R = R;
  m.mult.assign((size_t)std::max<int64_t>(R, 1), 0.0);
  for (int64_t i = 1; i <= R; ++i) if (keep[i]) m.mult[i - 1] = rowname_num(gseq[i]);
  m.spec = &S;
  m.job = J;
  m.job.R = (int32_t)R;
  m.eq.assign((size_t)ncol, 0);
  for (int64_t g = 0; g + 1 < ncol; ++g)
    m.eq[g] = std::memcmp(&S.cols[g0 + g], &S.cols[g0 + g + 1], sizeof(SgAmpCol)) == 0;
  return true;
}

// 1: every call takes the host-built path (tests compare the two); default
// 0, changed by sg_set_amp_policy
static std::atomic<int> g_amp_host{-1};
static bool amp_device_enabled() {
  int h = g_amp_host.load();
  if (h < 0) {
    h = 0;  // sg_set_amp_policy(1) forces the host-built matrices (tests)
    g_amp_host.store(h);
  }
  return h == 0;
}

// ---------------------------------------------------- host evaluator
// cubic piece of the upsampled pitch (host fp64 evaluator for the bookkeeping)
struct HSeg {
  double t0;
  double prefix;
  double y, b, c, d;
};

struct HostSyl {
  std::vector<HSeg> segs;
  double sr;
  double integr(int64_t u) const {  // cumsum(pitch_up)[u] / sr, u 1-based
    int64_t lo = 0, hi = (int64_t)segs.size() - 1;
    while (lo < hi) { int64_t m = (lo + hi + 1) / 2; if (segs[m].t0 < (double)u) lo = m; else hi = m - 1; }
    const HSeg& s = segs[lo];
    const double m = (double)u - s.t0;
    const double S1 = m * (m + 1) / 2, S2 = m * (m + 1) * (2 * m + 1) / 6, S3 = S1 * S1;
    return (s.prefix + s.y * m + s.b * S1 + s.c * S2 + s.d * S3) / sr;
  }
};

struct HostEpoch {
  const EpochMat* M;
  const HostSyl* S;
  int64_t u0, n, G;
  vec knots;
  // W(j) in fp64, same formula/row order as R/source.R:396-419
  double W(int64_t j) const {
    const double v = r_seqint_at(knots.front(), knots.back(), n, j);
    int64_t i = 0, jj = G - 1;
    while (i < jj - 1) { int64_t ij = (i + jj) / 2; if (v < knots[ij]) jj = ij; else i = ij; }
    const double t = (v - knots[i]) / (knots[jj] - knots[i]);
    const double integ = S->integr(u0 + j);
    const double *A0 = M->col(i), *A1 = M->col(jj);
    double acc = 0;
    for (int64_t r = 0; r < M->R; ++r) {
      if (M->mult[r] == 0) continue;
      const double y0 = A0[r], y1 = A1[r];
      double am;
      if (v == knots[jj]) am = y1;
      else if (v == knots[i]) am = y0;
      else am = y0 + (y1 - y0) * t;
      acc = acc + std::sin(2 * M_PI * integ * M->mult[r]) * am;
    }
    return acc;
  }
  // W(j) by Clenshaw's recurrence over rows r -> multiplier (r + 1) / D (one
  // sin/cos per sample instead of one sin per row). *err bounds |Wfast - W|:
  // the recurrence (~R^2 eps), and R's 15-digit multipliers (rowname
  // round trip) against (r + 1) / D, times the row amplitudes.
  double Wfast(int64_t j, double* err) const {
    double f;
    Wfast_n<1>(j, 1, &f, err);
    return f;
  }
  // Wfast of the n <= K samples j0 .. j0 + n - 1: per sample the same operations
  // in the same order, the K row recurrences interleaved (independent dependency
  // chains keep the FP pipes busy; one chain is latency-bound)
  template <int K>
  void Wfast_n(int64_t j0, int n, double* f, double* err) const {
    const double *A0[K], *A1[K];
    double t[K], c2[K], th[K], integ[K], b1[K], b2[K], sabs[K];
    int sel[K];  // 0: interpolate; 1: on knot jj (y1); 2: on knot i (y0)
    for (int l = 0; l < K; ++l) {
      const int64_t j = j0 + (l < n ? l : n - 1);
      const double v = r_seqint_at(knots.front(), knots.back(), this->n, j);
      int64_t i = 0, jj = G - 1;
      while (i < jj - 1) { int64_t ij = (i + jj) / 2; if (v < knots[ij]) jj = ij; else i = ij; }
      t[l] = (v - knots[i]) / (knots[jj] - knots[i]);
      integ[l] = S->integr(u0 + j);
      double x = integ[l] / (double)M->D;
      x -= std::rint(x);
      th[l] = 2 * M_PI * x;
      c2[l] = 2 * std::cos(th[l]);
      A0[l] = M->col(i);
      A1[l] = M->col(jj);
      sel[l] = v == knots[jj] ? 1 : (v == knots[i] ? 2 : 0);
      b1[l] = b2[l] = sabs[l] = 0;
    }
    for (int64_t r = M->R - 1; r >= 0; --r) {
      const bool zero = M->mult[r] == 0;
      for (int l = 0; l < K; ++l) {
        const double y0 = A0[l][r], y1 = A1[l][r];
        const double am = zero ? 0.0 : (sel[l] == 1 ? y1 : (sel[l] == 2 ? y0 : y0 + (y1 - y0) * t[l]));
        const double b = am + c2[l] * b1[l] - b2[l];
        b2[l] = b1[l];
        b1[l] = b;
        sabs[l] += std::fabs(am);
      }
    }
    const double Rr = (double)M->R;
    for (int l = 0; l < n; ++l) {
      err[l] = sabs[l] * (Rr * Rr * 1e-15 + 1e-14 * std::fabs(integ[l]) * Rr / (double)M->D) + 1e-300;
      f[l] = b1[l] * std::sin(th[l]);
    }
  }
  // sign-exact W for the zero-crossing search: the fast value where its error
  // bound cannot change the sign, else R's row-by-row sum
  double Wsign(int64_t j) const {
    if (!fast_ok) return W(j);
    double err;
    const double f = Wfast(j, &err);
    return std::fabs(f) > 1e3 * err ? f : W(j);
  }
  // Wsign of j0 .. j0 + n - 1 (n <= 4)
  void Wsign_n(int64_t j0, int n, double* out) const {
    if (!fast_ok) {
      for (int l = 0; l < n; ++l) out[l] = W(j0 + l);
      return;
    }
    double f[4], e[4];
    Wfast_n<4>(j0, n, f, e);
    for (int l = 0; l < n; ++l) out[l] = std::fabs(f[l]) > 1e3 * e[l] ? f[l] : W(j0 + l);
  }
  bool fast_ok = false;  // every present row's multiplier is (r + 1) / D
  void init_fast() {
    static const bool exact_only = std::getenv("SG_XFADE_EXACT") != nullptr;  // test knob: R's row sums only
    fast_ok = M->D >= 1 && !exact_only;
    for (int64_t r = 0; r < M->R && fast_ok; ++r)
      if (M->mult[r] != 0 && std::fabs(M->mult[r] * (double)M->D - (double)(r + 1)) > 1e-9) fast_ok = false;
  }
};

// --------------------------------------------------- crossFade chain
struct HTerm { int64_t e; int64_t j0; double w0, w1, w2; };
struct HPiece { int64_t start, len; std::vector<HTerm> t; };

struct Chain {
  std::vector<HPiece> P;
  const std::vector<HostEpoch>* E;
  int64_t L() const { return P.empty() ? 0 : P.back().start + P.back().len; }
  double at(int64_t k) const {  // 0-based
    int64_t lo = 0, hi = (int64_t)P.size() - 1;
    while (lo < hi) { int64_t m = (lo + hi + 1) / 2; if (P[m].start <= k) lo = m; else hi = m - 1; }
    const HPiece& p = P[lo];
    const double q = (double)(k - p.start);
    double v = 0;
    for (const HTerm& t : p.t) v += (t.w0 + q * (t.w1 + q * t.w2)) * (*E)[t.e].W(t.j0 + (k - p.start));
    return v;
  }
  // the same value where only its sign matters (zero-crossing search): fast
  // Clenshaw terms with an error bound, R's exact sum when the bound is close
  double sign_at(int64_t k) const {
    int64_t lo = 0, hi = (int64_t)P.size() - 1;
    while (lo < hi) { int64_t m = (lo + hi + 1) / 2; if (P[m].start <= k) lo = m; else hi = m - 1; }
    const HPiece& p = P[lo];
    const double q = (double)(k - p.start);
    double v = 0, err = 0;
    for (const HTerm& t : p.t) {
      const HostEpoch& ep = (*E)[t.e];
      if (!ep.fast_ok) return at(k);
      double e;
      const double w = t.w0 + q * (t.w1 + q * t.w2);
      v += w * ep.Wfast(t.j0 + (k - p.start), &e);
      err += std::fabs(w) * e;
    }
    return std::fabs(v) > 1e3 * (err + 1e-300) ? v : at(k);
  }
  // sign_at of k0 .. k0 + n - 1 (n <= 4): blocks of Wfast per term when the
  // samples share a piece, the same per-sample sums and decisions as sign_at
  void sign_at_n(int64_t k0, int n, double* out) const {
    int64_t lo = 0, hi = (int64_t)P.size() - 1;
    while (lo < hi) { int64_t m = (lo + hi + 1) / 2; if (P[m].start <= k0) lo = m; else hi = m - 1; }
    const HPiece& p = P[lo];
    bool block = k0 + n <= p.start + p.len;
    for (const HTerm& t : p.t) block = block && (*E)[t.e].fast_ok;
    if (!block) {
      for (int l = 0; l < n; ++l) out[l] = sign_at(k0 + l);
      return;
    }
    double v[4] = {0, 0, 0, 0}, err[4] = {0, 0, 0, 0}, f[4], e[4];
    for (const HTerm& t : p.t) {
      (*E)[t.e].Wfast_n<4>(t.j0 + (k0 - p.start), n, f, e);
      for (int l = 0; l < n; ++l) {
        const double q = (double)(k0 + l - p.start);
        const double w = t.w0 + q * (t.w1 + q * t.w2);
        v[l] += w * f[l];
        err[l] += std::fabs(w) * e[l];
      }
    }
    for (int l = 0; l < n; ++l) out[l] = std::fabs(v[l]) > 1e3 * (err[l] + 1e-300) ? v[l] : at(k0 + l);
  }
  void truncate(int64_t newL) {
    while (!P.empty() && P.back().start >= newL) P.pop_back();
    if (!P.empty() && P.back().start + P.back().len > newL) P.back().len = newL - P.back().start;
  }
};

// findZeroCrossing(), R/utilities_soundgen.R:255-295, 1-based, 0 = NA.
// ab(k0, n, out) evaluates the 0-based samples k0 .. k0 + n - 1 (n <= 4): the
// scans read them through a 4-sample block in their direction of travel
template <class FB>
static int64_t find_zero_crossing(FB&& ab, int64_t len, int64_t location) {
  if (len < 1 || location < 1 || location > len) return 0;
  if (len == 1 && location == 1) return location;
  double blk[4];
  int64_t b0 = 0, bn = 0;
  bool back = true;
  auto a = [&](int64_t k) {
    if (k < b0 || k >= b0 + bn) {
      b0 = back ? std::max<int64_t>(0, k - 3) : k;
      bn = back ? k - b0 + 1 : std::min<int64_t>(4, len - k);
      ab(b0, (int)bn, blk);
    }
    return blk[k - b0];
  };
  int64_t zl = 0, zr = 0, i = 0;
  if (location > 1) {
    i = location;
    double cur = a(i - 1);
    while (i > 1) {
      const double prev = a(i - 2);
      if (cur > 0 && prev < 0) { zl = i - 1; break; }
      cur = prev;
      i = i - 1;
    }
  }
  if (location < len) i = location;
  back = false;
  if (i < len - 1) {
    double cur = a(i - 1);
    while (i < (len - 1)) {
      const double nxt = a(i);
      if (nxt > 0 && cur < 0) { zr = i; break; }
      cur = nxt;
      i = i + 1;
    }
  }
  if (!zl && !zr) return 0;
  if (!zl) return zr;
  if (!zr) return zl;
  return (std::llabs(zl - location) <= std::llabs(zr - location)) ? zl : zr;
}

static HTerm rebase(const HTerm& t, double s) {  // weight polynomial shifted by s samples
  HTerm o = t;
  o.j0 = t.j0 + (int64_t)s;
  o.w0 = t.w0 + t.w1 * s + t.w2 * s * s;
  o.w1 = t.w1 + 2 * t.w2 * s;
  o.w2 = t.w2;
  return o;
}

// crossFade(A, W_e), R/utilities_soundgen.R:328-375
static void cross_fade(Chain& A, const HostEpoch& W, int64_t e, double sr, double crossLen) {
  const int64_t LA = A.L();
  const int64_t zc1 = find_zero_crossing([&](int64_t k0, int n, double* o) { A.sign_at_n(k0, n, o); }, LA, LA);
  if (zc1) {
    A.truncate(zc1);
    A.P.push_back(HPiece{zc1, 1, {}});
  }
  const int64_t zc2 = find_zero_crossing([&](int64_t j0, int n, double* o) { W.Wsign_n(j0, n, o); }, W.n, 1);
  const int64_t w0 = zc2;  // W' = W[zc2 ..] (0-based)
  const int64_t lenW = W.n - w0;
  const int64_t L1 = A.L();
  double cl = std::floor(crossLen * sr / 1000);
  if ((double)(L1 - 1) < cl) cl = (double)(L1 - 1);
  if ((double)(lenW - 1) < cl) cl = (double)(lenW - 1);
  if (cl < 2) {
    A.P.push_back(HPiece{L1, lenW, {HTerm{e, w0, 1, 0, 0}}});
    return;
  }
  const int64_t c = (int64_t)cl;
  const int64_t idx1 = L1 - c;
  const double by = 1.0 / (double)(c - 1);
  // split A's pieces over [idx1, L1) into crossfade sub-pieces
  std::vector<HPiece> tail;
  for (const HPiece& p : A.P) {
    const int64_t s = std::max(p.start, idx1), en = std::min(p.start + p.len, L1);
    if (s >= en) continue;
    HPiece np{s, en - s, {}};
    const double off = (double)(s - idx1);  // q_global at sub-piece start
    for (const HTerm& t : p.t) {
      HTerm r = rebase(t, (double)(s - p.start));
      // multiply by down(q) = 1 - (off + q) * by
      const double a0 = 1 - off * by, a1 = -by;
      if (r.w2 != 0 && a1 != 0) throw SgError(SG_E_UNSUPPORTED, "crossFade: nested crossfades deeper than 2");
      HTerm m = r;
      m.w0 = r.w0 * a0;
      m.w1 = r.w0 * a1 + r.w1 * a0;
      m.w2 = r.w1 * a1 + r.w2 * a0;
      np.t.push_back(m);
    }
    // + up(q) * W'[off + q]
    np.t.push_back(HTerm{e, w0 + (int64_t)off, off * by, by, 0});
    if ((int)np.t.size() > SG_MAX_TERMS) throw SgError(SG_E_UNSUPPORTED, "crossFade: too many overlapping terms");
    tail.push_back(np);
  }
  A.truncate(idx1);
  for (auto& p : tail) A.P.push_back(p);
  if (lenW - c > 0) A.P.push_back(HPiece{L1, lenW - c, {HTerm{e, w0 + c, 1, 0, 0}}});
}

// ----------------------------------------------------------- planner
// samples per sine-bank task
static constexpr int64_t task_max() { return SG_TASK_MAX; }

// segment b continues segment a's line: both linear, same slope, and b's
// offset equals a's line at b's start (to rounding)
static bool lin_continues(const SgSeg& a, const SgSeg& b) {
  if (a.c2 != 0 || a.c3 != 0 || a.c4 != 0 || b.c2 != 0 || b.c3 != 0 || b.c4 != 0 || a.c1 != b.c1) return false;
  const double at = a.c0 + a.c1 * (b.t0 - a.t0);
  return std::fabs(at - b.c0) <= 1e-12 * std::max(1.0, std::fabs(b.c0));
}

int64_t plan_harmonics(Batch& B, const double* pitch_in, int64_t len, const sg_harm_params& P,
                       const sg_anchors& amplAnchors, Rng& R, int64_t out_off, bool dry_run, bool to_fs,
                       int64_t* fs_off, std::vector<HarmProbe>* probes) {
  ProfScope ps(PF_HARM);
  const double sr = P.samplingRate;
  if (len < 2) throw SgError(SG_E_DOMAIN, "generateHarmonics: pitch contour too short");
  vec pitch(pitch_in, pitch_in + len);
  if (P.vibratoDep > 0)
    for (int64_t i = 0; i < len; ++i)
      pitch[i] *= std::pow(2.0, std::sin(2 * M_PI * (double)(i + 1) * P.vibratoFreq / P.pitchSamplingRate) * P.vibratoDep / 12);
  // getGlottalCycles()
  std::vector<int64_t> gc;
  for (double i = 1; i < (double)len;) {
    gc.push_back((int64_t)i);
    const double st = std::floor(P.pitchSamplingRate / pitch[(int64_t)i - 1]);
    i = i + (st > 2 ? st : 2);
  }
  const int64_t nGC = (int64_t)gc.size();
  vec ppg(nGC);
  for (int64_t g = 0; g < nGC; ++g) ppg[g] = pitch[gc[g] - 1];
  bool useAmpl = false;
  for (int i = 0; i < amplAnchors.n; ++i) if (amplAnchors.value[i] < -P.throwaway) useAmpl = true;
  vec rolloffAmpl(nGC, 0.0);
  if (useAmpl) {
    vec ac;
    smooth_contour(amplAnchors, nGC, false, 0, true, 0, true, -P.throwaway, ac, sr);
    for (int64_t g = 0; g < nGC; ++g) rolloffAmpl[g] = (ac[g] / std::fabs(P.throwaway) - 1) * P.rolloff_perAmpl;
  }
  vec rw(nGC, 1.0), vf_on(nGC, 1.0), jit_on(nGC, 1.0), drift;
  if (P.temperature > 0) {
    rw = get_random_walk(R, nGC, P.temperature, 0.3, 1, vec{P.randomWalk_trendStrength, -P.randomWalk_trendStrength}, false);
    vec r0100 = rw;
    zero_one(r0100);
    for (auto& v : r0100) v *= 100;
    vec rwbin(nGC, 0.0);
    if (P.nonlinBalance == 100) rwbin.assign(nGC, 2.0);
    else if (P.nonlinBalance != 0) {
      const double q1 = noise_threshold(1, P.nonlinBalance), q2 = noise_threshold(2, P.nonlinBalance);
      for (int64_t g = 0; g < nGC; ++g) { if (r0100[g] > q1) rwbin[g] = 1; if (r0100[g] > q2) rwbin[g] = 2; }
      vec ml(nGC);
      for (int64_t g = 0; g < nGC; ++g) ml[g] = std::ceil(P.shortestEpoch / 1000 * ppg[g]);
      clumper(rwbin, ml);
    }
    const double m = r_mean(rw);
    for (int64_t g = 0; g < nGC; ++g) { rw[g] = rw[g] - m + 1; vf_on[g] = rwbin[g] > 0; jit_on[g] = rwbin[g] == 2; }
  }
  if (P.jitterDep > 0 && P.nonlinBalance > 0) {
    vec idx{1.0};
    double i = 1;
    while (i < (double)nGC) {
      const double ratio = ppg[(int64_t)i - 1] * P.jitterLen / 1000;
      i = idx.back() + ratio;
      idx.push_back(i);
    }
    vec idx2;
    for (double v0 : idx) {
      const double v = r_round(v0);
      if (v > (double)nGC) continue;
      // unique(): idx is strictly increasing, so its rounded values are
      // non-decreasing and a repeat can only equal the last value kept
      if (idx2.empty() || idx2.back() != v) idx2.push_back(v);
    }
    vec jit(idx2.size());
    for (size_t k = 0; k < idx2.size(); ++k) {
      const double z = R.rnorm(0, P.jitterDep / 12);
      const int64_t q = (int64_t)idx2[k] - 1;
      jit[k] = std::pow(2.0, z * rw[q] * jit_on[q]);
    }
    vec jpg = idx2.size() == 1 ? vec(nGC, jit[0]) : r_spline(idx2, jit, nGC);
    for (int64_t g = 0; g < nGC; ++g) ppg[g] *= jpg[g];
  }
  if (P.temperature > 0) {
    const double rws = .9 - P.temperature * P.pitchDriftFreq - 1.2 / (1 + std::exp(-.008 * ((double)nGC - 10))) + .6;
    const double rwr = P.temperature * P.pitchDriftDep + (double)nGC / 1000 / 12;
    drift = get_random_walk(R, nGC, rwr, rws, 1, vec{0.0}, false);
    const double m = r_mean(drift);
    for (int64_t g = 0; g < nGC; ++g) { drift[g] = std::pow(2.0, drift[g] - m); ppg[g] *= drift[g]; }
  }
  for (auto& v : ppg) { if (v > P.pitchCeiling) v = P.pitchCeiling; if (v < P.pitchFloor) v = P.pitchFloor; }
  const double pmin = r_min(ppg);
  const int64_t nH = (int64_t)std::ceil((sr / 2 - pmin) / pmin);
  vec ro(nGC), roo(nGC), rk(nGC);
  for (int64_t g = 0; g < nGC; ++g) {
    const double w = rw[g];
    ro[g] = (P.rolloff + rolloffAmpl[g]) * w * w * w;
    roo[g] = P.rolloffOct * w * w * w;
    rk[g] = P.rolloffKHz * w;
  }
  // amplitude matrices: built on the device from per-cycle parameters (spec),
  // or on the host (roll, mats[].A) where the formula path does not apply
  int64_t H = 0;
  AmpSpec spec;
  std::vector<int32_t> lastf;  // per cycle: last finite rolloff row (1-based)
  bool dev_amps = amp_device_enabled() && rolloff_spec(ppg, nH, ro, roo, P.rolloffParab, P.rolloffParabHarm, rk, 200,
                                                       P.throwaway, sr, spec, H, lastf);
  vec roll;
  if (!dev_amps) roll = get_rolloff(ppg, nH, ro, roo, P.rolloffParab, P.rolloffParabHarm, rk, 200, P.throwaway, sr, H);
  const bool shimmer = P.shimmerDep > 0 && P.nonlinBalance > 0;
  if (dev_amps) spec.lsh.assign((size_t)nGC, 0.0);
  if (shimmer)
    for (int64_t g = 0; g < nGC; ++g) {
      const double z = R.rnorm(0, P.shimmerDep / 100);
      const double e = z * rw[g] * jit_on[g];
      const double sh = std::pow(2.0, e);
      if (dev_amps) {
        spec.cols[g].sh = sh;
        spec.lsh[g] = e;
      } else {
        for (int64_t h = 0; h < H; ++h) roll[g * H + h] *= sh;
      }
    }
  std::vector<EpochMat> mats;
  ProfScope pfry(PF_FRY);
  const bool fry = P.subDep > 0 && P.nonlinBalance > 0;
  vec sf, sd;
  if (fry) {
    sf.resize(nGC);
    sd.resize(nGC);
    for (int64_t g = 0; g < nGC; ++g) { const double w4 = std::pow(rw[g], 4); sf[g] = P.subFreq * w4; sd[g] = P.subDep * w4 * vf_on[g]; }
  }
  if (dev_amps) {
    if (fry)
      for (int64_t g = 0; g < nGC; ++g) spec.cols[g].sbw = sd[g];
    const std::vector<FryEpoch> eps = fry ? fry_epochs(ppg, sf, P.shortestEpoch) : std::vector<FryEpoch>{{0, nGC - 1, 0}};
    for (const FryEpoch& e : eps) {
      mats.emplace_back();
      if (e.nsub == 0) {
        plain_spec(spec, H, e.g0, e.g1, lastf, mats.back());
      } else if (!fry_spec(spec, H, e.g0, e.g1, e.nsub, lastf, mats.back())) {
        dev_amps = false;  // a threshold call too close to decide for the device: host path
        break;
      }
    }
    if (!dev_amps) {
      mats.clear();
      roll = get_rolloff(ppg, nH, ro, roo, P.rolloffParab, P.rolloffParabHarm, rk, 200, P.throwaway, sr, H);
      if (shimmer)
        for (int64_t g = 0; g < nGC; ++g)
          for (int64_t h = 0; h < H; ++h) roll[g * H + h] *= spec.cols[g].sh;
    }
  }
  if (!dev_amps) {
    if (fry) mats = get_vocal_fry(roll, H, ppg, sf, sd, P.throwaway, P.shortestEpoch);
    else mats.push_back(fry_per_epoch(roll.data(), H, 0, nGC - 1, ppg, 0, vec(nGC, 0.0), 0));
    for (EpochMat& m : mats) m.float_pattern();
  }
  // upsample(): gcLen, gc_up, cumulative-pitch segments
  vec gcl(nGC);
  for (int64_t g = 0; g < nGC; ++g) gcl[g] = r_round(sr / ppg[g]);
  vec cs = r_cumsum(gcl);
  vec gc_up(nGC + 1);
  gc_up[0] = 1;
  for (int64_t g = 0; g < nGC; ++g) gc_up[g + 1] = cs[g];
  const int64_t N = (int64_t)cs[nGC - 1];
  HostSyl HS;
  HS.sr = sr;
  if (nGC == 1) {
    HS.segs.push_back(HSeg{0, 0, ppg[0], 0, 0, 0});
  } else if (nGC == 2) {
    const double by = (ppg[1] - ppg[0]) / (double)(N - 1);
    HS.segs.push_back(HSeg{0, 0, ppg[0] - by, by, 0, 0});
  } else {
    vec t(nGC);
    t[0] = 1; t[nGC - 1] = (double)N;
    for (int64_t i = 2; i <= nGC - 1; ++i) t[i - 1] = cs[i - 2] + r_round(gcl[i - 1] / 2);
    Spline s = fmm_spline(t, ppg);
    long double pre = s.y[0];
    for (int64_t k = 0; k + 1 < nGC; ++k) {
      HS.segs.push_back(HSeg{t[k], (double)pre, s.y[k], s.b[k], s.c[k], s.d[k]});
      const long double M = (long double)(t[k + 1] - t[k]);
      const long double S1 = M * (M + 1) / 2, S2 = M * (M + 1) * (2 * M + 1) / 6, S3 = S1 * S1;
      pre += s.y[k] * M + s.b[k] * S1 + s.c[k] * S2 + s.d[k] * S3;
    }
  }
  // epochs
  std::vector<HostEpoch> HE(mats.size());
  for (size_t e = 0; e < mats.size(); ++e) {
    HostEpoch& he = HE[e];
    he.M = &mats[e]; he.S = &HS;
    he.u0 = (int64_t)gc_up[mats[e].g0];
    const int64_t u1 = (int64_t)gc_up[mats[e].g1 + 1];
    he.n = u1 - he.u0 + 1;
    he.G = mats[e].g1 - mats[e].g0 + 1;
    if (he.G < 2) throw SgError(SG_E_DOMAIN, "approx: need at least two non-NA values to interpolate");
    he.knots.assign(gc_up.begin() + mats[e].g0, gc_up.begin() + mats[e].g1 + 1);
    he.init_fast();
  }
  // crossFade chain → pieces (host fp64 decisions)
  ProfScope pxf(PF_XFADE);
  Chain A;
  A.E = &HE;
  A.P.push_back(HPiece{0, 1, {}});  // waveform = 0
  for (size_t e = 0; e < mats.size(); ++e) cross_fade(A, HE[e], (int64_t)e, sr, 15);
  const int64_t Lsyl = A.L();
  if (dry_run || B.draws_only) return Lsyl;  // every draw of the syllable precedes this
  if (probes) {  // up to 4 glottal cycles' spectra (formant-filter conditioning)
    const int64_t np = std::min<int64_t>(4, nGC);
    for (int64_t q = 0; q < np; ++q) {
      const int64_t g = (2 * q + 1) * nGC / (2 * np);
      HarmProbe hp;
      hp.t = (int64_t)gc_up[g] - 1;
      hp.f0 = ppg[g];
      if (dev_amps) {
        hp.amp.resize((size_t)H);
        for (int64_t h = 0; h < H; ++h) hp.amp[h] = roll_value(spec.cols[g], spec.J, spec.lg.data(), (int)h);
      } else {
        hp.amp.assign(roll.begin() + g * H, roll.begin() + (g + 1) * H);
      }
      probes->push_back(std::move(hp));
    }
  }
  if (to_fs) {  // a fresh fs slot whose 16-B residue is out_off's (the syllable's offset in its bout)
    out_off = fs_alloc(B, Lsyl + 3) + (out_off & 3);
    if (fs_off) *fs_off = out_off;
  }

  // ------------------------------------------------ emit device arrays
  ProfScope pem(PF_EMIT);
  const int32_t syl_idx = (int32_t)B.syls.size();
  SgSyllable sy{};
  sy.L = Lsyl;
  sy.out_off = out_off;
  sy.dst_fs = to_fs ? 1 : 0;
  sy.max_slot = syl_idx;
  const double lf = P.attackLen > 0 ? std::floor(P.attackLen * sr / 1000) : 0;
  sy.fade = (int32_t)(lf >= 2 ? std::min<double>(lf, (double)Lsyl) : 0);
  sy.env = useAmpl ? contour_desc(B, amplAnchors, Lsyl, true, 0, false, 0, true, sr) : SgContour{};
  if (!useAmpl) { sy.env.kind = 0; sy.env.lo = -INFINITY; sy.env.hi = INFINITY; }
  if (P.temperature > 0) {
    sy.drift.nk = (int32_t)nGC;
    sy.drift.k_off = (int64_t)B.cknots.size();
    sy.drift.x0 = gc_up[0];
    sy.drift.x1 = gc_up[nGC - 1];
    B.cknots.insert(B.cknots.end(), gc_up.begin(), gc_up.begin() + nGC);
    B.cknots.insert(B.cknots.end(), drift.begin(), drift.end());
    // per interval t, for sg_harm_finalize's fp32 chunk path: the first sample kb_t whose
    // u (xout = seq.int(x0, x1, L), as the device forms it) reaches x_t, and the line
    // dm(k) = a_t + b_t (k - kb_t) of approx() over the interval in samples, as
    // (double kb_t, float a_t | float b_t bits) after x[] and y[]
    const double* xk = &B.cknots[sy.drift.k_off];
    const double* yk = xk + nGC;
    const int64_t L = Lsyl;
    const double x0 = sy.drift.x0, x1 = sy.drift.x1;
    const double by = L > 1 ? (x1 - x0) / (double)(L - 1) : 0.0;
    auto u_at = [&](int64_t k) -> double {
      if (k == 0) return x0;
      if (k == L - 1) return x1;
      return (k < L / 2) ? x0 + (double)k * by : x1 - (double)(L - 1 - k) * by;
    };
    std::vector<double> lines((size_t)(2 * nGC));
    for (int64_t t = 0; t < nGC; ++t) {
      int64_t kb = 0;
      if (t > 0 && by > 0) {
        kb = (int64_t)std::ceil((xk[t] - x0) / by);
        kb = std::max<int64_t>(0, std::min<int64_t>(kb, L));
        while (kb > 0 && u_at(kb - 1) >= xk[t]) --kb;
        while (kb < L && u_at(kb) < xk[t]) ++kb;
      }
      const double sl = t + 1 < nGC && xk[t + 1] > xk[t] ? (yk[t + 1] - yk[t]) / (xk[t + 1] - xk[t]) : 0.0;
      const double uk = kb < L ? u_at(kb) : x1;
      const float a = (float)std::fma(sl, uk - xk[t], yk[t]), bstep = (float)(sl * by);
      uint32_t ua, ub;
      std::memcpy(&ua, &a, 4);
      std::memcpy(&ub, &bstep, 4);
      const uint64_t bits = (uint64_t)ua | ((uint64_t)ub << 32);
      lines[(size_t)(2 * t)] = (double)kb;
      std::memcpy(&lines[(size_t)(2 * t + 1)], &bits, 8);
    }
    B.cknots.insert(B.cknots.end(), lines.begin(), lines.end());
  }
  const int32_t seg_off = (int32_t)B.segs.size();
  for (const HSeg& h : HS.segs) {
    // sum_{x=1..m} (y + b x + c x^2 + d x^3) = y m + b S1 + c S2 + d S3 expanded in powers of m
    const long double y = h.y, b = h.b, c = h.c, d = h.d, isr = 1.0L / (long double)sr;
    SgSeg g;
    g.t0 = h.t0;
    g.c0 = (double)((long double)h.prefix * isr);
    g.c1 = (double)((y + b / 2 + c / 6) * isr);
    g.c2 = (double)((b / 2 + c / 2 + d / 4) * isr);
    g.c3 = (double)((c / 3 + d / 2) * isr);
    g.c4 = (double)((d / 4) * isr);
    B.segs.push_back(g);
  }
  int64_t col0 = -1;
  if (dev_amps) {
    col0 = (int64_t)B.ampcols.size();
    B.ampcols.insert(B.ampcols.end(), spec.cols.begin(), spec.cols.end());
    B.amp_lg_rows = std::max<int64_t>(B.amp_lg_rows, H);
  }
  std::vector<int32_t> ep_index(mats.size());
  // destination offset of each epoch's direct piece, to keep the fp32 copy
  // in the finalize kernel 16-byte aligned on both sides
  std::vector<int64_t> dk(mats.size(), 0);
  for (const HPiece& p : A.P)
    if (p.t.size() == 1 && p.t[0].w0 == 1 && p.t[0].w1 == 0 && p.t[0].w2 == 0) dk[p.t[0].e] = p.start - p.t[0].j0;
  for (size_t e = 0; e < mats.size(); ++e) {
    const EpochMat& m = mats[e];
    const HostEpoch& he = HE[e];
    SgEpoch d{};
    const int64_t want = (((out_off + dk[e]) % 4) + 4) % 4;
    B.w_total += ((want - B.w_total % 4) + 4) % 4;
    d.w_off = B.w_total;
    B.w_total += he.n;
    d.n = (int32_t)he.n;
    d.G = (int32_t)he.G;
    d.R = (int32_t)((m.R + SG_ROW_CHUNK - 1) / SG_ROW_CHUNK * SG_ROW_CHUNK);
    d.u0 = (int32_t)he.u0;
    d.seg_off = seg_off;
    d.nseg = (int32_t)HS.segs.size();
    d.x1 = he.knots.front();
    d.xG = he.knots.back();
    d.xby = he.n > 1 ? (d.xG - d.x1) / (double)(he.n - 1) : 0.0;
    d.invD = 1.0 / (double)m.D;
    d.knot_off = (int64_t)B.knots.size();
    B.knots.insert(B.knots.end(), he.knots.begin(), he.knots.end());
    // [G][R] amplitudes (device array, built by sg_amp_build at upload from the
    // job: formula, or the host-built values); a task reads its two columns
    d.amp_off = B.amp_total;
    B.amp_total += (int64_t)d.G * d.R;
    {
      SgAmpJob j = dev_amps ? m.job : SgAmpJob{};
      j.amp_off = d.amp_off;
      j.G = d.G;
      j.R = (int32_t)m.R;
      j.Rp = d.R;
      if (dev_amps) {
        j.src_off = -1;
        j.col0 = col0;
      } else {
        j.src_off = (int64_t)B.ampsrc.size();
        j.col0 = -1;
        B.ampsrc.resize(B.ampsrc.size() + (size_t)d.G * d.R);
        float* a = B.ampsrc.data() + j.src_off;
        for (int64_t g = 0; g < he.G; ++g) {
          float* row = a + g * d.R;
          for (int64_t r = 0; r < m.R; ++r) row[r] = (float)m.A[g * m.R + r];
          std::fill(row + m.R, row + d.R, 0.0f);
        }
      }
      B.ampjobs.push_back(j);
    }
    d.syl = syl_idx;
    d.dj0 = d.dj1 = 0;
    d.dk0 = 0;
    ep_index[e] = (int32_t)B.epochs.size();
    B.epochs.push_back(d);
    B.harm_samples += he.n;
    B.harm_terms += he.n * (int64_t)d.R;
    B.harm_amp_bytes += (int64_t)d.G * d.R * 4;
  }
  // pieces; the single full-weight piece of each epoch becomes its direct window
  sy.piece0 = (int32_t)B.pieces.size();
  for (const HPiece& p : A.P) {
    SgPiece d{};
    d.start = p.start;
    d.len = (int32_t)p.len;
    d.nterms = (int32_t)p.t.size();
    for (size_t k = 0; k < p.t.size(); ++k) {
      const HTerm& t = p.t[k];
      const SgEpoch& ep = B.epochs[ep_index[t.e]];
      d.t[k].src = ep.w_off + t.j0;
      d.t[k].w0 = (float)t.w0; d.t[k].w1 = (float)t.w1; d.t[k].w2 = (float)t.w2;
    }
    if (p.t.size() == 1 && p.t[0].w0 == 1 && p.t[0].w1 == 0 && p.t[0].w2 == 0) {
      SgEpoch& ep = B.epochs[ep_index[p.t[0].e]];
      ep.dj0 = (int32_t)p.t[0].j0;
      ep.dj1 = (int32_t)(p.t[0].j0 + p.len);
      ep.dk0 = p.start - p.t[0].j0;
      d.nterms = -1;  // marks a direct piece (max handled by the sine-bank kernel)
      d.t[0].src = ep.w_off + p.t[0].j0;
      d.t[0].w0 = 1;
    }
    B.pieces.push_back(d);
  }
  sy.npiece = (int32_t)(B.pieces.size() - sy.piece0);
  B.syls.push_back(sy);
  // sine-bank wave tasks: <= SG_TASK_MAX samples inside one amplitude
  // interval, or inside a run of intervals with equal columns
  B.syls.back().task0 = (int64_t)B.tasks.size();
  ProfScope ptk(PF_TASKS);
  const int64_t nseg = (int64_t)HS.segs.size();
  for (size_t e = 0; e < mats.size(); ++e) {
    const HostEpoch& he = HE[e];
    const SgEpoch& ep = B.epochs[ep_index[e]];
    // sample boundaries of the intervals: jb[i] = first j with xout_j >= knot i+1
    std::vector<int64_t> jb(he.G - 1);
    std::vector<char> cst(he.G - 1);
    std::vector<int32_t> rn(he.G - 1);
    int64_t ja = 0;
    for (int64_t i = 0; i + 1 < he.G; ++i) {
      int64_t g = he.n;
      if (i + 2 < he.G) {
        const double xb = he.knots[i + 1];
        g = (int64_t)std::floor((xb - he.knots.front()) / ep.xby);
        if (g < ja) g = ja;
        if (g > he.n) g = he.n;
        while (g > ja && r_seqint_at(he.knots.front(), he.knots.back(), he.n, g - 1) >= xb) --g;
        while (g < he.n && r_seqint_at(he.knots.front(), he.knots.back(), he.n, g) < xb) ++g;
      }
      jb[i] = g;
      ja = g;
      const EpochMat& m = mats[e];
      const bool c = m.eq[i] != 0;  // dA[i] = 0: one chain
      cst[i] = c;
      // rows the device recurrence needs: up to the last nonzero A (or dA) row
      const int64_t last = std::max<int64_t>(m.lnz[i], c ? 0 : m.lnz[i + 1]);
      rn[i] = (int32_t)((last + 3) / 4 * 4);
    }
    int64_t k = 0;
    ja = 0;
    for (int64_t i = 0; i + 1 < he.G;) {
      int64_t i1 = i + 1;  // span [i, i1) of intervals
      if (cst[i])
        while (i1 + 1 < he.G && cst[i1]) ++i1;
      const int64_t jend = jb[i1 - 1];
      for (int64_t j0 = ja; j0 < jend;) {
        const double u = (double)(he.u0 + j0);
        while (k + 1 < nseg && HS.segs[k + 1].t0 < u) ++k;
        int64_t len = std::min<int64_t>(task_max(), jend - j0);
        // a linear segment continues through the following segments that lie
        // on the same line (constant pitch: one FMM piece per glottal cycle,
        // all with equal slope), so a task may span them with segment k's
        // coefficients; phase drift from the merge stays ~1e-12 cycles
        int64_t kk = k;
        while (kk + 1 < nseg && lin_continues(B.segs[seg_off + kk], B.segs[seg_off + kk + 1])) ++kk;
        if (kk + 1 < nseg) {  // stay inside segments k..kk: u <= t0[kk+1]
          const int64_t jmax = (int64_t)HS.segs[kk + 1].t0 - he.u0 + 1;
          if (j0 + len > jmax) len = jmax - j0;
        }
        const SgSeg& S = B.segs[seg_off + k];
        SgWTask T{};
        T.w_off = ep.w_off;
        T.a_off = ep.amp_off + i * ep.R;
        T.d_off = ep.amp_off + (i + 1) * ep.R;  // A[i + 1]
        T.dk0 = ep.dk0;
        // phase in cycles of the epoch's lowest multiplier: integr / D folded into the
        // coefficients (the device evaluates the polynomial only)
        T.c0 = S.c0 * ep.invD; T.c1 = S.c1 * ep.invD; T.c2 = S.c2 * ep.invD; T.c3 = S.c3 * ep.invD;
        T.c4 = S.c4 * ep.invD;
        T.invD = ep.invD;
        T.rdx = (float)(1.0 / (he.knots[i + 1] - he.knots[i]));
        T.tc0 = (float)(r_seqint_at(he.knots.front(), he.knots.back(), he.n, j0) - he.knots[i]);
        T.xby = (float)ep.xby;
        T.mbase = (int32_t)((double)(he.u0 + j0) - S.t0);
        T.R = ep.R;
        {  // a span of equal columns: the rows of its intervals (equal A; dA zero)
          int32_t m = 0;
          for (int64_t q = i; q < i1; ++q) m = std::max(m, rn[q]);
          T.Rn = m;
        }
        T.j0 = (int32_t)j0; T.len = (int32_t)len;
        T.dj0 = ep.dj0; T.dj1 = ep.dj1;
        T.syl = ep.syl;
        T.flags = (cst[i] ? SG_TASK_CONST : 0) | (S.c2 == 0 && S.c3 == 0 && S.c4 == 0 ? SG_TASK_LIN : 0) |
                  (B.syls[ep.syl].env.kind != 0 ? SG_TASK_ENV : 0);
        B.tasks.push_back(T);
        j0 += len;
      }
      ja = jend;
      i = i1;
    }
  }
  B.syls.back().ntask = (int32_t)((int64_t)B.tasks.size() - B.syls.back().task0);
  return Lsyl;
}

int64_t fh_alloc(Batch& B, int64_t n) {
  const int64_t o = B.fh_total;
  B.fh_total += (n + 31) / 32 * 32;  // 256-B aligned regions
  return o;
}

// The syllable's epoch waveforms move from W to a fresh W64 range (same relative
// layout; its epochs are consecutive in W), its tasks take the fp64 class and
// its output goes to fh. W keeps the now unused floats (scratch only).
int64_t syllable_to_fp64(Batch& B, int s) {
  SgSyllable& sy = B.syls[s];
  int64_t wlo = INT64_MAX, whi = 0;
  for (int64_t t = sy.task0; t < sy.task0 + sy.ntask; ++t) {
    const SgWTask& T = B.tasks[t];
    wlo = std::min<int64_t>(wlo, T.w_off + T.j0);
    whi = std::max<int64_t>(whi, T.w_off + T.j0 + T.len);
  }
  for (int32_t p = sy.piece0; p < sy.piece0 + sy.npiece; ++p) {
    const SgPiece& pc = B.pieces[p];
    for (int q = 0; q < (pc.nterms < 0 ? 1 : pc.nterms); ++q) {
      wlo = std::min<int64_t>(wlo, pc.t[q].src);
      whi = std::max<int64_t>(whi, pc.t[q].src + pc.len);
    }
  }
  if (wlo > whi) wlo = whi = 0;
  const int64_t base = B.w64_total - wlo;
  B.w64_total += (whi - wlo + 31) / 32 * 32;
  for (int64_t t = sy.task0; t < sy.task0 + sy.ntask; ++t) {
    SgWTask& T = B.tasks[t];
    T.w_off += base;
    T.flags |= SG_TASK_HP;
  }
  for (int32_t p = sy.piece0; p < sy.piece0 + sy.npiece; ++p) {
    SgPiece& pc = B.pieces[p];
    for (int q = 0; q < (pc.nterms < 0 ? 1 : pc.nterms); ++q) pc.t[q].src += base;
  }
  sy.hp = 1;
  sy.out_off = fh_alloc(B, sy.L);
  return sy.out_off;
}

// drift-knot interval of sample k: largest i in [0, nk - 2] with x[i] <= u(k),
// u(k) exactly as sg_devfn.h linear_at computes it
static int32_t drift_interval(const Batch& B, const SgSyllable& sy, int64_t k) {
  const SgLinear& l = sy.drift;
  const double* x = &B.cknots[l.k_off];
  const int64_t L = sy.L;
  double u;
  if (k == 0) u = l.x0;
  else if (k == L - 1) u = l.x1;
  else {
    const double by = (l.x1 - l.x0) / (double)(L - 1);
    u = (k < L / 2) ? l.x0 + (double)k * by : l.x1 - (double)(L - 1 - k) * by;
  }
  int a = 0, b = l.nk - 1;
  while (a < b - 1) { const int ab = (a + b) >> 1; if (u < x[ab]) b = ab; else a = ab; }
  return a;
}

// noiseThresholdsDict$q1 / $q2 [nonlinBalance + 1] (R/sysdata.rda, built by
// data-raw/noiseThresholdsDict.R:1-19: 100 / (1 + exp(-slope (amount - midpoint))),
// slope -0.1, midpoints 33 and 66); R truncates the index. Pinned value for
// value against the decoded sysdata.rda (tests/test_rda_fixtures.py).
double noise_threshold(int which, double nonlinBalance) {
  const double k = (double)(int64_t)(nonlinBalance + 1) - 1;
  return 100 / (1 + std::exp(0.1 * (k - (which == 1 ? 33 : 66))));
}

void tile_syllables(Batch& B, int first_syl) {
  constexpr int64_t STILE = 1024;
  for (int s = first_syl; s < (int)B.syls.size(); ++s) {
    const SgSyllable& sy = B.syls[s];
    int32_t p = sy.piece0;
    for (int64_t k0 = 0; k0 < sy.L; k0 += STILE) {
      while (p + 1 < sy.piece0 + sy.npiece && B.pieces[p + 1].start <= k0) ++p;
      SgSylTile t{};
      t.syl = s;
      t.piece = p;
      t.k0 = k0;
      int32_t pw = p;
      for (int w = 0; w < 4; ++w) {
        const int64_t c0 = std::min<int64_t>(k0 + 256 * w, sy.L - 1);
        while (pw + 1 < sy.piece0 + sy.npiece && B.pieces[pw + 1].start <= c0) ++pw;
        t.wpiece[w] = pw;
        t.wdrift[w] = sy.drift.nk > 1 ? drift_interval(B, sy, c0) : 0;
      }
      B.syl_tiles.push_back(t);
    }
  }
}

}  // namespace sg

extern "C" int sg_set_amp_policy(int32_t host_built) {
  if (host_built < 0 || host_built > 1) return SG_E_ARG;
  sg::g_amp_host.store(host_built);
  return SG_OK;
}
