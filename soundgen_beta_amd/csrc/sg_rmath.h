// sg_rmath.h — host-side restatement of the R-base semantics the planner
// needs for bit-exact bookkeeping (R 3.4.0):
//   round() half-even, seq()/seq.int(), spline(method="fmm"), approx(),
//   cumsum/sum/mean in long double, rnorm() without a draw when sd == 0.
#pragma once
#include <cmath>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "soundgen_hip.h"

namespace sg {

// Planner scratch memory. A call's temporaries (rolloff matrices, epoch
// amplitudes, contours: tens of KB to MB each) come from a per-thread pool of
// power-of-two blocks that outlives the call, so the next call reuses pages
// already faulted in instead of mapping, zeroing and unmapping fresh ones
// (sg_scratch.cpp). Small blocks go straight to malloc.
void* scratch_alloc(size_t bytes);
void scratch_free(void* p, size_t bytes) noexcept;
void scratch_trim() noexcept;  // return the calling thread's pool to the system

// Bulk blocks of 8 MB and up are 2 MB-aligned and marked for transparent huge
// pages: a plan's host arrays run to GBs, and faulting them in 4 KB pages (on
// the planning threads, then again in the merge) cost more than writing them.
void* bulk_alloc(size_t bytes);
void bulk_free(void* p, size_t bytes) noexcept;
size_t bulk_trim() noexcept;  // free every cached bulk block; returns the bytes released
constexpr size_t SG_BULK_HUGE = size_t(8) << 20;

template <class T>
struct ScratchAlloc {
  using value_type = T;
  ScratchAlloc() = default;
  template <class U>
  ScratchAlloc(const ScratchAlloc<U>&) noexcept {}
  T* allocate(size_t n) { return static_cast<T*>(scratch_alloc(n * sizeof(T))); }
  void deallocate(T* p, size_t n) noexcept { scratch_free(p, n * sizeof(T)); }
  template <class U>
  bool operator==(const ScratchAlloc<U>&) const noexcept { return true; }
  template <class U>
  bool operator!=(const ScratchAlloc<U>&) const noexcept { return false; }
};

using vec = std::vector<double, ScratchAlloc<double>>;

struct SgError : std::runtime_error {
  int code;
  SgError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

inline double r_round(double x) { return std::nearbyint(x); }

inline double r_sum(const double* x, size_t n) {
  long double s = 0;
  for (size_t i = 0; i < n; ++i) s += x[i];
  return (double)s;
}
inline double r_mean(const vec& x) {
  const size_t n = x.size();
  long double s = 0;
  for (double v : x) s += v;
  s /= n;
  if (std::isfinite((double)s)) {
    long double t = 0;
    for (double v : x) t += (v - s);
    s += t / n;
  }
  return (double)s;
}
inline double r_max(const vec& x) {
  double m = -INFINITY;
  for (double v : x) { if (std::isnan(v)) return NAN; if (v > m) m = v; }
  return m;
}
inline double r_min(const vec& x) {
  double m = INFINITY;
  for (double v : x) { if (std::isnan(v)) return NAN; if (v < m) m = v; }
  return m;
}
inline vec r_cumsum(const vec& x) {
  vec o(x.size());
  long double s = 0;
  for (size_t i = 0; i < x.size(); ++i) { s += x[i]; o[i] = (double)s; }
  return o;
}
// seq(from, to, length.out = n), R 3.4 seq.default
inline vec r_seq_len(double from, double to, int64_t n) {
  vec a(n > 0 ? n : 0);
  if (n <= 0) return a;
  if (n == 1) { a[0] = from; return a; }
  if (n == 2) { a[0] = from; a[1] = to; return a; }
  if (from == to) { for (auto& v : a) v = from; return a; }
  const double by = (to - from) / (double)(n - 1);
  a[0] = from;
  for (int64_t i = 1; i < n - 1; ++i) a[i] = from + (double)i * by;
  a[n - 1] = to;
  return a;
}
// element i of seq.int(from, to, length.out = n) (R seq.c, symmetric interior)
inline double r_seqint_at(double from, double to, int64_t n, int64_t i) {
  if (i == 0) return from;
  if (i == n - 1) return to;
  const double by = (to - from) / (double)(n - 1);
  return (i < n / 2) ? from + (double)i * by : to - (double)(n - 1 - i) * by;
}
inline vec r_seqint_len(double from, double to, int64_t n) {
  vec a(n > 0 ? n : 0);
  for (int64_t i = 0; i < n; ++i) a[i] = r_seqint_at(from, to, n, i);
  return a;
}
// seq(from, to, by = by), by > 0
inline vec r_seq_by(double from, double to, double by) {
  const double del = to - from;
  if (del == 0.0 && to == 0.0) return vec{to};
  const double dd = std::fabs(del) / std::fmax(std::fabs(to), std::fabs(from));
  if (dd < 100 * 2.220446049250313e-16) return vec{from};
  const double nn = del / by;
  if (nn < 0) return vec{};
  const int64_t n = (int64_t)(nn + 1e-10);
  vec a(n + 1);
  for (int64_t i = 0; i <= n; ++i) { double x = from + (double)i * by; a[i] = x > to ? to : x; }
  return a;
}

// FMM cubic spline coefficients (stats/src/splines.c fmm_spline)
struct Spline {
  vec x, y, b, c, d;
  size_t n() const { return x.size(); }
  // spline_eval with R's sticky-interval rule; `i` carries between calls.
  double eval(double ul, int64_t& i) const {
    const int64_t n_1 = (int64_t)x.size() - 1;
    if (ul < x[i] || (i < n_1 && x[i + 1] < ul)) {
      i = 0;
      int64_t j = (int64_t)x.size();
      do { int64_t k = (i + j) / 2; if (ul < x[k]) j = k; else i = k; } while (j > i + 1);
    }
    const double dx = ul - x[i];
    return y[i] + dx * (b[i] + dx * (c[i] + dx * d[i]));
  }
};
inline Spline fmm_spline(const vec& xin, const vec& yin) {
  Spline s;
  s.x = xin; s.y = yin;
  const int64_t n = (int64_t)xin.size();
  s.b.assign(n, 0); s.c.assign(n, 0); s.d.assign(n, 0);
  if (n < 2) return s;
  double* x = s.x.data() - 1; double* y = s.y.data() - 1;
  double* b = s.b.data() - 1; double* c = s.c.data() - 1; double* d = s.d.data() - 1;
  double t;
  if (n < 3) {
    t = (y[2] - y[1]);
    b[1] = t / (x[2] - x[1]); b[2] = b[1];
    c[1] = c[2] = d[1] = d[2] = 0.0;
    return s;
  }
  const int64_t nm1 = n - 1;
  d[1] = x[2] - x[1];
  c[2] = (y[2] - y[1]) / d[1];
  for (int64_t i = 2; i < n; i++) {
    d[i] = x[i + 1] - x[i];
    b[i] = 2.0 * (d[i - 1] + d[i]);
    c[i + 1] = (y[i + 1] - y[i]) / d[i];
    c[i] = c[i + 1] - c[i];
  }
  b[1] = -d[1]; b[n] = -d[nm1];
  c[1] = c[n] = 0.0;
  if (n > 3) {
    c[1] = c[3] / (x[4] - x[2]) - c[2] / (x[3] - x[1]);
    c[n] = c[nm1] / (x[n] - x[n - 2]) - c[n - 2] / (x[nm1] - x[n - 3]);
    c[1] = c[1] * d[1] * d[1] / (x[4] - x[1]);
    c[n] = -c[n] * d[nm1] * d[nm1] / (x[n] - x[n - 3]);
  }
  for (int64_t i = 2; i <= n; i++) {
    t = d[i - 1] / b[i - 1];
    b[i] = b[i] - t * d[i - 1];
    c[i] = c[i] - t * c[i - 1];
  }
  c[n] = c[n] / b[n];
  for (int64_t i = nm1; i >= 1; i--) c[i] = (c[i] - d[i] * c[i + 1]) / b[i];
  b[n] = (y[n] - y[n - 1]) / d[n - 1] + d[n - 1] * (c[n - 1] + 2.0 * c[n]);
  for (int64_t i = 1; i <= nm1; i++) {
    b[i] = (y[i + 1] - y[i]) / d[i] - d[i] * (c[i + 1] + 2.0 * c[i]);
    d[i] = (c[i + 1] - c[i]) / d[i];
    c[i] = 3.0 * c[i];
  }
  c[n] = 3.0 * c[n];
  d[n] = d[nm1];
  return s;
}
// spline(x, y, n)$y
inline vec r_spline(const vec& x, const vec& y, int64_t n) {
  Spline s = fmm_spline(x, y);
  vec out(n);
  int64_t i = 0;
  for (int64_t l = 0; l < n; ++l) out[l] = s.eval(r_seqint_at(x.front(), x.back(), n, l), i);
  return out;
}
// std::log2(k) of a positive integer k, from a table for the bins of any window
inline double log2_int(int64_t k) {
  static const std::vector<double> tab = [] {
    std::vector<double> t(16385);
    for (size_t i = 1; i < t.size(); ++i) t[i] = std::log2((double)i);
    return t;
  }();
  return k > 0 && k < (int64_t)tab.size() ? tab[(size_t)k] : std::log2((double)k);
}
// approx1 (stats/src/approx.c), rule = 1
inline double approx1(double v, const double* x, const double* y, int64_t n) {
  int64_t i = 0, j = n - 1;
  if (v < x[i] || v > x[j]) return NAN;
  while (i < j - 1) { int64_t ij = (i + j) / 2; if (v < x[ij]) j = ij; else i = ij; }
  if (v == x[j]) return y[j];
  if (v == x[i]) return y[i];
  return y[i] + (y[j] - y[i]) * ((v - x[i]) / (x[j] - x[i]));
}
inline vec r_approx_n(const vec& x, const vec& y, int64_t n) {
  if (x.size() <= 1) throw SgError(SG_E_DOMAIN, "approx: need at least two non-NA values to interpolate");
  vec out(n);
  for (int64_t l = 0; l < n; ++l)
    out[l] = approx1(r_seqint_at(x.front(), x.back(), n, l), x.data(), y.data(), (int64_t)x.size());
  return out;
}

// ---- injected random streams (R draw order) ----
struct Rng {
  const sg_random* s = nullptr;
  int64_t in = 0, iu = 0;
  double norm() {
    if (s && in < s->n_normals) return s->normals[in++];
    if (s && s->norm_cb) return s->norm_cb(s->user);
    throw SgError(SG_E_RANDOM, "normal stream exhausted");
  }
  double unif() {
    if (s && iu < s->n_uniforms) return s->uniforms[iu++];
    if (s && s->unif_cb) return s->unif_cb(s->user);
    throw SgError(SG_E_RANDOM, "uniform stream exhausted");
  }
  // n consecutive runif() draws as floats (out may be null: draws consumed, discarded);
  // past the injected array, blocks through the bulk callback when there is one
  void unif_f32(int64_t n, float* out) {
    int64_t k = 0;
    if (s) {
      const int64_t avail = std::max<int64_t>(0, std::min<int64_t>(n, s->n_uniforms - iu));
      if (out)
        for (int64_t q = 0; q < avail; ++q) out[q] = (float)s->uniforms[iu + q];
      iu += avail;
      k = avail;
      if (k < n && s->unif_n_cb) {
        double blk[1024];
        while (k < n) {
          const int64_t m = std::min<int64_t>(n - k, 1024);
          s->unif_n_cb(s->user, blk, m);
          if (out)
            for (int64_t q = 0; q < m; ++q) out[k + q] = (float)blk[q];
          k += m;
        }
      }
    }
    for (; k < n; ++k) {
      const double x = unif();
      if (out) out[k] = (float)x;
    }
  }
  // rnorm(1, mu, sd): no draw when sd == 0 (nmath/rnorm.c)
  double rnorm(double mu, double sd) {
    if (sd == 0.0 || !std::isfinite(mu)) return mu;
    return mu + sd * norm();
  }
  // rgamma(1, shape, rate): the gamma callback (R's own rgamma) when bound,
  // else Marsaglia-Tsang on the injected streams
  double rgamma(double shape, double rate) {
    if (!(shape > 0) || !(rate > 0)) return NAN;
    if (s && s->gamma_cb) return s->gamma_cb(s->user, shape, rate);
    double boost = 1.0, a = shape;
    if (a < 1.0) { boost = std::pow(unif(), 1.0 / a); a += 1.0; }
    const double d = a - 1.0 / 3.0, c = 1.0 / std::sqrt(9.0 * d);
    for (int it = 0; it < 1000; ++it) {
      double z, v;
      do { z = norm(); v = 1.0 + c * z; } while (v <= 0.0);
      v = v * v * v;
      const double u = unif();
      if (std::log(u) < 0.5 * z * z + d - d * v + d * std::log(v)) return d * v * boost / rate;
    }
    throw SgError(SG_E_RANDOM, "rgamma rejection loop did not terminate");
  }
};

inline double HzToSemitones(double h) { return std::log2(h / 16.3516) * 12; }
inline double semitonesToHz(double s) { return 16.3516 * std::pow(2.0, s / 12); }

}  // namespace sg
