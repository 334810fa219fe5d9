/*
 * sg_oracle.c — TEST INFRASTRUCTURE ONLY (the parity checker / CPU baseline).
 *
 * Plain-C, IEEE-double restatement of the reference soundgen synthesis path
 * (nemochina2008/soundgen_beta, R package soundgen 1.0.0) and of the R-base /
 * seewave numerics it calls. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this; the product library never does.
 *
 * PARITY STATUS: R is absent from the build container and the reference ships
 * no golden vectors for this path, so this restatement is
 * "parity unpinned" against R itself. It is pinned against: analytic
 * known-answer tests, an independent NumPy restatement (tests/), the seewave
 * istft/stft definitions, and fixtures in tests/golden/ generated from it
 * (tools/r_golden.R regenerates them from real R where R exists).
 *
 * R-base semantics restated from R 3.4.0 sources (not vendored, see
 * SURVEY.md Appendix A): spline(method="fmm") [stats/src/splines.c],
 * approx() [stats/src/approx.c], seq()/seq.int(), round() (half-even),
 * cumsum/sum/mean (long double), rnorm() (mean + sd*Z, no draw when sd==0),
 * sample() (pre-3.6 "Rounding" + ProbSampleNoReplace with revsort).
 * rgamma() uses Marsaglia-Tsang on the injected streams (NOT R's
 * Ahrens-Dieter; documented in DESIGN.md) — only reached at temperature > 0.
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/soundgen_hip.h"

#define OR_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------ errors */
static __thread char g_err[512];  /* per thread: bench.py runs oracle calls on a thread pool */
static int fail(int code, const char* msg) {
  snprintf(g_err, sizeof g_err, "%s", msg);
  return code;
}
OR_API const char* or_last_error(void) { return g_err; }
OR_API void or_free(void* p) { free(p); }

#define TRY(x) do { int _rc = (x); if (_rc < 0) { rc = _rc; goto done; } } while (0)

/* ------------------------------------------------------------------ vectors */
typedef struct { double* v; int64_t n; } dv;
static dv dv_new(int64_t n) {
  dv a; a.n = n; a.v = (double*)calloc((size_t)(n > 0 ? n : 1), sizeof(double));
  return a;
}
static void dv_free(dv* a) { free(a->v); a->v = NULL; a->n = 0; }
static dv dv_copy(const double* x, int64_t n) {
  dv a = dv_new(n); if (n) memcpy(a.v, x, (size_t)n * sizeof(double)); return a;
}
static void dv_append(dv* a, const double* x, int64_t n) {
  a->v = (double*)realloc(a->v, (size_t)(a->n + n > 0 ? a->n + n : 1) * sizeof(double));
  if (n) memcpy(a->v + a->n, x, (size_t)n * sizeof(double));
  a->n += n;
}
static void dv_append_zeros(dv* a, int64_t n) {
  if (n <= 0) return;
  a->v = (double*)realloc(a->v, (size_t)(a->n + n) * sizeof(double));
  memset(a->v + a->n, 0, (size_t)n * sizeof(double));
  a->n += n;
}

/* ------------------------------------------------------------------ random */
typedef struct { const sg_random* s; int64_t in, iu; } rng_t;
static int rng_norm(rng_t* r, double* z) {
  if (r && r->s && r->in < r->s->n_normals) { *z = r->s->normals[r->in++]; return 0; }
  if (r && r->s && r->s->norm_cb) { *z = r->s->norm_cb(r->s->user); return 0; }
  return fail(SG_E_RANDOM, "normal stream exhausted");
}
static int rng_unif(rng_t* r, double* u) {
  if (r && r->s && r->iu < r->s->n_uniforms) { *u = r->s->uniforms[r->iu++]; return 0; }
  if (r && r->s && r->s->unif_cb) { *u = r->s->unif_cb(r->s->user); return 0; }
  return fail(SG_E_RANDOM, "uniform stream exhausted");
}
/* R rnorm(1, mu, sd): no draw when sd == 0 (nmath/rnorm.c) */
static int r_rnorm1(rng_t* r, double mu, double sd, double* out) {
  if (sd == 0.0 || !isfinite(mu)) { *out = mu; return 0; }
  double z; int rc = rng_norm(r, &z); if (rc) return rc;
  *out = mu + sd * z; return 0;
}
/* rgamma(1, shape, rate): Marsaglia-Tsang on the injected streams. */
static int r_rgamma1(rng_t* r, double shape, double rate, double* out) {
  if (!(shape > 0) || !(rate > 0)) { *out = NAN; return 0; }
  if (r && r->s && r->s->gamma_cb) { *out = r->s->gamma_cb(r->s->user, shape, rate); return 0; }
  double boost = 1.0, a = shape;
  if (a < 1.0) {
    double u; int rc = rng_unif(r, &u); if (rc) return rc;
    boost = pow(u, 1.0 / a); a += 1.0;
  }
  double d = a - 1.0 / 3.0, c = 1.0 / sqrt(9.0 * d);
  for (int it = 0; it < 1000; ++it) {
    double z, u, v; int rc;
    do { if ((rc = rng_norm(r, &z))) return rc; v = 1.0 + c * z; } while (v <= 0.0);
    v = v * v * v;
    if ((rc = rng_unif(r, &u))) return rc;
    if (log(u) < 0.5 * z * z + d - d * v + d * log(v)) { *out = d * v * boost / rate; return 0; }
  }
  return fail(SG_E_RANDOM, "rgamma rejection loop did not terminate");
}

/* ------------------------------------------------------------------ R base */
static double r_round(double x) { return nearbyint(x); } /* round(x, 0): half-even */
static double r_sum(const double* x, int64_t n) {
  long double s = 0; for (int64_t i = 0; i < n; ++i) s += x[i]; return (double)s;
}
static double r_mean(const double* x, int64_t n) {
  long double s = 0; for (int64_t i = 0; i < n; ++i) s += x[i];
  s /= n;
  if (isfinite((double)s)) {
    long double t = 0; for (int64_t i = 0; i < n; ++i) t += (x[i] - s);
    s += t / n;
  }
  return (double)s;
}
static double r_max(const double* x, int64_t n) {
  double m = -INFINITY; for (int64_t i = 0; i < n; ++i) { if (isnan(x[i])) return NAN; if (x[i] > m) m = x[i]; } return m;
}
static double r_min(const double* x, int64_t n) {
  double m = INFINITY; for (int64_t i = 0; i < n; ++i) { if (isnan(x[i])) return NAN; if (x[i] < m) m = x[i]; } return m;
}
static void r_cumsum(const double* x, double* out, int64_t n) {
  long double s = 0; for (int64_t i = 0; i < n; ++i) { s += x[i]; out[i] = (double)s; }
}
/* seq(from, to, length.out = n)  (R 3.4 seq.default) */
static dv r_seq_len(double from, double to, int64_t n) {
  dv a = dv_new(n);
  if (n <= 0) return a;
  if (n == 1) { a.v[0] = from; return a; }
  if (n == 2) { a.v[0] = from; a.v[1] = to; return a; }
  if (from == to) { for (int64_t i = 0; i < n; ++i) a.v[i] = from; return a; }
  double by = (to - from) / (double)(n - 1);
  a.v[0] = from;
  for (int64_t i = 1; i < n - 1; ++i) a.v[i] = from + (double)i * by;
  a.v[n - 1] = to;
  return a;
}
/* seq.int(from, to, length.out = n)  (R 3.4 seq.c; symmetric interior) */
static dv r_seqint_len(double from, double to, int64_t n) {
  dv a = dv_new(n);
  if (n <= 0) return a;
  a.v[0] = from;
  if (n > 1) a.v[n - 1] = to;
  if (n > 2) {
    double by = (to - from) / (double)(n - 1);
    for (int64_t i = 1; i < n - 1; ++i)
      a.v[i] = (i < n / 2) ? from + (double)i * by : to - (double)(n - 1 - i) * by;
  }
  return a;
}
/* seq(from, to, by = by) (R 3.4 seq.default, by > 0) */
static dv r_seq_by(double from, double to, double by) {
  double del = to - from;
  if (del == 0.0 && to == 0.0) { dv a = dv_new(1); a.v[0] = to; return a; }
  double dd = fabs(del) / fmax(fabs(to), fabs(from));
  if (dd < 100 * 2.220446049250313e-16) { dv a = dv_new(1); a.v[0] = from; return a; }
  double nn = del / by;
  if (nn < 0) { dv a = dv_new(0); return a; }
  int64_t n = (int64_t)(nn + 1e-10);
  dv a = dv_new(n + 1);
  for (int64_t i = 0; i <= n; ++i) { double x = from + (double)i * by; a.v[i] = x > to ? to : x; }
  return a;
}

/* ---- spline(method = "fmm") — stats/src/splines.c ---- */
typedef struct { int64_t n; double *x, *y, *b, *c, *d; } spl_t;
static void spl_free(spl_t* s) { free(s->x); free(s->y); free(s->b); free(s->c); free(s->d); memset(s, 0, sizeof *s); }
static spl_t fmm_coef(const double* xin, const double* yin, int64_t n) {
  spl_t s; s.n = n;
  s.x = (double*)malloc(n * sizeof(double)); s.y = (double*)malloc(n * sizeof(double));
  s.b = (double*)calloc(n, sizeof(double)); s.c = (double*)calloc(n, sizeof(double)); s.d = (double*)calloc(n, sizeof(double));
  memcpy(s.x, xin, n * sizeof(double)); memcpy(s.y, yin, n * sizeof(double));
  if (n < 2) return s;
  double *x = s.x - 1, *y = s.y - 1, *b = s.b - 1, *c = s.c - 1, *d = s.d - 1, t;
  if (n < 3) {
    t = (y[2] - y[1]); b[1] = t / (x[2] - x[1]); b[2] = b[1];
    c[1] = c[2] = d[1] = d[2] = 0.0; return s;
  }
  const int64_t nm1 = n - 1; int64_t i;
  d[1] = x[2] - x[1];
  c[2] = (y[2] - y[1]) / d[1];
  for (i = 2; i < n; i++) {
    d[i] = x[i + 1] - x[i];
    b[i] = 2.0 * (d[i - 1] + d[i]);
    c[i + 1] = (y[i + 1] - y[i]) / d[i];
    c[i] = c[i + 1] - c[i];
  }
  b[1] = -d[1]; b[n] = -d[nm1]; c[1] = c[n] = 0.0;
  if (n > 3) {
    c[1] = c[3] / (x[4] - x[2]) - c[2] / (x[3] - x[1]);
    c[n] = c[nm1] / (x[n] - x[n - 2]) - c[n - 2] / (x[nm1] - x[n - 3]);
    c[1] = c[1] * d[1] * d[1] / (x[4] - x[1]);
    c[n] = -c[n] * d[nm1] * d[nm1] / (x[n] - x[n - 3]);
  }
  for (i = 2; i <= n; i++) { t = d[i - 1] / b[i - 1]; b[i] = b[i] - t * d[i - 1]; c[i] = c[i] - t * c[i - 1]; }
  c[n] = c[n] / b[n];
  for (i = nm1; i >= 1; i--) c[i] = (c[i] - d[i] * c[i + 1]) / b[i];
  b[n] = (y[n] - y[n - 1]) / d[n - 1] + d[n - 1] * (c[n - 1] + 2.0 * c[n]);
  for (i = 1; i <= nm1; i++) {
    b[i] = (y[i + 1] - y[i]) / d[i] - d[i] * (c[i + 1] + 2.0 * c[i]);
    d[i] = (c[i + 1] - c[i]) / d[i];
    c[i] = 3.0 * c[i];
  }
  c[n] = 3.0 * c[n]; d[n] = d[nm1];
  return s;
}
static void spl_eval(const spl_t* s, const double* u, double* v, int64_t nu) {
  const int64_t n_1 = s->n - 1; int64_t i = 0;
  for (int64_t l = 0; l < nu; l++) {
    double ul = u[l];
    if (ul < s->x[i] || (i < n_1 && s->x[i + 1] < ul)) {
      i = 0; int64_t j = s->n;
      do { int64_t k = (i + j) / 2; if (ul < s->x[k]) j = k; else i = k; } while (j > i + 1);
    }
    double dx = ul - s->x[i];
    v[l] = s->y[i] + dx * (s->b[i] + dx * (s->c[i] + dx * s->d[i]));
  }
}
/* spline(x, y, n): xout = seq.int(min(x), max(x), length.out = n) */
static dv r_spline(const double* x, const double* y, int64_t nx, int64_t n) {
  spl_t s = fmm_coef(x, y, nx);
  dv xo = r_seqint_len(x[0], x[nx - 1], n);
  dv out = dv_new(n);
  spl_eval(&s, xo.v, out.v, n);
  dv_free(&xo); spl_free(&s);
  return out;
}
/* ---- approx() linear, rule = 1 — stats/src/approx.c ---- */
static double approx1(double v, const double* x, const double* y, int64_t n) {
  int64_t i = 0, j = n - 1;
  if (v < x[i] || v > x[j]) return NAN;
  while (i < j - 1) { int64_t ij = (i + j) / 2; if (v < x[ij]) j = ij; else i = ij; }
  if (v == x[j]) return y[j];
  if (v == x[i]) return y[i];
  return y[i] + (y[j] - y[i]) * ((v - x[i]) / (x[j] - x[i]));
}
static int r_approx_n(const double* x, const double* y, int64_t nx, int64_t n, dv* out) {
  if (nx <= 1) return fail(SG_E_DOMAIN, "approx: need at least two non-NA values to interpolate");
  dv xo = r_seqint_len(x[0], x[nx - 1], n);
  *out = dv_new(n);
  for (int64_t l = 0; l < n; ++l) out->v[l] = approx1(xo.v[l], x, y, nx);
  dv_free(&xo);
  return 0;
}

/* ------------------------------------------------------------ loess (1-D)
 * loess(y ~ x, span = f) then predict(., newx) with R 3.4 stats defaults:
 * degree 2, family "gaussian" (no robustness iterations), surface
 * "interpolate", statistics "approximate", cell 0.2. Restated from the
 * published netlib dloess algorithm that R's stats/src/loessf.f carries
 * (lowesd, lowesb -> ehg131: ehg126 bounding box, ehg124 k-d tree, ehg139/ehg127
 * vertex fits; lowese -> ehg133/ehg128 cubic Hermite interpolation) and
 * loessc.c (nf, span * cell). PARITY UNPINNED: R is absent here; this follows
 * the algorithm as published, not R output. x ascending, distinct. */
typedef struct {
  int n;              /* data points */
  double vx[64];      /* vertices (creation order) */
  double val[64], slope[64];
  int nv;
  /* cells (BFS order): point range [l, u] (1-based), vertex ids, split */
  int cl[128], cu[128], cv0[128], cv1[128], split[128], lo_son[128], hi_son[128];
  double xi[128];
  int nc;
} lo_tree;

/* one-sided Jacobi SVD of B (m x 3, column-major in b[3][m]) -> sigma, V */
static void svd3(double b[3][16], int m, double sigma[3], double V[3][3]) {
  for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) V[i][j] = i == j;
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0;
    for (int p = 0; p < 2; ++p)
      for (int q = p + 1; q < 3; ++q) {
        double al = 0, be = 0, ga = 0;
        for (int i = 0; i < m; ++i) { al += b[p][i] * b[p][i]; be += b[q][i] * b[q][i]; ga += b[p][i] * b[q][i]; }
        if (ga == 0 || fabs(ga) <= 1e-300) continue;
        off = fmax(off, fabs(ga) / sqrt(al * be));
        const double zeta = (be - al) / (2 * ga);
        const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1 + zeta * zeta));
        const double c = 1 / sqrt(1 + t * t), sn = c * t;
        for (int i = 0; i < m; ++i) {
          const double bp = b[p][i], bq = b[q][i];
          b[p][i] = c * bp - sn * bq;
          b[q][i] = sn * bp + c * bq;
        }
        for (int i = 0; i < 3; ++i) {
          const double vp = V[i][p], vq = V[i][q];
          V[i][p] = c * vp - sn * vq;
          V[i][q] = sn * vp + c * vq;
        }
      }
    if (off < 1e-15) break;
  }
  for (int j = 0; j < 3; ++j) {
    double s2 = 0;
    for (int i = 0; i < m; ++i) s2 += b[j][i] * b[j][i];
    sigma[j] = sqrt(s2);
  }
}

/* lo_build / lo_vertex_fit: the fit has a NaN vertex (not an error code) */
#define LO_ZERO_WIDTH 1

/* local quadratic fit at vertex v (ehg127): value and slope */
static int lo_vertex_fit(const double* x, const double* y, int n, int nf, double f, double v, double* val,
                         double* slope) {
  double d2[64]; int ord[64];
  for (int i = 0; i < n; ++i) { d2[i] = (x[i] - v) * (x[i] - v); ord[i] = i; }
  for (int i = 1; i < n; ++i)  /* stable insertion sort by distance */
    for (int j = i; j > 0 && d2[ord[j]] < d2[ord[j - 1]]; --j) { int t = ord[j]; ord[j] = ord[j - 1]; ord[j - 1] = t; }
  const double rho = d2[ord[nf - 1]] * (f > 1 ? f : 1.0);
  /* rho = 0 (a vertex on a data point with floor(n f) = 1): the tricube
   * weights are 0/0, so the vertex value is NaN. loess() itself returns;
   * predict()'s .C(C_loess_ifit, ..., vval) then stops on the NaN (NAOK is
   * FALSE), which is the try-error smooth_loess retries with span + 0.1. */
  if (!(rho > 0)) return LO_ZERO_WIDTH;
  double b[3][16], eta[16];
  const int m = nf < 3 ? 3 : nf;
  for (int i = 0; i < m; ++i) { b[0][i] = b[1][i] = b[2][i] = 0; eta[i] = 0; }
  for (int i = 0; i < nf; ++i) {
    const int k = ord[i];
    double w = sqrt(d2[k] / rho);
    w = sqrt((1 - w * w * w) * (1 - w * w * w) * (1 - w * w * w));
    const double dx = x[k] - v;
    b[0][i] = w; b[1][i] = w * dx; b[2][i] = w * dx * dx;
    eta[i] = w * y[k];
  }
  double colnor[3];
  for (int j = 0; j < 3; ++j) {  /* equilibrate columns */
    double sc = 0;
    for (int i = 0; i < m; ++i) sc += b[j][i] * b[j][i];
    sc = sqrt(sc);
    if (sc > 0) { for (int i = 0; i < m; ++i) b[j][i] /= sc; colnor[j] = sc; } else colnor[j] = 1;
  }
  double bw[3][16];
  memcpy(bw, b, sizeof b);
  double sigma[3], V[3][3];
  svd3(bw, m, sigma, V);
  double smax = fmax(sigma[0], fmax(sigma[1], sigma[2]));
  const double tol = smax * (100 * DBL_EPSILON);
  double gam[3];
  for (int j = 0; j < 3; ++j) {  /* gamma_j = u_j . eta / sigma_j, u_j = (B V)_j / sigma_j */
    if (sigma[j] > tol) {
      double ue = 0;
      for (int i = 0; i < m; ++i) ue += bw[j][i] / sigma[j] * eta[i];
      gam[j] = ue / sigma[j];
    } else gam[j] = 0;
  }
  double s0 = 0, s1 = 0;
  for (int j = 0; j < 3; ++j) { s0 += V[0][j] * gam[j]; s1 += V[1][j] * gam[j]; }
  *val = s0 / colnor[0];
  *slope = s1 / colnor[1];
  return 0;
}

static int lo_build(const double* x, const double* y, int n, double f, lo_tree* T) {
  if (n < 1 || n > 48) return fail(SG_E_UNSUPPORTED, "loess: 1..48 points");
  if (floor(n * f + 1e-5) <= 0) return fail(SG_E_DOMAIN, "loess: span is too small");
  const int nf = (int)fmin((double)n, floor(n * f));
  if (nf <= 0) return fail(SG_E_DOMAIN, "loess: span is too small");
  const int fc = (int)floor(n * (f * 0.2));
  double alpha = x[0], beta = x[0];
  for (int i = 1; i < n; ++i) { alpha = fmin(alpha, x[i]); beta = fmax(beta, x[i]); }
  const double mu = 0.005 * fmax(beta - alpha, 1e-10 * fmax(fabs(alpha), fabs(beta)) + 1e-30);
  T->n = n; T->nv = 2; T->vx[0] = alpha - mu; T->vx[1] = beta + mu;
  T->nc = 1; T->cl[0] = 1; T->cu[0] = n; T->cv0[0] = 0; T->cv1[0] = 1;
  for (int p = 0; p < T->nc; ++p) {
    const int l = T->cl[p], u = T->cu[p];
    int leaf = (u - l + 1) <= fc || (T->vx[T->cv1[p]] - T->vx[T->cv0[p]]) <= 0;
    int m = (l + u) / 2;
    if (!leaf) {
      /* ties go to the high son: step m to a position where x changes */
      int off = 0;
      while (!(m + off >= u || m + off < l)) {
        if (x[m + off - 1] == x[m + off]) { off = -off; if (off >= 0) off++; }
        else { m += off; break; }
      }
      leaf = T->vx[T->cv0[p]] == x[m - 1] || T->vx[T->cv1[p]] == x[m - 1];
    }
    T->split[p] = !leaf;
    if (leaf) continue;
    if (T->nc + 2 > 128 || T->nv + 1 > 64) return fail(SG_E_UNSUPPORTED, "loess: k-d tree too large");
    T->xi[p] = x[m - 1];
    const int vn = T->nv++;
    T->vx[vn] = x[m - 1];
    const int a = T->nc++, b = T->nc++;
    T->lo_son[p] = a; T->hi_son[p] = b;
    T->cl[a] = l; T->cu[a] = m; T->cv0[a] = T->cv0[p]; T->cv1[a] = vn;
    T->cl[b] = m + 1; T->cu[b] = u; T->cv0[b] = vn; T->cv1[b] = T->cv1[p];
  }
  int nan_vertex = 0;
  for (int v = 0; v < T->nv; ++v) {
    const int rc = lo_vertex_fit(x, y, n, nf, f, T->vx[v], &T->val[v], &T->slope[v]);
    if (rc == LO_ZERO_WIDTH) { T->val[v] = T->slope[v] = NAN; nan_vertex = 1; }
    else if (rc) return rc;
  }
  return nan_vertex ? LO_ZERO_WIDTH : 0;
}

static double lo_eval(const lo_tree* T, double z) {
  int p = 0;
  while (T->split[p]) p = z <= T->xi[p] ? T->lo_son[p] : T->hi_son[p];
  const int a = T->cv0[p], b = T->cv1[p];
  const double v0 = T->vx[a], v1 = T->vx[b];
  const double h = (z - v0) / (v1 - v0);
  const double phi0 = (1 - h) * (1 - h) * (1 + 2 * h), phi1 = h * h * (3 - 2 * h);
  const double psi0 = h * (1 - h) * (1 - h), psi1 = -h * h * (1 - h);
  return phi0 * T->val[a] + phi1 * T->val[b] + (psi0 * T->slope[a] + psi1 * T->slope[b]) * (v1 - v0);
}

/* the loess branch of getSmoothContour(), R/smoothContours.R:119-154:
 * anchors (t in [0, 1], values) -> contour over 1..len */
static int smooth_loess(const double* t, const double* val, int64_t n, int64_t len, double duration_ms,
                        int has_floor, double vfloor, double* out) {
  if (n > 48) return fail(SG_E_UNSUPPORTED, "loess: too many anchors");
  /* anchors_long[anchor_time_points] = value: positions truncate, 0 drops, last wins */
  double xv[48], yv[48]; int nx = 0;
  for (int64_t i = 0; i < n; ++i) {
    double tp = t[i] / 1.0 * (double)len;  /* (t - min) / max * len with t already in [0, 1] */
    if (tp == 0) tp = 1;
    const int64_t idx = (int64_t)tp;
    if (idx < 1 || idx > len) continue;
    int k = 0;
    while (k < nx && xv[k] != (double)idx) ++k;
    if (k == nx) { xv[nx] = (double)idx; yv[nx] = val[i]; ++nx; } else yv[k] = val[i];
  }
  for (int i = 1; i < nx; ++i)  /* data frame rows in time order */
    for (int j = i; j > 0 && xv[j] < xv[j - 1]; --j) {
      double a = xv[j]; xv[j] = xv[j - 1]; xv[j - 1] = a;
      a = yv[j]; yv[j] = yv[j - 1]; yv[j - 1] = a;
    }
  double span = (1 / (1 + exp(duration_ms / 500)) + 0.5) / pow(1.1, (double)(n - 3));
  /* smoothContour = try(predict(l, time)); while (try-error) span = span + 0.1
   * (R/smoothContours.R:133-143). RESTATED, UNPINNED: that predict() fails
   * exactly when a vertex value is NaN (LO_ZERO_WIDTH) follows from .C's NAOK
   * rule, not from R output. */
  for (int k = 0;; ++k) {
    lo_tree T;
    const int rc = lo_build(xv, yv, nx, span, &T);
    if (rc != LO_ZERO_WIDTH) { if (rc) return rc; break; }
    if (k == 200) return fail(SG_E_DOMAIN, "loess: no span gives a finite fit");
    span = span + 0.1;
  }
  for (int iter = 0; iter < 200; ++iter) {
    lo_tree T;
    int rc = lo_build(xv, yv, nx, span, &T);
    /* a zero-width fit inside the valueFloor loop would leave R comparing a
     * try-error string against valueFloor: not restated */
    if (rc == LO_ZERO_WIDTH) return fail(SG_E_UNSUPPORTED, "loess: zero-width fit inside the valueFloor refits");
    if (rc) return rc;
    int below = 0;
    for (int64_t k = 0; k < len; ++k) {
      const double z = (double)(k + 1);
      out[k] = (z < xv[0] || z > xv[nx - 1]) ? NAN : lo_eval(&T, z);
      if (has_floor && out[k] < vfloor - 1e-6) below = 1;
    }
    if (!below) return 0;
    span = span / 1.1;  /* less smoothing until no value falls below the floor */
  }
  return fail(SG_E_DOMAIN, "loess: contour stays below valueFloor");
}

/* ------------------------------------------------------- soundgen helpers */
static double HzToSemitones(double h) { return log2(h / 16.3516) * 12; }
static double semitonesToHz(double s) { return 16.3516 * pow(2.0, s / 12); }

/* getSmoothContour(), R/smoothContours.R:53-227 (len given). Returns 1 with
 * out->n == 0 for R's NA. method: 0 = loess(default), 1 = spline. */
static int get_smooth_contour(sg_anchors an, int64_t len, int thisIsPitch,
                              int method, int has_floor, double vfloor,
                              int has_ceil, double vceil, double sr, dv* out) {
  out->v = NULL; out->n = 0;
  if (an.n <= 0) return 0;                      /* NA anchors */
  int64_t n = an.n;
  if (n > 10 && method == 0) method = 1;
  dv t = dv_copy(an.time, n), val = dv_copy(an.value, n);
  if (has_floor) for (int64_t i = 0; i < n; ++i) if (val.v[i] < vfloor) val.v[i] = vfloor;
  if (has_ceil) for (int64_t i = 0; i < n; ++i) if (val.v[i] > vceil) val.v[i] = vceil;
  if (thisIsPitch) {
    for (int64_t i = 0; i < n; ++i) val.v[i] = HzToSemitones(val.v[i]);
    if (has_floor) vfloor = HzToSemitones(vfloor);
    if (has_ceil) vceil = HzToSemitones(vceil);
  }
  /* R/smoothContours.R:92-101: len = NULL (here len < 0) keeps the times in ms,
   * len = floor(duration_ms sr / 1000); a given len rescales them to 0..1 */
  double dur_ms = (double)len / sr * 1000;
  dv traw = dv_copy(t.v, n);
  const int len_null = len < 0;
  if (len_null) {
    dur_ms = r_max(t.v, n) - r_min(t.v, n);
    len = (int64_t)floor(dur_ms * sr / 1000);
    if (!(dur_ms != 0)) len = 0;
  }
  double tmin = r_min(t.v, n);
  for (int64_t i = 0; i < n; ++i) t.v[i] -= tmin;
  double tmax = r_max(t.v, n);
  for (int64_t i = 0; i < n; ++i) t.v[i] /= tmax;
  if (len <= 0) { dv_free(&t); dv_free(&val); dv_free(&traw); return 0; }
  int rc = 0;
  if (n == 1) {
    *out = dv_new(len); for (int64_t i = 0; i < len; ++i) out->v[i] = val.v[0];
  } else if (n == 2) {
    *out = r_seq_len(val.v[0], val.v[1], len);
  } else {
    if (method != 1) {
      *out = dv_new(len);
      rc = smooth_loess(t.v, val.v, n, len, dur_ms, has_floor, vfloor, out->v);
      if (rc) { dv_free(out); out->n = 0; goto done; }
    } else {
      *out = r_spline(len_null ? traw.v : t.v, val.v, n, len);
    }
    for (int64_t i = 0; i < len; ++i) {
      if (has_floor && out->v[i] < vfloor) out->v[i] = vfloor;
      if (has_ceil && out->v[i] > vceil) out->v[i] = vceil;
    }
  }
  for (int64_t i = 0; i < out->n; ++i) if (isnan(out->v[i])) out->v[i] = 0;
  if (thisIsPitch) for (int64_t i = 0; i < out->n; ++i) out->v[i] = semitonesToHz(out->v[i]);
done:
  dv_free(&t); dv_free(&val); dv_free(&traw);
  return rc;
}

/* getGlottalCycles(), R/utilities_soundgen.R:477-486 — 1-based indices */
static dv get_glottal_cycles(const double* pitch, int64_t len, double psr) {
  dv gc = dv_new(0);
  double i = 1;
  while (i < len) {
    dv_append(&gc, &i, 1);
    double st = floor(psr / pitch[(int64_t)i - 1]);
    i = i + (st > 2 ? st : 2);
  }
  return gc;
}

/* zeroOne(), R/utilities_math.R:58-61 */
static void zero_one(double* x, int64_t n) {
  double mn = r_min(x, n); for (int64_t i = 0; i < n; ++i) x[i] -= mn;
  double mx = r_max(x, n); for (int64_t i = 0; i < n; ++i) x[i] /= mx;
}

/* getRandomWalk(), R/utilities_math.R:289-326. method 0 linear, 1 spline.
 * trend: n_trend values. trend_lazy_rnorm: trend = rnorm(1) evaluated lazily
 * (R/sourceSpectrum.R:405) — drawn only when len >= 2. */
static int get_random_walk(rng_t* r, int64_t len, double rw_range, double rw_smoothing,
                           int method, const double* trend, int n_trend, int trend_lazy_rnorm, dv* out) {
  if (len < 2) {
    double g; int rc = r_rgamma1(r, 1.0 / (rw_range * rw_range), 1.0 / (rw_range * rw_range), &g);
    if (rc) return rc;
    *out = dv_new(1); out->v[0] = g; return 0;
  }
  double tr_lazy;
  if (trend_lazy_rnorm) { int rc = r_rnorm1(r, 0.0, 1.0, &tr_lazy); if (rc) return rc; trend = &tr_lazy; n_trend = 1; }
  double p = pow(2.0, 1.0 / rw_smoothing);
  double nd = floor(p > 2 ? p : 2);
  dv tshort = dv_new(0);
  if (n_trend > 1) {
    nd = r_round(nd / 2) * 2;
    int64_t each = (int64_t)(nd / n_trend);
    for (int k = 0; k < n_trend; ++k) for (int64_t e = 0; e < each; ++e) dv_append(&tshort, &trend[k], 1);
  } else {
    dv_append(&tshort, trend, 1);
  }
  dv rw_long; int rc = 0;
  if (nd > (double)len) {
    dv z = dv_new(len);
    for (int64_t i = 0; i < len; ++i) { rc = r_rnorm1(r, tshort.v[i % tshort.n], 1.0, &z.v[i]); if (rc) { dv_free(&z); dv_free(&tshort); return rc; } }
    rw_long = dv_new(len); r_cumsum(z.v, rw_long.v, len); dv_free(&z);
  } else {
    int64_t n = (int64_t)nd;
    dv z = dv_new(n);
    for (int64_t i = 0; i < n; ++i) { rc = r_rnorm1(r, tshort.v[i % tshort.n], 1.0, &z.v[i]); if (rc) { dv_free(&z); dv_free(&tshort); return rc; } }
    dv rs = dv_new(n); r_cumsum(z.v, rs.v, n); dv_free(&z);
    dv xs = dv_new(n); for (int64_t i = 0; i < n; ++i) xs.v[i] = (double)(i + 1);
    if (method == 0) { rc = r_approx_n(xs.v, rs.v, n, len, &rw_long); }
    else rw_long = r_spline(xs.v, rs.v, n, len);
    dv_free(&rs); dv_free(&xs);
    if (rc) { dv_free(&tshort); return rc; }
  }
  dv_free(&tshort);
  double mn = r_min(rw_long.v, len);
  for (int64_t i = 0; i < len; ++i) rw_long.v[i] -= mn;
  double mx = 0; for (int64_t i = 0; i < len; ++i) { double a = fabs(rw_long.v[i]); if (a > mx || isnan(a)) mx = a; }
  for (int64_t i = 0; i < len; ++i) rw_long.v[i] = rw_long.v[i] / mx * rw_range;
  *out = rw_long;
  return 0;
}

/* clumper(), R/utilities_math.R:555-600 (s: values, minLength vector or scalar) */
static int cmp_dbl(const void* a, const void* b) { double x = *(const double*)a, y = *(const double*)b; return (x > y) - (x < y); }
static void clumper(double* s, int64_t n, const double* minLen_in, int64_t nml) {
  double mlmax = r_max(minLen_in, nml);
  if (mlmax < 2) return;
  dv ml = dv_new(nml); for (int64_t i = 0; i < nml; ++i) ml.v[i] = r_round(minLen_in[i]);
  int nuniq = 1; for (int64_t i = 1; i < n; ++i) { int seen = 0; for (int64_t j = 0; j < i; ++j) if (s[j] == s[i]) { seen = 1; break; } if (!seen) { nuniq = 2; break; } }
  if (nuniq < 2 || (nml == 1 && n < ml.v[0]) || n < ml.v[0]) {
    dv tmp = dv_copy(s, n); qsort(tmp.v, n, sizeof(double), cmp_dbl);
    double med = (n % 2) ? tmp.v[n / 2] : (tmp.v[n / 2 - 1] + tmp.v[n / 2]) / 2.0;
    double rm = r_round(med); for (int64_t i = 0; i < n; ++i) s[i] = rm;
    dv_free(&tmp); dv_free(&ml); return;
  }
  if (nml == 1 || nml != n) { double v0 = ml.v[0]; dv_free(&ml); ml = dv_new(n); for (int64_t i = 0; i < n; ++i) ml.v[i] = (nml == 1) ? v0 : minLen_in[i % nml]; for (int64_t i = 0; i < n; ++i) ml.v[i] = r_round(ml.v[i]); }
  double c = 0;
  for (int64_t i = 1; i < n; ++i) {
    if (s[i - 1] == s[i]) c = c + 1;
    else if (c < ml.v[i]) { s[i] = s[i - 1]; c = c + 1; }
    else c = 1;
  }
  double mlast = ml.v[n - 1];
  int64_t lo = (int64_t)((double)n - mlast + 1); if (lo < 2) lo = 2; /* 1-based */
  int64_t cnt = 0; for (int64_t k = lo; k <= n; ++k) if (s[k - 1] == s[n - 1]) cnt++;
  if ((double)cnt < mlast) {
    int64_t nidx = n - lo + 1;                 /* idx = rev(idx_min) */
    int64_t* idx = (int64_t*)malloc(nidx * sizeof(int64_t));
    for (int64_t k = 0; k < nidx; ++k) idx[k] = n - k;
    double cc = 1; int64_t ii = 2;
    while (ii <= nidx && s[idx[ii - 1] - 1] == s[idx[ii - 1] - 2] && ii < nidx) { cc++; ii++; }
    if (cc < mlast) { double v = s[lo - 1]; for (int64_t k = 0; k < nidx; ++k) s[idx[k] - 1] = v; }
    free(idx);
  }
  dv_free(&ml);
}

/* noiseThresholdsDict, data-raw/noiseThresholdsDict.R */
static double noise_q(int which, double nonlinBalance) {
  int64_t k = (int64_t)(nonlinBalance + 1) - 1; /* R truncates the index */
  double mid = which == 1 ? 33 : 66;
  return 100 / (1 + exp(0.1 * ((double)k - mid)));
}

OR_API double or_noise_threshold(int which, double nonlinBalance) { return noise_q(which, nonlinBalance); }

/* getIntegerRandomWalk(), R/utilities_math.R:352-387 */
static void get_integer_random_walk(const double* rw, int64_t len, double nonlinBalance,
                                    const double* minLength, double* out) {
  if (nonlinBalance == 0) { for (int64_t i = 0; i < len; ++i) out[i] = 0; return; }
  if (nonlinBalance == 100) { for (int64_t i = 0; i < len; ++i) out[i] = 2; return; }
  double q1 = noise_q(1, nonlinBalance), q2 = noise_q(2, nonlinBalance);
  for (int64_t i = 0; i < len; ++i) { out[i] = 0; if (rw[i] > q1) out[i] = 1; if (rw[i] > q2) out[i] = 2; }
  clumper(out, len, minLength, len);
}

/* getRolloff(), R/sourceSpectrum.R:71-186. Vector parameters are per gc.
 * out: nH x nGC col-major buffer; returns kept rows in *H (compacted). */
static int get_rolloff(const double* pitch, int64_t nGC, int64_t nH,
                       const double* rolloff, const double* rolloffOct,
                       double rolloffParab, double rolloffParabHarm, double rolloffParabCeiling,
                       const double* rolloffKHz, double baseline, double throwaway,
                       double sr, dv* out, int64_t* H) {
  if (nH < 1) return fail(SG_E_DOMAIN, "getRolloff: nHarmonics < 1");
  dv r = dv_new(nH * nGC);
#define R_(h, g) r.v[(g) * nH + (h)]
  int anyOct = 0; for (int64_t g = 0; g < nGC; ++g) if (rolloffOct[g] != 0) anyOct = 1;
  for (int64_t h = 0; h < nH; ++h)
    for (int64_t g = 0; g < nGC; ++g) {
      double hh = (double)(h + 1);
      double delta = (anyOct && h >= 1) ? rolloffOct[g] * (pitch[g] * hh - baseline) / 1000 : 0.0;
      double v = ((rolloff[g] + rolloffKHz[g] * (pitch[g] - baseline) / 1000) * log2(hh)) + delta;
      if (hh * pitch[g] >= sr / 2) v = -INFINITY;
      R_(h, g) = v;
    }
  if (rolloffParab != 0) {
    for (int64_t g = 0; g < nGC; ++g) {
      /* R/sourceSpectrum.R:104-110: a ceiling sets the count per gc */
      double rph = isnan(rolloffParabCeiling) ? r_round(rolloffParabHarm) : r_round(rolloffParabCeiling / pitch[g]);
      if (rph == 2) rph = 3;
      double a = -4 * rolloffParab / ((rph - 1) * (rph - 1));
      double b = -a * (1 + rph), c = a * rph;
      if (rph < 3) { if (rph < 2) R_(0, g) = R_(0, g) + rolloffParab; }
      else {
        if (rph > nH) { dv_free(&r); return fail(SG_E_DOMAIN, "getRolloff: subscript out of bounds (rolloffParabHarm > nHarmonics)"); }
        for (int64_t k = 1; k <= (int64_t)rph; ++k) R_(k - 1, g) = R_(k - 1, g) + a * k * k + b * k + c;
      }
    }
  }
  for (int64_t i = 0; i < nH * nGC; ++i) if (r.v[i] < throwaway) r.v[i] = -INFINITY;
  for (int64_t g = 0; g < nGC; ++g) {
    double mx = -INFINITY; for (int64_t h = 0; h < nH; ++h) if (R_(h, g) > mx) mx = R_(h, g);
    for (int64_t h = 0; h < nH; ++h) R_(h, g) = R_(h, g) - mx;
  }
  for (int64_t i = 0; i < nH * nGC; ++i) r.v[i] = pow(2.0, r.v[i] / 10);
  int64_t k = 0;
  dv o = dv_new(nH * nGC);
  for (int64_t h = 0; h < nH; ++h) {
    long double s = 0; for (int64_t g = 0; g < nGC; ++g) s += R_(h, g);
    if ((double)s > 0) { for (int64_t g = 0; g < nGC; ++g) o.v[g * nH + k] = R_(h, g); k++; }
  }
#undef R_
  /* compact to k rows */
  dv c2 = dv_new(k * nGC);
  for (int64_t g = 0; g < nGC; ++g) for (int64_t h = 0; h < k; ++h) c2.v[g * k + h] = o.v[g * nH + h];
  dv_free(&o); dv_free(&r);
  *out = c2; *H = k;
  return 0;
}

/* An amplitude matrix with row multipliers (times_f0 from rownames). */
typedef struct { dv A; int64_t nrow, ncol; dv mult; } ampmat;
static void ampmat_free(ampmat* m) { dv_free(&m->A); dv_free(&m->mult); }

static double rowname_num(double x) { /* as.numeric(as.character(x)): 15 significant digits */
  char buf[64]; snprintf(buf, sizeof buf, "%.15g", x); return strtod(buf, NULL);
}

/* getVocalFry_per_epoch(), R/subharmonics.R:25-86 */
static void vocal_fry_per_epoch(const double* roll, int64_t H, int64_t ncol, const double* pitch,
                                int64_t nSub, const double* sbw, double throwaway01, ampmat* res) {
  if (nSub < 1) {
    res->A = dv_copy(roll, H * ncol); res->nrow = H; res->ncol = ncol;
    res->mult = dv_new(H); for (int64_t h = 0; h < H; ++h) res->mult.v[h] = (double)(h + 1);
    return;
  }
  dv gseq = r_seq_by(0, (double)(H + 1), 1.0 / (double)(nSub + 1));
  int64_t nr = gseq.n;
  dv rn = dv_new(nr * ncol);
#define RN(i, g) rn.v[(g) * nr + (i)]
  for (int64_t i = 0; i < nr * ncol; ++i) rn.v[i] = NAN;
  for (int64_t g = 0; g < ncol; ++g) { RN(0, g) = 0; RN(nr - 1, g) = 0; }
  /* match(rownames(rolloff), rownames(rolloff_new)) */
  char a[64], b[64];
  for (int64_t h = 0; h < H; ++h) {
    snprintf(a, sizeof a, "%.15g", (double)(h + 1));
    for (int64_t i = 0; i < nr; ++i) {
      snprintf(b, sizeof b, "%.15g", gseq.v[i]);
      if (strcmp(a, b) == 0) { for (int64_t g = 0; g < ncol; ++g) RN(i, g) = roll[g * H + h]; break; }
    }
  }
  /* multipliers: dnorm(d, 0, sd)/dnorm(0, 0, sd) */
  dv ml = dv_new(nSub * ncol);
  for (int64_t s = 1; s <= nSub; ++s)
    for (int64_t g = 0; g < ncol; ++g) {
      double d = pitch[g] * (double)s / (double)(nSub + 1), sd = sbw[g], v;
      if (sd == 0) v = (d == 0) ? NAN : 0.0;
      else v = exp(-0.5 * (d / sd) * (d / sd));
      ml.v[(s - 1) * ncol + g] = v;
    }
  for (int64_t block = 1; block <= H + 1; ++block) {
    int64_t row_lwr = 1 + (block - 1) * (nSub + 1);
    int64_t row_upr = row_lwr + nSub + 1;
    double Alin = rn.v[row_lwr - 1], Blin = rn.v[row_upr - 1];  /* linear index: column 1 */
    for (int64_t gg = 1; gg <= nSub; ++gg) {
      int64_t row = row_lwr + gg;  /* g_idx[gg] */
      for (int64_t g = 0; g < ncol; ++g)
        RN(row - 1, g) = Alin * ml.v[(gg - 1) * ncol + g] + Blin * ml.v[(nSub - gg) * ncol + g];
    }
  }
  for (int64_t i = 0; i < nr * ncol; ++i) if (rn.v[i] < throwaway01) rn.v[i] = 0;
  int64_t k = 0;
  res->A = dv_new(nr * ncol); res->mult = dv_new(nr);
  dv keep = dv_new(nr);
  for (int64_t i = 0; i < nr; ++i) {
    long double s = 0; for (int64_t g = 0; g < ncol; ++g) s += RN(i, g);
    keep.v[i] = ((double)s > 0) ? 1 : 0;
  }
  for (int64_t i = 0; i < nr; ++i) if (keep.v[i] != 0) {
    for (int64_t g = 0; g < ncol; ++g) res->A.v[g * nr + k] = RN(i, g);
    res->mult.v[k] = rowname_num(gseq.v[i]); k++;
  }
#undef RN
  dv A2 = dv_new(k * ncol);
  for (int64_t g = 0; g < ncol; ++g) for (int64_t h = 0; h < k; ++h) A2.v[g * k + h] = res->A.v[g * nr + h];
  dv_free(&res->A); res->A = A2; res->nrow = k; res->ncol = ncol; res->mult.n = k;
  dv_free(&keep); dv_free(&ml); dv_free(&rn); dv_free(&gseq);
}

/* getVocalFry(), R/subharmonics.R:108-163 → epochs (1-based start,end) */
static int get_vocal_fry(const double* roll, int64_t H, const double* pitch, int64_t nGC,
                         const double* subFreq, const double* subDep_in, double throwaway,
                         double shortestEpoch, ampmat** mats, int64_t** starts, int64_t** ends, int64_t* nEp) {
  dv nsub = dv_new(nGC);
  double mx = -INFINITY;
  for (int64_t g = 0; g < nGC; ++g) { double v = r_round(pitch[g] / subFreq[g]) - 1; if (v < 0) v = 0; nsub.v[g] = v; if (v > mx) mx = v; }
  if (mx < 1) {
    *nEp = 1; *mats = (ampmat*)calloc(1, sizeof(ampmat));
    (*mats)[0].A = dv_copy(roll, H * nGC); (*mats)[0].nrow = H; (*mats)[0].ncol = nGC;
    (*mats)[0].mult = dv_new(H); for (int64_t h = 0; h < H; ++h) (*mats)[0].mult.v[h] = (double)(h + 1);
    *starts = (int64_t*)malloc(sizeof(int64_t)); *ends = (int64_t*)malloc(sizeof(int64_t));
    (*starts)[0] = 1; (*ends)[0] = nGC; dv_free(&nsub); return 0;
  }
  double throwaway01 = pow(2.0, throwaway / 10);
  dv minlen = dv_new(nGC);
  for (int64_t g = 0; g < nGC; ++g) { double period_ms = 1000 / pitch[g]; minlen.v[g] = r_round(shortestEpoch / period_ms); }
  if (nGC > 1) clumper(nsub.v, nGC, minlen.v, nGC);
  int64_t ne = 1; for (int64_t g = 1; g < nGC; ++g) if (nsub.v[g] != nsub.v[g - 1]) ne++;
  *nEp = ne; *mats = (ampmat*)calloc(ne, sizeof(ampmat));
  *starts = (int64_t*)malloc(ne * sizeof(int64_t)); *ends = (int64_t*)malloc(ne * sizeof(int64_t));
  int64_t e = 0; (*starts)[0] = 1;
  for (int64_t g = 1; g < nGC; ++g) if (nsub.v[g] != nsub.v[g - 1]) { (*ends)[e] = g; e++; (*starts)[e] = g + 1; }
  (*ends)[ne - 1] = nGC;
  for (e = 0; e < ne; ++e) {
    int64_t s0 = (*starts)[e] - 1, s1 = (*ends)[e] - 1, nc = s1 - s0 + 1;
    double ns = nsub.v[s1];
    vocal_fry_per_epoch(roll + s0 * H, H, nc, pitch + s0, (int64_t)ns, subDep_in + s0, throwaway01, &(*mats)[e]);
  }
  dv_free(&nsub); dv_free(&minlen);
  return 0;
}

/* findZeroCrossing(), R/utilities_soundgen.R:255-295 (1-based; 0 = NA) */
static int64_t find_zero_crossing(const double* a, int64_t len, int64_t location) {
  if (len < 1 || location < 1 || location > len) return 0;
  if (len == 1 && location == 1) return location;
  int64_t zl = 0, zr = 0, i = 0;
  if (location > 1) {
    i = location;
    while (i > 1) { if (a[i - 1] > 0 && a[i - 2] < 0) { zl = i - 1; break; } i = i - 1; }
  }
  if (location < len) i = location;
  while (i < (len - 1)) { if (a[i] > 0 && a[i - 1] < 0) { zr = i; break; } i = i + 1; }
  if (!zl && !zr) return 0;
  if (!zl) return zr;
  if (!zr) return zl;
  return (llabs(zl - location) <= llabs(zr - location)) ? zl : zr;
}

/* crossFade(), R/utilities_soundgen.R:328-375 */
static dv cross_fade(dv a1, dv a2, double sr, double crossLen) {
  int64_t zc1 = find_zero_crossing(a1.v, a1.n, a1.n);
  dv A1, A2;
  if (zc1) { A1 = dv_copy(a1.v, zc1); dv_append_zeros(&A1, 1); } else A1 = dv_copy(a1.v, a1.n);
  int64_t zc2 = find_zero_crossing(a2.v, a2.n, 1);
  if (zc2) A2 = dv_copy(a2.v + zc2, a2.n - zc2); else A2 = dv_copy(a2.v, a2.n);
  double cl = floor(crossLen * sr / 1000);
  if ((double)(A1.n - 1) < cl) cl = (double)(A1.n - 1);
  if ((double)(A2.n - 1) < cl) cl = (double)(A2.n - 1);
  dv out;
  if (cl < 2) { out = A1; dv_append(&out, A2.v, A2.n); dv_free(&A2); return out; }
  int64_t c = (int64_t)cl;
  dv m = r_seq_len(0, 1, c);
  int64_t idx1 = A1.n - c;
  out = dv_copy(A1.v, idx1);
  for (int64_t k = 0; k < c; ++k) {
    double v = m.v[c - 1 - k] * A1.v[idx1 + k] + m.v[k] * A2.v[k];
    dv_append(&out, &v, 1);
  }
  dv_append(&out, A2.v + c, A2.n - c);
  dv_free(&m); dv_free(&A1); dv_free(&A2);
  return out;
}

/* fadeInOut(), R/utilities_soundgen.R:440-459 */
static void fade_in_out(double* a, int64_t n, int do_in, int do_out, double length_fade) {
  if ((!do_in && !do_out) || length_fade < 2) return;
  int64_t lf = (int64_t)length_fade; if (lf > n) lf = n;
  dv f = r_seq_len(0, 1, lf);
  if (do_in) for (int64_t i = 0; i < lf; ++i) a[i] *= f.v[i];
  if (do_out) for (int64_t i = 0; i < lf; ++i) a[n - lf + i] *= f.v[lf - 1 - i];
  dv_free(&f);
}

/* matchLengths(..., 'central'), R/utilities_math.R:413-444 */
static dv match_lengths_central(dv s, int64_t len) {
  if (s.n == len) return dv_copy(s.v, s.n);
  dv t;
  if (s.n < len) { t = dv_new(len); dv_append(&t, s.v, s.n); dv_append_zeros(&t, len); }
  else t = dv_copy(s.v, s.n);
  double halflen = (double)len / 2, center = (1 + (double)t.n) / 2;
  int64_t start = (int64_t)ceil(center - halflen);
  dv out = dv_copy(t.v + start - 1, len);
  dv_free(&t);
  return out;
}

/* addVectors(), R/utilities_math.R:500-526 (note: pads v2 with
 * insertionPoint zeros, not insertionPoint - 1) */
static dv add_vectors(dv v1, dv v2, double ip) {
  dv a, b;
  if (ip > 1) { a = dv_copy(v1.v, v1.n); b = dv_new((int64_t)ip); dv_append(&b, v2.v, v2.n); }
  else if (ip < 1) { a = dv_new((int64_t)(1 - ip)); dv_append(&a, v1.v, v1.n); b = dv_copy(v2.v, v2.n); }
  else { a = dv_copy(v1.v, v1.n); b = dv_copy(v2.v, v2.n); }
  for (int64_t i = 0; i < a.n; ++i) if (isnan(a.v[i])) a.v[i] = 0;
  for (int64_t i = 0; i < b.n; ++i) if (isnan(b.v[i])) b.v[i] = 0;
  if (b.n > a.n) dv_append_zeros(&a, b.n - a.n); else if (a.n > b.n) dv_append_zeros(&b, a.n - b.n);
  for (int64_t i = 0; i < a.n; ++i) a.v[i] += b.v[i];
  dv_free(&b);
  return a;
}

/* getSigmoid(), R/utilities_math.R:639-653 */
static dv get_sigmoid(int64_t len, double sr, double freq, double shape, double spikiness) {
  double from = -exp(-shape * spikiness), to = exp(shape * spikiness), slope = exp(fabs(shape)) * 5;
  int64_t lo = (int64_t)ceil(sr / freq / 2);
  dv a = r_seq_len(from, to, lo);
  for (int64_t i = 0; i < lo; ++i) a.v[i] = 1 / (1 + exp(-a.v[i] * slope));
  zero_one(a.v, lo);
  dv out = dv_new(len);
  for (int64_t i = 0; i < len; ++i) { int64_t k = i % (2 * lo); out.v[i] = k < lo ? a.v[k] : a.v[2 * lo - 1 - k]; }
  dv_free(&a);
  return out;
}

/* rnorm_bounded(), R/utilities_math.R:187-231 (n <= 64) */
static int rnorm_bounded(rng_t* r, int64_t n, const double* mean_in, int64_t nmean,
                         const double* sd_in, int64_t nsd, const double* low, const double* high,
                         int roundToInteger, double* out) {
  double mean[64], sd[64];
  if (n > 64) return fail(SG_E_UNSUPPORTED, "rnorm_bounded: n > 64");
  for (int64_t i = 0; i < n; ++i) { mean[i] = mean_in[nmean >= n ? i : 0]; sd[i] = sd_in[nsd >= n ? i : 0]; }
  if (low || high) for (int64_t i = 0; i < n; ++i) {   /* warning + clamp of out-of-range means */
    if (low && mean[i] < low[i]) mean[i] = low[i];
    if (high && mean[i] > high[i]) mean[i] = high[i];
  }
  int anysd = 0; for (int64_t i = 0; i < n; ++i) if (sd[i] != 0) anysd = 1;
  if (!anysd) { for (int64_t i = 0; i < n; ++i) out[i] = roundToInteger ? r_round(mean[i]) : mean[i]; return 0; }
  int rc;
  for (int64_t i = 0; i < n; ++i) { if ((rc = r_rnorm1(r, mean[i], sd[i], &out[i]))) return rc; }
  if (roundToInteger) for (int64_t i = 0; i < n; ++i) out[i] = r_round(out[i]);
  if (!low && !high) return 0;
  for (int64_t i = 0; i < n; ++i) {
    double lo = low ? low[i] : -INFINITY, hi = high ? high[i] : INFINITY;
    int guard = 0;
    while (out[i] < lo || out[i] > hi) {
      if ((rc = r_rnorm1(r, mean[i], sd[i], &out[i]))) return rc;
      if (roundToInteger) for (int64_t k = 0; k < n; ++k) out[k] = r_round(out[k]);
      if (++guard > 100000) return fail(SG_E_RANDOM, "rnorm_bounded: rejection loop too long");
    }
  }
  return 0;
}

/* ------------------------------------------------------ generateHarmonics */
static int gen_harm(const double* pitch_in, int64_t len, const sg_harm_params* P,
                    sg_anchors amplAnchors, rng_t* Rp, double** out, int64_t* out_len) {
  int rc = 0;
#define R (*Rp)
  dv pitch = dv_copy(pitch_in, len), gc = {0}, ppg = {0}, rw = {0}, rwbin = {0}, drift = {0};
  dv rolloffAmpl = {0}, roll = {0}, integr = {0}, wave = {0}, up_pitch = {0}, gc_up = {0};
  dv vf_on = {0}, jit_on = {0};
  ampmat* mats = NULL; int64_t *es = NULL, *ee = NULL, nEp = 0;
  double sr = P->samplingRate;
  *out = NULL; *out_len = 0;
  if (len < 2) { rc = fail(SG_E_DOMAIN, "generateHarmonics: pitch contour too short"); goto done; }
  if (P->vibratoDep > 0)
    for (int64_t i = 0; i < len; ++i)
      pitch.v[i] *= pow(2.0, sin(2 * M_PI * (double)(i + 1) * P->vibratoFreq / P->pitchSamplingRate) * P->vibratoDep / 12);
  gc = get_glottal_cycles(pitch.v, len, P->pitchSamplingRate);
  int64_t nGC = gc.n;
  ppg = dv_new(nGC); for (int64_t g = 0; g < nGC; ++g) ppg.v[g] = pitch.v[(int64_t)gc.v[g] - 1];
  /* amplitude contour per gc */
  int useAmpl = 0;
  if (amplAnchors.n > 0) for (int i = 0; i < amplAnchors.n; ++i) if (amplAnchors.value[i] < -P->throwaway) useAmpl = 1;
  rolloffAmpl = dv_new(nGC);
  if (useAmpl) {
    dv ac; TRY(get_smooth_contour(amplAnchors, nGC, 0, 0, 1, 0, 1, -P->throwaway, sr, &ac));
    for (int64_t g = 0; g < nGC; ++g) rolloffAmpl.v[g] = (ac.v[g] / fabs(P->throwaway) - 1) * P->rolloff_perAmpl;
    dv_free(&ac);
  }
  vf_on = dv_new(nGC); jit_on = dv_new(nGC);
  if (P->temperature > 0) {
    double tr[2] = { P->randomWalk_trendStrength, -P->randomWalk_trendStrength };
    TRY(get_random_walk(&R, nGC, P->temperature, 0.3, 1, tr, 2, 0, &rw));
    dv r0100 = dv_copy(rw.v, nGC); zero_one(r0100.v, nGC); for (int64_t g = 0; g < nGC; ++g) r0100.v[g] *= 100;
    dv ml = dv_new(nGC); for (int64_t g = 0; g < nGC; ++g) ml.v[g] = ceil(P->shortestEpoch / 1000 * ppg.v[g]);
    rwbin = dv_new(nGC);
    get_integer_random_walk(r0100.v, nGC, P->nonlinBalance, ml.v, rwbin.v);
    dv_free(&r0100); dv_free(&ml);
    double m = r_mean(rw.v, nGC);
    for (int64_t g = 0; g < nGC; ++g) { rw.v[g] = rw.v[g] - m + 1; vf_on.v[g] = rwbin.v[g] > 0; jit_on.v[g] = rwbin.v[g] == 2; }
  } else {
    rw = dv_new(nGC); for (int64_t g = 0; g < nGC; ++g) { rw.v[g] = 1; vf_on.v[g] = 1; jit_on.v[g] = 1; }
  }
  /* jitter */
  if (P->jitterDep > 0 && P->nonlinBalance > 0) {
    dv idx = dv_new(0); double one = 1; dv_append(&idx, &one, 1);
    double i = 1;
    while (i < nGC) {
      double ratio = ppg.v[(int64_t)i - 1] * P->jitterLen / 1000;
      i = idx.v[idx.n - 1] + ratio; dv_append(&idx, &i, 1);
    }
    dv idx2 = dv_new(0);
    for (int64_t k = 0; k < idx.n; ++k) {
      double v = r_round(idx.v[k]);
      if (v > nGC) continue;
      int dup = 0; for (int64_t q = 0; q < idx2.n; ++q) if (idx2.v[q] == v) { dup = 1; break; }
      if (!dup) dv_append(&idx2, &v, 1);
    }
    dv_free(&idx);
    dv jit = dv_new(idx2.n);
    for (int64_t k = 0; k < idx2.n; ++k) {
      double z; TRY(r_rnorm1(&R, 0, P->jitterDep / 12, &z));
      int64_t q = (int64_t)idx2.v[k] - 1;
      jit.v[k] = pow(2.0, z * rw.v[q] * jit_on.v[q]);
    }
    dv jpg;
    if (idx2.n == 1) { jpg = dv_new(nGC); for (int64_t g = 0; g < nGC; ++g) jpg.v[g] = jit.v[0]; }
    else jpg = r_spline(idx2.v, jit.v, idx2.n, nGC);
    for (int64_t g = 0; g < nGC; ++g) ppg.v[g] *= jpg.v[g];
    dv_free(&jpg); dv_free(&jit); dv_free(&idx2);
  }
  /* slow drift */
  if (P->temperature > 0) {
    double rws = .9 - P->temperature * P->pitchDriftFreq - 1.2 / (1 + exp(-.008 * ((double)nGC - 10))) + .6;
    double rwr = P->temperature * P->pitchDriftDep + (double)nGC / 1000 / 12;
    double zero = 0;
    TRY(get_random_walk(&R, nGC, rwr, rws, 1, &zero, 1, 0, &drift));
    double m = r_mean(drift.v, drift.n);
    for (int64_t g = 0; g < nGC; ++g) { drift.v[g] = pow(2.0, drift.v[g] - m); ppg.v[g] *= drift.v[g]; }
  }
  for (int64_t g = 0; g < nGC; ++g) { if (ppg.v[g] > P->pitchCeiling) ppg.v[g] = P->pitchCeiling; if (ppg.v[g] < P->pitchFloor) ppg.v[g] = P->pitchFloor; }
  double pmin = r_min(ppg.v, nGC);
  int64_t nH = (int64_t)ceil((sr / 2 - pmin) / pmin);
  {
    dv ro = dv_new(nGC), roo = dv_new(nGC), rk = dv_new(nGC);
    for (int64_t g = 0; g < nGC; ++g) {
      double w = rw.v[g];
      ro.v[g] = (P->rolloff + rolloffAmpl.v[g]) * w * w * w;
      roo.v[g] = P->rolloffOct * w * w * w;
      rk.v[g] = P->rolloffKHz * w;
    }
    int64_t H;
    rc = get_rolloff(ppg.v, nGC, nH, ro.v, roo.v, P->rolloffParab, P->rolloffParabHarm, NAN, rk.v, 200, P->throwaway, sr, &roll, &H);
    dv_free(&ro); dv_free(&roo); dv_free(&rk);
    if (rc) goto done;
    /* shimmer */
    if (P->shimmerDep > 0 && P->nonlinBalance > 0) {
      for (int64_t g = 0; g < nGC; ++g) {
        double z; TRY(r_rnorm1(&R, 0, P->shimmerDep / 100, &z));
        double sh = pow(2.0, z * rw.v[g] * jit_on.v[g]);
        for (int64_t h = 0; h < H; ++h) roll.v[g * H + h] *= sh;
      }
    }
    if (P->subDep > 0 && P->nonlinBalance > 0) {
      dv sf = dv_new(nGC), sd = dv_new(nGC);
      for (int64_t g = 0; g < nGC; ++g) { double w4 = pow(rw.v[g], 4); sf.v[g] = P->subFreq * w4; sd.v[g] = P->subDep * w4 * vf_on.v[g]; }
      rc = get_vocal_fry(roll.v, H, ppg.v, nGC, sf.v, sd.v, P->throwaway, P->shortestEpoch, &mats, &es, &ee, &nEp);
      dv_free(&sf); dv_free(&sd);
      if (rc) goto done;
    } else {
      nEp = 1; mats = (ampmat*)calloc(1, sizeof(ampmat));
      mats[0].A = dv_copy(roll.v, H * nGC); mats[0].nrow = H; mats[0].ncol = nGC;
      mats[0].mult = dv_new(H); for (int64_t h = 0; h < H; ++h) mats[0].mult.v[h] = (double)(h + 1);
      es = (int64_t*)malloc(sizeof(int64_t)); ee = (int64_t*)malloc(sizeof(int64_t)); es[0] = 1; ee[0] = nGC;
    }
  }
  /* upsample(), R/utilities_soundgen.R:392-416 */
  {
    dv gcl = dv_new(nGC); for (int64_t g = 0; g < nGC; ++g) gcl.v[g] = r_round(sr / ppg.v[g]);
    dv c = dv_new(nGC); r_cumsum(gcl.v, c.v, nGC);
    gc_up = dv_new(nGC + 1); gc_up.v[0] = 1; for (int64_t g = 0; g < nGC; ++g) gc_up.v[g + 1] = c.v[g];
    int64_t N = (int64_t)c.v[nGC - 1];
    if (nGC == 1) { up_pitch = dv_new(N); for (int64_t i = 0; i < N; ++i) up_pitch.v[i] = ppg.v[0]; }
    else if (nGC == 2) up_pitch = r_seq_len(ppg.v[0], ppg.v[1], N);
    else {
      dv t = dv_new(nGC); t.v[0] = 1; t.v[nGC - 1] = (double)N;
      for (int64_t i = 2; i <= nGC - 1; ++i) t.v[i - 1] = c.v[i - 2] + r_round(gcl.v[i - 1] / 2);
      up_pitch = r_spline(t.v, ppg.v, nGC, N);
      dv_free(&t);
    }
    integr = dv_new(N); r_cumsum(up_pitch.v, integr.v, N);
    for (int64_t i = 0; i < N; ++i) integr.v[i] /= sr;
    dv_free(&gcl); dv_free(&c);
  }
  /* synthesis per epoch + crossFade */
  wave = dv_new(1); wave.v[0] = 0;
  for (int64_t e = 0; e < nEp; ++e) {
    int64_t u0 = (int64_t)gc_up.v[es[e] - 1], u1 = (int64_t)gc_up.v[ee[e]];  /* 1-based sample idx */
    int64_t Ne = u1 - u0 + 1;
    int64_t G = ee[e] - es[e] + 1;
    ampmat* m = &mats[e];
    dv we = dv_new(Ne);
    dv xk = dv_new(G); for (int64_t g = 0; g < G; ++g) xk.v[g] = gc_up.v[es[e] - 1 + g];
    for (int64_t h = 0; h < m->nrow; ++h) {
      double tf = m->mult.v[h];
      dv yrow = dv_new(G); for (int64_t g = 0; g < G; ++g) yrow.v[g] = m->A.v[g * m->nrow + h];
      dv am; rc = r_approx_n(xk.v, yrow.v, G, Ne, &am);
      dv_free(&yrow);
      if (rc) { dv_free(&we); dv_free(&xk); goto done; }
      for (int64_t j = 0; j < Ne; ++j) we.v[j] = we.v[j] + sin(2 * M_PI * integr.v[u0 - 1 + j] * tf) * am.v[j];
      dv_free(&am);
    }
    dv_free(&xk);
    dv nw = cross_fade(wave, we, sr, 15);
    dv_free(&wave); dv_free(&we); wave = nw;
  }
  /* post-synthesis */
  if (useAmpl) {
    dv env; TRY(get_smooth_contour(amplAnchors, wave.n, 0, 0, 1, 0, 0, 0, sr, &env));
    for (int64_t i = 0; i < wave.n; ++i) wave.v[i] *= pow(2.0, env.v[i] / 10);
    dv_free(&env);
  }
  {
    double mx = r_max(wave.v, wave.n);
    for (int64_t i = 0; i < wave.n; ++i) wave.v[i] /= mx;
  }
  if (P->attackLen > 0) fade_in_out(wave.v, wave.n, 1, 1, floor(P->attackLen * sr / 1000));
  if (P->temperature > 0) {
    dv xk = dv_copy(gc_up.v, nGC);
    dv du; TRY(r_approx_n(xk.v, drift.v, nGC, wave.n, &du));
    for (int64_t i = 0; i < wave.n; ++i) wave.v[i] *= du.v[i];
    dv_free(&du); dv_free(&xk);
  }
  *out = wave.v; *out_len = wave.n; wave.v = NULL;
done:
  dv_free(&pitch); dv_free(&gc); dv_free(&ppg); dv_free(&rw); dv_free(&rwbin); dv_free(&drift);
  dv_free(&rolloffAmpl); dv_free(&roll); dv_free(&integr); dv_free(&wave); dv_free(&up_pitch);
  dv_free(&gc_up); dv_free(&vf_on); dv_free(&jit_on);
  if (mats) { for (int64_t e = 0; e < nEp; ++e) ampmat_free(&mats[e]); free(mats); }
  free(es); free(ee);
#undef R
  return rc;
}
OR_API int or_generate_harmonics(const double* pitch_in, int64_t len, const sg_harm_params* P,
                                 sg_anchors amplAnchors, const sg_random* rnd, double** out, int64_t* out_len) {
  rng_t R = { rnd, 0, 0 };
  return gen_harm(pitch_in, len, P, amplAnchors, &R, out, out_len);
}

/* ------------------------------------------------------------------ FFT */
/* Mixed-radix recursive DFT (any n), fp64: X[k] = sum x[j] exp(sgn*2*pi*i*jk/n) */
static void fft_rec(const double* re, const double* im, int64_t n, int64_t stride, double* ore, double* oim, int sgn) {
  if (n == 1) { ore[0] = re[0]; oim[0] = im[0]; return; }
  int64_t p = 0;
  for (int64_t f = 2; f * f <= n; ++f) if (n % f == 0) { p = f; break; }
  if (!p) { /* prime: direct DFT */
    for (int64_t k = 0; k < n; ++k) {
      long double sr = 0, si = 0;
      for (int64_t j = 0; j < n; ++j) {
        double ang = sgn * 2 * M_PI * (double)((j * k) % n) / (double)n;
        double c = cos(ang), s = sin(ang);
        double xr = re[j * stride], xi = im[j * stride];
        sr += xr * c - xi * s; si += xr * s + xi * c;
      }
      ore[k] = (double)sr; oim[k] = (double)si;
    }
    return;
  }
  int64_t m = n / p;
  double* tre = (double*)malloc(n * sizeof(double)); double* tim = (double*)malloc(n * sizeof(double));
  for (int64_t q = 0; q < p; ++q) fft_rec(re + q * stride, im + q * stride, m, stride * p, tre + q * m, tim + q * m, sgn);
  for (int64_t k = 0; k < n; ++k) {
    long double sr = 0, si = 0;
    int64_t kk = k % m;
    for (int64_t q = 0; q < p; ++q) {
      double ang = sgn * 2 * M_PI * (double)((q * k) % n) / (double)n;
      double c = cos(ang), s = sin(ang);
      double xr = tre[q * m + kk], xi = tim[q * m + kk];
      sr += xr * c - xi * s; si += xr * s + xi * c;
    }
    ore[k] = (double)sr; oim[k] = (double)si;
  }
  free(tre); free(tim);
}
OR_API void or_fft(const double* re, const double* im, int64_t n, int inverse, double* ore, double* oim) {
  fft_rec(re, im, n, 1, ore, oim, inverse ? 1 : -1);
}

/* seewave::istft(stft, ovlp, wl, wn = "hanning"), seewave.r:3447-3486.
 * stft: nr x nc complex (col-major, re/im separate; im may be NULL). The
 * inverse has length(X) = 2 nr points (wl - 1 for an odd wl) and is divided
 * by that length; xprim * win then recycles xprim against the wl-point
 * window (:3477-3479): sample i of the frame is xprim[i mod 2 nr] * win[i]. */
static dv istft(const double* zre, const double* zim, int64_t nr, int64_t nc, double ovlp, int64_t wl) {
  double h = (double)wl * (100 - ovlp) / 100;
  double xlen = (double)wl + (double)(nc - 1) * h;
  dv x = dv_new((int64_t)xlen);
  dv win = dv_new(wl);
  for (int64_t i = 0; i < wl; ++i) win.v[i] = 0.5 - 0.5 * cos(2 * M_PI * (double)i / (double)(wl - 1));
  double* Xr = (double*)malloc(wl * sizeof(double)); double* Xi = (double*)malloc(wl * sizeof(double));
  double* yr = (double*)malloc(wl * sizeof(double)); double* yi = (double*)malloc(wl * sizeof(double));
  dv bs = r_seq_by(0, h * (double)(nc - 1), h);
  for (int64_t f = 0; f < bs.n; ++f) {
    double b = bs.v[f];
    int64_t col = (int64_t)(1 + b / h) - 1;
    const double* cr = zre + col * nr; const double* ci = zim ? zim + col * nr : NULL;
    for (int64_t k = 0; k < nr; ++k) { Xr[k] = cr[k]; Xi[k] = ci ? ci[k] : 0; }
    const int64_t n2 = 2 * nr;  /* length(X) */
    Xr[nr] = cr[nr - 1]; Xi[nr] = 0;
    for (int64_t k = 1; k < nr; ++k) { Xr[n2 - k] = cr[k]; Xi[n2 - k] = ci ? -ci[k] : 0; }
    fft_rec(Xr, Xi, n2, 1, yr, yi, 1);
    for (int64_t i = 0; i < wl; ++i) {  /* (b+1):(b+wl) truncated */
      int64_t q = (int64_t)(b + 1 + (double)i) - 1;
      if (q < x.n) x.v[q] = x.v[q] + (yr[i % n2] / (double)n2) * win.v[i];
    }
  }
  long double W0 = 0; for (int64_t i = 0; i < wl; ++i) W0 += win.v[i] * win.v[i];
  for (int64_t i = 0; i < x.n; ++i) x.v[i] = x.v[i] * h / (double)W0;
  free(Xr); free(Xi); free(yr); free(yi); dv_free(&win); dv_free(&bs);
  return x;
}
OR_API int or_istft(const double* zre, const double* zim, int64_t nr, int64_t nc, double ovlp, int64_t wl, double** out, int64_t* out_len) {
  dv x = istft(zre, zim, nr, nc, ovlp, wl); *out = x.v; *out_len = x.n; return 0;
}
/* seewave::stft(wave, wl, zp = 0, step, wn = "hamming", complex = TRUE) */
static void stft(const double* wave, int64_t L, int64_t wl, const double* step, int64_t nc, double* zre, double* zim) {
  (void)L;
  int64_t nr = wl / 2;
  double* W = (double*)malloc(wl * sizeof(double));
  for (int64_t i = 0; i < wl; ++i) W[i] = 0.54 - 0.46 * cos(2 * M_PI * (double)i / (double)(wl - 1));
  double *xr = (double*)malloc(wl * sizeof(double)), *xi = (double*)calloc(wl, sizeof(double));
  double *yr = (double*)malloc(wl * sizeof(double)), *yi = (double*)malloc(wl * sizeof(double));
  for (int64_t f = 0; f < nc; ++f) {
    double x0 = step[f];
    for (int64_t i = 0; i < wl; ++i) { int64_t q = (int64_t)(x0 + (double)i) - 1; xr[i] = wave[q] * W[i]; xi[i] = 0; }
    fft_rec(xr, xi, wl, 1, yr, yi, -1);
    for (int64_t k = 0; k < nr; ++k) { zre[f * nr + k] = yr[k] / (double)wl; zim[f * nr + k] = yi[k] / (double)wl; }
  }
  free(W); free(xr); free(xi); free(yr); free(yi);
}
OR_API int or_stft(const double* wave, int64_t L, int64_t wl, const double* step, int64_t nc, double* zre, double* zim) {
  stft(wave, L, wl, step, nc, zre, zim); return 0;
}

/* ------------------------------------------------------ generateNoise */
static int generate_noise(rng_t* R, int64_t len, sg_anchors noiseAnchors, double rolloffNoise, double attackLen,
                          int64_t wl, double sr, double overlap, double throwaway,
                          const double* filterNoise, int64_t fnc, dv* out) {
  (void)throwaway;
  int rc = 0;
  dv bs = {0}, step = {0}, filt = {0}, zf = {0}, br = {0}, br2 = {0};
  TRY(get_smooth_contour(noiseAnchors, len, 0, 0, 1, -120, 1, 40, sr, &bs));
  if (bs.n == 0) { *out = dv_new(len); goto done; }  /* NA contour → zeros */
  for (int64_t i = 0; i < bs.n; ++i) bs.v[i] = pow(2.0, bs.v[i] / 10);
  {
    step = r_seq_by(1, (double)(len + wl), (double)wl - (overlap * (double)wl / 100));
    int64_t nr = wl / 2, nc = step.n;
    int64_t ncolF = filterNoise ? fnc : 1;
    filt = dv_new(nr * ncolF);
    for (int64_t c = 0; c < ncolF; ++c)
      for (int64_t k = 0; k < nr; ++k)
        filt.v[c * nr + k] = (filterNoise ? filterNoise[c * nr + k] : 1.0) * pow(2.0, rolloffNoise / 10 * log2((double)(k + 1)));
    dv fri = dv_new(nc);
    if (!filterNoise) for (int64_t c = 0; c < nc; ++c) fri.v[c] = 1;
    else { dv s = r_seq_len(1, (double)ncolF, nc); for (int64_t c = 0; c < nc; ++c) fri.v[c] = r_round(s.v[c]); dv_free(&s); }
    /* runif(nr * nc) with nr = wl / 2 (x.5 for an odd wl: floor(nr * nc) draws),
     * matrix(nrow = nr) keeps as.integer(nr) rows of them */
    zf = dv_new(nr * nc);
    const int64_t ndraw = (int64_t)((double)wl / 2 * (double)nc);
    for (int64_t q = 0; q < ndraw; ++q) {
      double u; rc = rng_unif(R, &u); if (rc) { dv_free(&fri); goto done; }
      if (q < nr * nc) { const int64_t c = q / nr, k = q % nr; zf.v[q] = u * filt.v[((int64_t)fri.v[c] - 1) * nr + k]; }
    }
    dv_free(&fri);
    br = istft(zf.v, NULL, nr, nc, overlap, wl);
    br2 = match_lengths_central(br, len);
    double mx = r_max(br2.v, br2.n);
    for (int64_t i = 0; i < len; ++i) br2.v[i] = br2.v[i] / mx * bs.v[i];
    fade_in_out(br2.v, len, 1, 1, floor(attackLen * sr / 1000));
    *out = br2; br2.v = NULL;
  }
done:
  dv_free(&bs); dv_free(&step); dv_free(&filt); dv_free(&zf); dv_free(&br); dv_free(&br2);
  return rc;
}
OR_API int or_generate_noise(int64_t len, sg_anchors noiseAnchors, double rolloffNoise, double attackLen,
                             int32_t wl, double sr, double overlap, double throwaway,
                             const double* filterNoise, int32_t fnc, const sg_random* rnd, double** out) {
  rng_t R = { rnd, 0, 0 }; dv o = {0};
  int rc = generate_noise(&R, len, noiseAnchors, rolloffNoise, attackLen, wl, sr, overlap, throwaway, filterNoise, fnc, &o);
  *out = o.v; return rc;
}

/* ------------------------------------------------ getSpectralEnvelope */
typedef struct { int64_t nc; double *time, *freq, *amp, *width; } fup_t; /* columns, length nc */
static void fup_free(fup_t* f) { free(f->time); free(f->freq); free(f->amp); free(f->width); }
static double* col_upsample(const double* t, const double* y, int64_t np, int64_t nPoints, double slf, int64_t nc, int* rc) {
  double* o = (double*)malloc(nc * sizeof(double));
  if (np > 1) {
    dv a; *rc = r_approx_n(t, y, np, (int64_t)(nPoints + pow(2.0, slf)), &a);
    if (*rc) { free(o); return NULL; }
    dv xs = dv_new(a.n); for (int64_t i = 0; i < a.n; ++i) xs.v[i] = (double)(i + 1);
    dv s = r_spline(xs.v, a.v, a.n, nc);
    memcpy(o, s.v, nc * sizeof(double));
    dv_free(&a); dv_free(&xs); dv_free(&s);
  } else for (int64_t i = 0; i < nc; ++i) o[i] = y[0];
  return o;
}
/* nrd = windowLength_points / 2 as R passes it: an odd window gives x.5, whose
 * matrices have as.integer(nrd) rows while bin_width keeps nrd (:419) */
static int spectral_envelope(rng_t* R, double nrd, int64_t nc, const sg_formants* F, double formantDep,
                             double rolloffLip, sg_anchors mouthAnchors, double mouthOpenThres, double openMouthBoost,
                             double vocalTract, double temperature, double formDrift, double formDisp,
                             double formantDepStoch, double slf, double sr, double speedSound, double* env) {
  int rc = 0;
  const int64_t nr = (int64_t)nrd;
  int nF = F ? F->n_formants : 0;
  int haveVT = !isnan(vocalTract) || (vocalTract != vocalTract && 0); /* NaN encodes NULL */
  double VT = vocalTract;
  int vtIsNull = isnan(vocalTract) && !(F && nF > 0 && 0);
  /* The R code distinguishes NULL (absent) from a computed NaN; we track it. */
  int vtComputedNaN = 0;
  fup_t* fu = NULL; int nfu = 0, cap = 0;
  dv mouth = {0}, mbin = {0};
  const int32_t* np = F ? F->n_points : NULL;
  (void)haveVT;
  if (vtIsNull && nF > 0) {  /* guess vocalTract from formant dispersion (length(formants[[1]]) > 2) */
    dv allf = dv_new(0); int64_t off = 0;
    for (int f = 0; f < nF; ++f) { dv_append(&allf, F->freq + off, np[f]); off += np[f]; }
    double fd;
    if (allf.n < 2) fd = NAN;
    else { dv d = dv_new(allf.n - 1); for (int64_t i = 0; i + 1 < allf.n; ++i) d.v[i] = allf.v[i + 1] - allf.v[i]; fd = r_mean(d.v, d.n); dv_free(&d); }
    VT = speedSound / 2 / fd; vtIsNull = 0; vtComputedNaN = isnan(VT);
    dv_free(&allf);
  }
  (void)vtComputedNaN;
  dv schwa_t = {0};
  double sch_time = 0, sch_freq = 0, sch_amp = 30, sch_width = 0; int32_t sch_np = 1;
  sg_formants SF;
  if (nF == 0 && !vtIsNull) {  /* schwa from vocalTract */
    sch_freq = speedSound / 4 / VT; sch_width = 50 * (1 + sch_freq * sch_freq / 6 / 1e6);
    SF.n_formants = 1; SF.f1_index = 0; SF.n_points = &sch_np; SF.time = &sch_time; SF.freq = &sch_freq; SF.amp = &sch_amp; SF.width = &sch_width;
    F = &SF; nF = 1; np = F->n_points;
  }
  (void)schwa_t;
  for (int64_t i = 0; i < nr * nc; ++i) env[i] = 0;
  if (nF > 0) {
    int64_t nPoints = 0; for (int f = 0; f < nF; ++f) if (np[f] > nPoints) nPoints = np[f];
    cap = nF + 64; fu = (fup_t*)calloc(cap, sizeof(fup_t)); nfu = nF;
    int64_t off = 0;
    for (int f = 0; f < nF; ++f) {
      fu[f].nc = nc;
      fu[f].time = col_upsample(F->time + off, F->time + off, np[f], nPoints, slf, nc, &rc); if (rc) goto done;
      fu[f].freq = col_upsample(F->time + off, F->freq + off, np[f], nPoints, slf, nc, &rc); if (rc) goto done;
      fu[f].amp = col_upsample(F->time + off, F->amp + off, np[f], nPoints, slf, nc, &rc); if (rc) goto done;
      fu[f].width = col_upsample(F->time + off, F->width + off, np[f], nPoints, slf, nc, &rc); if (rc) goto done;
      off += np[f];
    }
    if (temperature > 0) {
      double fdisp;
      if (vtIsNull && nF > 1) {
        dv ff = dv_new(nF); int64_t o2 = 0; for (int f = 0; f < nF; ++f) { ff.v[f] = F->freq[o2]; o2 += np[f]; }
        dv c2 = dv_new(nF); c2.v[0] = ff.v[0]; for (int f = 1; f < nF; ++f) c2.v[f] = ff.v[f] - ff.v[f - 1];
        fdisp = r_mean(c2.v, nF); dv_free(&ff); dv_free(&c2);
      } else if (!vtIsNull) fdisp = 2 * speedSound / (4 * VT);
      else fdisp = NAN;
      double sdG = fdisp * temperature * formDisp;
      double fmax = r_max(fu[nfu - 1].freq, nc);
      if (!isnan(sdG) && formantDepStoch > 0) {
        while (fmax < (sr / 2 - 1000)) {
          dv rw; double zero = 0;
          TRY(get_random_walk(R, nc, temperature * formDrift, 0, 1, &zero, 1, 0, &rw));
          if (rw.n > 1) { double m = r_mean(rw.v, rw.n); for (int64_t i = 0; i < rw.n; ++i) rw.v[i] = rw.v[i] - m + 1; }
          double g1, g2;
          TRY(r_rgamma1(R, fdisp * fdisp / (sdG * sdG), fdisp / (sdG * sdG), &g1));
          if (nfu >= cap) { cap *= 2; fu = (fup_t*)realloc(fu, cap * sizeof(fup_t)); }
          fup_t* t = &fu[nfu];
          t->nc = nc; t->time = (double*)malloc(nc * sizeof(double)); t->freq = (double*)malloc(nc * sizeof(double));
          t->amp = (double*)malloc(nc * sizeof(double)); t->width = (double*)malloc(nc * sizeof(double));
          for (int64_t c = 0; c < nc; ++c) {
            t->time[c] = fu[0].time[c];
            t->freq[c] = fu[nfu - 1].freq[c] + r_round(g1 * rw.v[rw.n > 1 ? c : 0]);
          }
          TRY(r_rgamma1(R, (formantDep / temperature) * (formantDep / temperature),
                        formantDepStoch * formantDep / ((formantDepStoch * temperature) * (formantDepStoch * temperature)), &g2));
          for (int64_t c = 0; c < nc; ++c) {
            t->amp[c] = r_round(g2 * rw.v[rw.n > 1 ? c : 0]);
            t->width[c] = 50 + (log2(t->freq[c]) - 5) * 20;
          }
          nfu++;
          dv_free(&rw);
          fmax = r_max(fu[nfu - 1].freq, nc);
        }
      }
      for (int f = 0; f < nfu; ++f)
        for (int cc = 2; cc <= 4; ++cc) {
          dv rw;
          TRY(get_random_walk(R, nc, temperature * formDrift, 0.3, 1, NULL, 1, 1, &rw));
          if (rw.n > 1) { double m = r_mean(rw.v, rw.n); for (int64_t i = 0; i < rw.n; ++i) rw.v[i] = rw.v[i] - m + 1; }
          double* col = cc == 2 ? fu[f].freq : cc == 3 ? fu[f].amp : fu[f].width;
          for (int64_t c = 0; c < nc; ++c) col[c] *= rw.v[rw.n > 1 ? c : 0];
          dv_free(&rw);
        }
    }
    double bw = sr / 2 / nrd;
    for (int f = 0; f < nfu; ++f)
      for (int64_t c = 0; c < nc; ++c) { fu[f].freq[c] = (fu[f].freq[c] - bw / 2) / bw + 1; fu[f].width[c] = fu[f].width[c] / bw; }
    mouth = dv_new(nc); mbin = dv_new(nc);
    int mouthNA = mouthAnchors.n < 1;
    for (int i = 0; i < mouthAnchors.n; ++i) if (isnan(mouthAnchors.value[i]) || isnan(mouthAnchors.time[i])) mouthNA = 1;
    if (mouthNA) { for (int64_t c = 0; c < nc; ++c) { mouth.v[c] = 0.5; mbin.v[c] = 1; } }
    else {
      dv mo; TRY(get_smooth_contour(mouthAnchors, nc, 0, 0, 1, 0, 1, 1, 16000, &mo));
      for (int64_t c = 0; c < nc; ++c) { double v = mo.v[c]; if (v < mouthOpenThres) v = 0; mouth.v[c] = v; mbin.v[c] = v > 0 ? 1 : 0; }
      dv_free(&mo);
    }
    int adj = !vtIsNull && isfinite(VT);
    for (int f = 0; f < nfu; ++f)
      for (int64_t c = 0; c < nc; ++c) {
        double ab = 0;
        if (adj) { double ah = (mouth.v[c] - 0.5) * speedSound / (4 * VT); ab = (ah - bw / 2) / bw + 1; }
        fu[f].freq[c] += ab;
        if (fu[f].freq[c] < 1) fu[f].freq[c] = 1;
      }
    /* nasalization */
    int anyClosed = 0; for (int64_t c = 0; c < nc; ++c) if (mbin.v[c] == 0) anyClosed = 1;
    if (anyClosed && F->f1_index >= 0) {
      int i1 = F->f1_index;
      if (nfu + 2 > cap) { cap = nfu + 2; fu = (fup_t*)realloc(fu, cap * sizeof(fup_t)); }
      fup_t* p = &fu[nfu]; fup_t* z = &fu[nfu + 1]; fup_t* f1 = &fu[i1];
      p->nc = z->nc = nc;
      p->time = (double*)malloc(nc * sizeof(double)); p->freq = (double*)malloc(nc * sizeof(double)); p->amp = (double*)malloc(nc * sizeof(double)); p->width = (double*)malloc(nc * sizeof(double));
      z->time = (double*)malloc(nc * sizeof(double)); z->freq = (double*)malloc(nc * sizeof(double)); z->amp = (double*)malloc(nc * sizeof(double)); z->width = (double*)malloc(nc * sizeof(double));
      for (int64_t c = 0; c < nc; ++c) {
        p->time[c] = f1->time[c]; p->freq[c] = f1->freq[c]; p->amp[c] = 0; p->width[c] = f1->width[c];
        if (mbin.v[c] == 0) {
          p->amp[c] = f1->amp[c] * 2 / 3; p->width[c] = f1->width[c] * 2 / 3;
          p->freq[c] = (f1->freq[c] > 550 / bw) ? f1->freq[c] - 250 / bw : f1->freq[c] + 250 / bw;
        }
      }
      for (int64_t c = 0; c < nc; ++c) {
        z->time[c] = f1->time[c]; z->freq[c] = f1->freq[c]; z->amp[c] = 0; z->width[c] = f1->width[c];
        if (mbin.v[c] == 0) {
          z->amp[c] = -f1->amp[c] * 2 / 3;
          z->freq[c] = (p->freq[c] + f1->freq[c]) / 2;
          z->width[c] = p->width[c];
        }
      }
      for (int64_t c = 0; c < nc; ++c) if (mbin.v[c] == 0) { f1->amp[c] = f1->amp[c] * 4 / 5; f1->width[c] = f1->width[c] * 5 / 4; }
      nfu += 2;
    }
    /* dgamma formants, normalised per column (log domain) */
    double* col = (double*)malloc(nr * sizeof(double));
    for (int f = 0; f < nfu; ++f)
      for (int64_t c = 0; c < nc; ++c) {
        double mg = fu[f].freq[c], sdg = fu[f].width[c];
        if (sdg == 0) sdg = 1;
        double shape = mg * mg / (sdg * sdg), rate = mg / (sdg * sdg);
        double lmax = -INFINITY;
        for (int64_t k = 0; k < nr; ++k) {
          double x = (double)(k + 1);
          double l = (shape - 1) * log(x) - rate * x;
          if (shape == 1) l = -rate * x;
          col[k] = l; if (l > lmax) lmax = l;
        }
        for (int64_t k = 0; k < nr; ++k) env[c * nr + k] += exp(col[k] - lmax) * fu[f].amp[c];
      }
    free(col);
    for (int64_t i = 0; i < nr * nc; ++i) env[i] *= formantDep;
  } else {
    mouth = dv_new(nc); mbin = dv_new(nc);
    for (int64_t c = 0; c < nc; ++c) { mouth.v[c] = 0.5; mbin.v[c] = 1; }
  }
  for (int64_t c = 0; c < nc; ++c)
    for (int64_t k = 0; k < nr; ++k) {
      double lip = rolloffLip * log2((double)(k + 1));
      env[c * nr + k] = (env[c * nr + k] + lip * mbin.v[c]) * pow(2.0, mouth.v[c] * openMouthBoost / 10);
    }
  for (int64_t i = 0; i < nr * nc; ++i) env[i] = pow(2.0, env[i] / 10);
done:
  if (fu) { for (int f = 0; f < nfu; ++f) fup_free(&fu[f]); free(fu); }
  dv_free(&mouth); dv_free(&mbin);
  return rc;
}
OR_API int or_spectral_envelope(int32_t nr, int32_t nc, const sg_formants* F, double formantDep, double rolloffLip,
                                sg_anchors mouthAnchors, double mouthOpenThres, double openMouthBoost, double vocalTract,
                                double temperature, double formDrift, double formDisp, double formantDepStoch,
                                double slf, double sr, double speedSound, const sg_random* rnd, double* out) {
  rng_t R = { rnd, 0, 0 };
  return spectral_envelope(&R, nr, nc, F, formantDep, rolloffLip, mouthAnchors, mouthOpenThres, openMouthBoost,
                           vocalTract, temperature, formDrift, formDisp, formantDepStoch, slf, sr, speedSound, out);
}

/* Formant filter block of soundgen(), R/soundgen.R:743-807 (wl already set) */
/* diagnostics (tests only): with capture on, the last formant filter's inputs are kept */
static int g_cap_on = 0;
static dv g_cap_sound = {0, 0}, g_cap_env = {0, 0};
static int64_t g_cap_nc = 0, g_cap_wl = 0;
static int formant_filter(const double* sound, int64_t L, const double* env, int64_t env_nc, int64_t wl,
                          double overlap, dv* out) {
  if (g_cap_on) {
    dv_free(&g_cap_sound); dv_free(&g_cap_env);
    g_cap_sound = dv_copy(sound, L); g_cap_env = dv_copy(env, env_nc * (wl / 2));
    g_cap_nc = env_nc; g_cap_wl = wl;
  }
  dv step = r_seq_by(1, (double)(L - wl > 1 ? L - wl : 1), (double)wl - (overlap * (double)wl / 100));
  int64_t nc = step.n, nr = wl / 2;
  double* zre = (double*)malloc(nr * nc * sizeof(double)); double* zim = (double*)malloc(nr * nc * sizeof(double));
  stft(sound, L, wl, step.v, nc, zre, zim);
  for (int64_t c = 0; c < nc; ++c)
    for (int64_t k = 0; k < nr; ++k) {
      double e = env[(env_nc == 1 ? 0 : c) * nr + k];
      zre[c * nr + k] *= e; zim[c * nr + k] *= e;
    }
  dv y = istft(zre, zim, nr, nc, overlap, wl);
  double mx = r_max(y.v, y.n);
  for (int64_t i = 0; i < y.n; ++i) y.v[i] /= mx;
  free(zre); free(zim); dv_free(&step);
  *out = y;
  return 0;
}
OR_API void or_debug_capture(int on) { g_cap_on = on; }
OR_API int64_t or_debug_captured(double* sound, double* env, int64_t* env_nc, int64_t* wl) {
  if (sound) memcpy(sound, g_cap_sound.v, g_cap_sound.n * sizeof(double));
  if (env) memcpy(env, g_cap_env.v, g_cap_env.n * sizeof(double));
  if (env_nc) *env_nc = g_cap_nc;
  if (wl) *wl = g_cap_wl;
  return g_cap_sound.n;
}
OR_API int or_formant_filter(const double* sound, int64_t L, const double* env, int32_t env_nc, int32_t wl,
                             double overlap, double** out, int64_t* out_len) {
  dv y; int rc = formant_filter(sound, L, env, env_nc, wl, overlap, &y);
  *out = y.v; *out_len = y.n; return rc;
}

OR_API int or_get_rolloff(const double* pitch, int32_t nGC, int32_t nH, double rolloff, double rolloffOct,
                          double rolloffParab, double rolloffParabHarm, double rolloffParabCeiling, double rolloffKHz,
                          double baseline, double throwaway, double sr, double* out, int32_t* out_rows) {
  dv ro = dv_new(nGC), roo = dv_new(nGC), rk = dv_new(nGC), r; int64_t H;
  for (int g = 0; g < nGC; ++g) { ro.v[g] = rolloff; roo.v[g] = rolloffOct; rk.v[g] = rolloffKHz; }
  int rc = get_rolloff(pitch, nGC, nH, ro.v, roo.v, rolloffParab, rolloffParabHarm, rolloffParabCeiling, rk.v, baseline,
                       throwaway, sr, &r, &H);
  if (!rc) { memcpy(out, r.v, H * nGC * sizeof(double)); *out_rows = (int32_t)H; dv_free(&r); }
  dv_free(&ro); dv_free(&roo); dv_free(&rk);
  return rc;
}

/* helpers exported for unit tests */
/* getSmoothContour() with len given (R/smoothContours.R:53-227); out has len values */
OR_API int or_smooth_contour(const double* time, const double* value, int64_t n, int64_t len, int thisIsPitch,
                             int method, int has_floor, double vfloor, int has_ceil, double vceil, double sr,
                             double* out) {
  sg_anchors an;
  an.n = (int32_t)n;
  an.time = time;
  an.value = value;
  dv c;
  const int rc = get_smooth_contour(an, len, thisIsPitch, method, has_floor, vfloor, has_ceil, vceil, sr, &c);
  if (rc) return rc;
  if (len < 0) len = c.n;  /* len = NULL: the caller sized out from the anchors' span */
  for (int64_t i = 0; i < len; ++i) out[i] = i < c.n ? c.v[i] : NAN;
  dv_free(&c);
  return 0;
}
/* loess(y ~ x, span) + predict at z[m] (R stats defaults, 1-D) */
OR_API int or_loess(const double* x, const double* y, int n, double span, const double* z, int64_t m, double* out) {
  lo_tree T;
  const int rc = lo_build(x, y, n, span, &T);
  if (rc == LO_ZERO_WIDTH) return fail(SG_E_DOMAIN, "loess: NaN vertex value (predict() stops: NA/NaN/Inf in foreign function call)");
  if (rc) return rc;
  for (int64_t i = 0; i < m; ++i) out[i] = (z[i] < x[0] || z[i] > x[n - 1]) ? NAN : lo_eval(&T, z[i]);
  return 0;
}
OR_API int64_t or_glottal_cycles(const double* pitch, int64_t len, double psr, double* out) {
  dv g = get_glottal_cycles(pitch, len, psr); memcpy(out, g.v, g.n * sizeof(double)); int64_t n = g.n; dv_free(&g); return n;
}
OR_API void or_spline(const double* x, const double* y, int64_t nx, int64_t n, double* out) {
  dv s = r_spline(x, y, nx, n); memcpy(out, s.v, n * sizeof(double)); dv_free(&s);
}
OR_API int or_approx(const double* x, const double* y, int64_t nx, int64_t n, double* out) {
  dv a; int rc = r_approx_n(x, y, nx, n, &a); if (!rc) { memcpy(out, a.v, n * sizeof(double)); dv_free(&a); } return rc;
}
/* splinefun(x, y, method = "fmm")(u) (stats splines.c: SplineCoef + SplineEval) */
OR_API void or_spline_at(const double* x, const double* y, int64_t nx, const double* u, int64_t nu, double* out) {
  spl_t s = fmm_coef(x, y, nx); spl_eval(&s, u, out, nu); spl_free(&s);
}
/* approx(x, y, xout = v)$y, linear, rule = 1 (stats approx.c approx1): NaN outside */
OR_API void or_approx_at(const double* x, const double* y, int64_t nx, const double* v, int64_t nv, double* out) {
  for (int64_t l = 0; l < nv; ++l) out[l] = approx1(v[l], x, y, nx);
}
OR_API int64_t or_find_zero_crossing(const double* a, int64_t len, int64_t location) { return find_zero_crossing(a, len, location); }
OR_API void or_clumper(double* s, int64_t n, const double* minLength, int64_t nml) { clumper(s, n, minLength, nml); }
OR_API int64_t or_cross_fade(const double* a1, int64_t n1, const double* a2, int64_t n2, double sr, double crossLen, double* out) {
  dv x = dv_copy(a1, n1), y = dv_copy(a2, n2), z = cross_fade(x, y, sr, crossLen);
  memcpy(out, z.v, z.n * sizeof(double)); int64_t n = z.n; dv_free(&x); dv_free(&y); dv_free(&z); return n;
}
OR_API int or_vocal_fry_epochs(const double* roll, int64_t H, const double* pitch, int64_t nGC, double subFreq,
                               double subDep, double throwaway, double shortestEpoch, int64_t* starts, int64_t* ends,
                               int64_t* nrows, int64_t max_ep, double* mult_out, double* amp_out) {
  dv sf = dv_new(nGC), sd = dv_new(nGC);
  for (int64_t g = 0; g < nGC; ++g) { sf.v[g] = subFreq; sd.v[g] = subDep; }
  ampmat* m; int64_t *es, *ee, ne;
  int rc = get_vocal_fry(roll, H, pitch, nGC, sf.v, sd.v, throwaway, shortestEpoch, &m, &es, &ee, &ne);
  dv_free(&sf); dv_free(&sd);
  if (rc) return rc;
  int64_t mo = 0, ao = 0;
  for (int64_t e = 0; e < ne && e < max_ep; ++e) {
    starts[e] = es[e]; ends[e] = ee[e]; nrows[e] = m[e].nrow;
    if (mult_out) { memcpy(mult_out + mo, m[e].mult.v, m[e].nrow * sizeof(double)); mo += m[e].nrow; }
    if (amp_out) { memcpy(amp_out + ao, m[e].A.v, m[e].nrow * m[e].ncol * sizeof(double)); ao += m[e].nrow * m[e].ncol; }
  }
  for (int64_t e = 0; e < ne; ++e) ampmat_free(&m[e]);
  free(m); free(es); free(ee);
  return (int)ne;
}

/* ------------------------------------------------------------ soundgen() */
static void or_default_harm_params(sg_harm_params* p);
static const char* PV_NAMES[] = {"repeatBout","nSyl","sylLen","pauseLen","temperature","maleFemale","creakyBreathy",
  "nonlinBalance","nonlinDep","jitterDep","jitterLen","vibratoFreq","vibratoDep","shimmerDep","attackLen","rolloff",
  "rolloffOct","rolloffParab","rolloffParabHarm","rolloffKHz","rolloffLip","formantDep","formantDepStoch","vocalTract",
  "subFreq","subDep","shortestEpoch","amDep","amFreq","amShape","samplingRate","windowLength","rolloffNoise"};
/* permittedValues rows 1..'rolloffNoise' (R/presets.R:22-56): default, low, high */
static const double PV[33][3] = {{1,1,20},{1,1,10},{300,20,5000},{200,20,1000},{.025,0,1},{0,-1,1},{0,-1,1},
  {0,0,100},{50,0,100},{3,0,24},{1,1,100},{5,3,10},{0,0,3},{0,0,100},{50,0,200},{-12,-60,0},{-12,-30,10},
  {0,-50,50},{3,1,20},{-6,-20,0},{6,0,20},{1,0,5},{30,0,60},{15.5,2,100},{100,10,1000},{100,0,500},{300,50,500},
  {0,0,100},{30,10,100},{0,-1,1},{16000,8000,44100},{40,5,100},{-14,-20,20}};
OR_API int or_permitted_value(int i, const char** name, double* v3) {
  if (i < 0 || i >= 33) return SG_E_ARG;
  *name = PV_NAMES[i];
  v3[0] = PV[i][0]; v3[1] = PV[i][1]; v3[2] = PV[i][2];
  return 0;
}
#define PV_SYLLEN_LOW 20.0
#define PV_SYLLEN_HIGH 5000.0
#define PV_PAUSE_LOW 20.0
#define PV_PAUSE_HIGH 1000.0

static double* arg_slot(sg_soundgen_args* a, int i) {
  double* s[33] = {&a->repeatBout,&a->nSyl,&a->sylLen,&a->pauseLen,&a->temperature,&a->maleFemale,&a->creakyBreathy,
    &a->nonlinBalance,&a->nonlinDep,&a->jitterDep,&a->jitterLen,&a->vibratoFreq,&a->vibratoDep,&a->shimmerDep,&a->attackLen,
    &a->rolloff,&a->rolloffOct,&a->rolloffParab,&a->rolloffParabHarm,&a->rolloffKHz,&a->rolloffLip,&a->formantDep,
    &a->formantDepStoch,&a->vocalTract,&a->subFreq,&a->subDep,&a->shortestEpoch,&a->amDep,&a->amFreq,&a->amShape,
    &a->samplingRate,&a->windowLength,&a->rolloffNoise};
  return s[i];
}

/* anchors as owned arrays */
typedef struct { int64_t n; double *t, *v; } anc_t;
static anc_t anc_from(sg_anchors a) { anc_t r; r.n = a.n; r.t = NULL; r.v = NULL; if (a.n > 0) { r.t = (double*)malloc(a.n * sizeof(double)); r.v = (double*)malloc(a.n * sizeof(double)); memcpy(r.t, a.time, a.n * sizeof(double)); memcpy(r.v, a.value, a.n * sizeof(double)); } return r; }
static void anc_free(anc_t* a) { free(a->t); free(a->v); a->t = a->v = NULL; a->n = 0; }
static sg_anchors anc_view(const anc_t* a) { sg_anchors r; r.n = (int32_t)a->n; r.time = a->t; r.value = a->v; return r; }

/* R's sample() building blocks (pre-3.6 "Rounding") */
static int r_unif_index(rng_t* R, double dn, int64_t* out) { double u; int rc = rng_unif(R, &u); if (rc) return rc; *out = (int64_t)floor(dn * u); return 0; }
static void revsort(double* a0, int* ib0, int n) {  /* R sort.c revsort, 1-based */
#define a(k) a0[(k) - 1]
#define ib(k) ib0[(k) - 1]
  int l, j, ir, i; double ra; int ii;
  if (n <= 1) return;
  l = (n >> 1) + 1; ir = n;
  for (;;) {
    if (l > 1) { l = l - 1; ra = a(l); ii = ib(l); }
    else { ra = a(ir); ii = ib(ir); a(ir) = a(1); ib(ir) = ib(1); if (--ir == 1) { a(1) = ra; ib(1) = ii; return; } }
    i = l; j = l << 1;
    while (j <= ir) {
      if (j < ir && a(j) > a(j + 1)) ++j;
      if (ra > a(j)) { a(i) = a(j); ib(i) = ib(j); j += (i = j); } else j = ir + 1;
    }
    a(i) = ra; ib(i) = ii;
  }
#undef a
#undef ib
}
/* sample(x of length n, 1, prob) without replacement → 1-based index */
static int r_sample_prob1(rng_t* R, const double* prob, int n, int* out) {
  double p[8]; int perm[8]; double tot = 0;
  for (int i = 0; i < n; ++i) tot += prob[i];
  for (int i = 0; i < n; ++i) { p[i] = prob[i] / tot; perm[i] = i + 1; }
  revsort(p, perm, n);
  double u; int rc = rng_unif(R, &u); if (rc) return rc;
  double rT = u, mass = 0; int j;
  for (j = 0; j < n - 1; j++) { mass += p[j]; if (rT <= mass) break; }
  *out = perm[j];
  return 0;
}

/* wiggleAnchors() for 2-column (time, value) anchors, R/utilities_soundgen.R:634-735 */
static int wiggle_anchors(rng_t* R, anc_t* df, double T, double coef, const double* low, const double* high, int allRows) {
  if (df->n < 1) return 0;
  for (int64_t i = 0; i < df->n; ++i) if (isnan(df->t[i]) || isnan(df->v[i])) return 0;
  double prob[3] = {1 - T, T / 2, T / 2};
  int action; int rc = r_sample_prob1(R, prob, 3, &action); if (rc) return rc;
  if (action == 3) {  /* add */
    if (df->n == 1) {
      double m = df->v[0], sd = df->v[0] * T * coef, na;
      if ((rc = rnorm_bounded(R, 1, &m, 1, &sd, 1, &low[1], &high[1], 0, &na))) return rc;
      df->t = (double*)realloc(df->t, 2 * sizeof(double)); df->v = (double*)realloc(df->v, 2 * sizeof(double));
      df->t[1] = 1; df->v[1] = na; df->n = 2; df->t[0] = 0;
    } else {
      int64_t a1; if ((rc = r_unif_index(R, (double)df->n, &a1))) return rc; a1 += 1;
      int64_t di; if ((rc = r_unif_index(R, 2.0, &di))) return rc;
      int64_t dir = di == 0 ? -1 : 1;
      int64_t a2 = (a1 + dir < 1 || a1 + dir > df->n) ? a1 - dir : a1 + dir;
      int64_t i1 = a1 < a2 ? a1 : a2, i2 = a1 < a2 ? a2 : a1;
      double nt = 0, nv = 0; { long double st = 0, sv = 0; for (int64_t k = i1; k <= i2; ++k) { st += df->t[k - 1]; sv += df->v[k - 1]; } nt = (double)(st / (i2 - i1 + 1)); nv = (double)(sv / (i2 - i1 + 1)); }
      int64_t nn = i1 + 1 + (df->n - i2 + 1);
      double* t2 = (double*)malloc(nn * sizeof(double)); double* v2 = (double*)malloc(nn * sizeof(double)); int64_t q = 0;
      for (int64_t k = 1; k <= i1; ++k) { t2[q] = df->t[k - 1]; v2[q++] = df->v[k - 1]; }
      t2[q] = nt; v2[q++] = nv;
      for (int64_t k = i2; k <= df->n; ++k) { t2[q] = df->t[k - 1]; v2[q++] = df->v[k - 1]; }
      free(df->t); free(df->v); df->t = t2; df->v = v2; df->n = nn;
    }
  } else if (action == 2) {  /* remove */
    int64_t idx = 0;
    if (allRows) { if ((rc = r_unif_index(R, (double)df->n, &idx))) return rc; idx += 1; }
    else if (df->n > 2) { if ((rc = r_unif_index(R, (double)(df->n - 2), &idx))) return rc; idx += 2; }
    if (idx) { for (int64_t k = idx; k < df->n; ++k) { df->t[k - 1] = df->t[k]; df->v[k - 1] = df->v[k]; } df->n--; }
  }
  double orig0 = df->t[0], orig1 = df->t[df->n - 1];
  double rng_[2];
  if (df->n == 1) { rng_[0] = df->t[0]; rng_[1] = df->v[0]; }
  else {
    rng_[0] = fabs(r_max(df->t, df->n) - r_min(df->t, df->n)); rng_[1] = fabs(r_max(df->v, df->n) - r_min(df->v, df->n));
    if (rng_[0] == 0) rng_[0] = fabs(df->t[0]);
    if (rng_[1] == 0) rng_[1] = fabs(df->v[0]);
  }
  double* cols[2] = {df->t, df->v};
  for (int i = 0; i < 2; ++i) {
    double sd = rng_[i] * T * coef;
    double lo[64], hi[64], w[64];
    if (df->n > 64) return fail(SG_E_UNSUPPORTED, "wiggleAnchors: too many anchors");
    for (int64_t k = 0; k < df->n; ++k) { lo[k] = low[i]; hi[k] = high[i]; }
    if ((rc = rnorm_bounded(R, df->n, cols[i], df->n, &sd, 1, lo, hi, 0, w))) return rc;
    memcpy(cols[i], w, df->n * sizeof(double));
  }
  if (!allRows) { df->t[0] = orig0; df->t[df->n - 1] = orig1; }
  return 0;
}

/* divideIntoSyllables(), R/utilities_soundgen.R:515-566 */
static int divide_into_syllables(rng_t* R, int64_t nSyl, double sylLen, double pauseLen, double T,
                                 double* st, double* en) {
  if (nSyl == 1) { st[0] = 0; en[0] = sylLen; return 0; }
  double c = 0; int rc;
  for (int64_t s = 0; s < nSyl; ++s) {
    double lo1 = PV_SYLLEN_LOW, hi1 = PV_SYLLEN_HIGH, lo2 = PV_PAUSE_LOW, hi2 = PV_PAUSE_HIGH, sd1 = sylLen * T, sd2 = pauseLen * T, d, p;
    if ((rc = rnorm_bounded(R, 1, &sylLen, 1, &sd1, 1, &lo1, &hi1, 0, &d))) return rc;
    if ((rc = rnorm_bounded(R, 1, &pauseLen, 1, &sd2, 1, &lo2, &hi2, 0, &p))) return rc;
    double start = 1 + c, end = start + d;
    st[s] = start; en[s] = end; c = end + p;
  }
  return 0;
}

static int formants_moving(const sg_formants* F) {
  if (!F || F->n_formants <= 0) return 0;
  for (int f = 0; f < F->n_formants; ++f) if (F->n_points[f] > 1) return 1;
  return 0;
}

OR_API int or_soundgen(const sg_soundgen_args* A_in, const sg_random* rnd, double** out, int64_t* out_len) {
  int rc = 0;
  rng_t R = { rnd, 0, 0 };
  sg_soundgen_args A = *A_in;
  anc_t pitchA = anc_from(A.pitchAnchors), pitchG = anc_from(A.pitchAnchorsGlobal), noiseA = anc_from(A.noiseAnchors);
  anc_t amplA = anc_from(A.amplAnchors), amplG = anc_from(A.amplAnchorsGlobal), mouthA = anc_from(A.mouthAnchors);
  dv bout = dv_new(0), voiced = {0}, sound = {0}, filtered = {0};
  dv* unvoiced = NULL; int64_t nUnv = 0;
  double* pitchDeltas = NULL;
  double* ffreq = NULL;
  *out = NULL; *out_len = 0;
  /* range checks (R/soundgen.R:279-302) */
  for (int i = 0; i < 33; ++i) {
    double* s = arg_slot(&A, i);
    if (isnan(*s) || *s < PV[i][1] || *s > PV[i][2]) {
      if (A.invalidArgAction == 1) { char m[128]; snprintf(m, sizeof m, "%s must be between %g and %g", PV_NAMES[i], PV[i][1], PV[i][2]); rc = fail(SG_E_ARG, m); goto done; }
      else if (A.invalidArgAction == 0) *s = PV[i][0];
    }
  }
  double sr = A.samplingRate;
  double wlp = floor(A.windowLength / 1000 * sr / 2) * 2;
  /* hyper-parameters (R/soundgen.R:337-379) */
  if (A.creakyBreathy < 0) {
    A.nonlinBalance = fmin(100, A.nonlinBalance - A.creakyBreathy * 50);
    A.jitterDep = fmax(0, A.jitterDep - A.creakyBreathy / 2);
    A.shimmerDep = fmax(0, A.shimmerDep - A.creakyBreathy * 5);
    A.subDep = A.subDep * pow(2.0, -A.creakyBreathy);
  } else if (A.creakyBreathy > 0) {
    anc_free(&noiseA); noiseA.n = 2; noiseA.t = (double*)malloc(2 * sizeof(double)); noiseA.v = (double*)malloc(2 * sizeof(double));
    noiseA.t[0] = 0; noiseA.t[1] = A.sylLen + 100;
    for (int k = 0; k < 2; ++k) { noiseA.v[k] = -120 + A.creakyBreathy * 160; if (noiseA.v[k] > 40) noiseA.v[k] = 40; }
  }
  A.rolloff = A.rolloff - A.creakyBreathy * 10;
  A.rolloffOct = A.rolloffOct - A.creakyBreathy * 5;
  A.subFreq = 2 * (A.subFreq - 50) / (1 + exp(-.1 * (50 - A.nonlinDep))) + 50;
  A.jitterDep = 2 * A.jitterDep / (1 + exp(.1 * (50 - A.nonlinDep)));
  /* formants (possibly scaled by maleFemale): owned copies */
  int nF = A.formants.n_formants, nFN = A.formantsNoise.n_formants;
  int64_t totF = 0, totFN = 0;
  for (int f = 0; f < nF; ++f) totF += A.formants.n_points[f];
  for (int f = 0; f < nFN; ++f) totFN += A.formantsNoise.n_points[f];
  ffreq = (double*)malloc((totF + 1) * sizeof(double));
  if (totF) memcpy(ffreq, A.formants.freq, totF * sizeof(double));
  if (A.maleFemale != 0) {
    if (pitchA.n > 0) for (int64_t i = 0; i < pitchA.n; ++i) pitchA.v[i] *= pow(2.0, A.maleFemale);
    for (int64_t i = 0; i < totF; ++i) ffreq[i] *= pow(1.25, A.maleFemale);
    A.vocalTract = A.vocalTract * (1 - .25 * A.maleFemale);
  }
  sg_formants Fm = A.formants; Fm.freq = ffreq;
  /* nSyl / repeatBout stochastic rounding: rbinom(1, 1, p) — no draw when p == 0 */
  double nSyl = A.nSyl, repeatBout = A.repeatBout;
  /* rbinom(1, 1, p): R's inversion for size 1 (nmath/rbinom.c) -> (u >= 1 - p) for p <= .5, (u < p) above */
  { double p = nSyl - floor(nSyl); if (p != 0) { double u; TRY(rng_unif(&R, &u)); nSyl = floor(nSyl) + (p <= .5 ? (u >= 1 - p) : (u < p)); } }
  { double p = repeatBout - floor(repeatBout); if (p != 0) { double u; TRY(rng_unif(&R, &u)); repeatBout = floor(repeatBout) + (p <= .5 ? (u >= 1 - p) : (u < p)); } }
  int64_t nS = (int64_t)nSyl, nB = (int64_t)repeatBout;
  pitchDeltas = (double*)malloc((nS > 0 ? nS : 1) * sizeof(double));
  {
    int anyNZ = 0; for (int64_t i = 0; i < pitchG.n; ++i) if (pitchG.v[i] != 0) anyNZ = 1;
    if (pitchG.n > 0 && anyNZ && nS > 1) {
      dv pd; TRY(get_smooth_contour(anc_view(&pitchG), nS, 0, 1, 0, 0, 0, 0, 16000, &pd));
      for (int64_t s = 0; s < nS; ++s) pitchDeltas[s] = pow(2.0, pd.v[s] / 12);
      dv_free(&pd);
    } else for (int64_t s = 0; s < nS; ++s) pitchDeltas[s] = 1;
  }
  if (pitchA.n > 0) {
    double mn = r_min(pitchA.t, pitchA.n); if (mn < 0) for (int64_t i = 0; i < pitchA.n; ++i) pitchA.t[i] -= mn;
    double mx = r_max(pitchA.t, pitchA.n); if (mx > 1) for (int64_t i = 0; i < pitchA.n; ++i) pitchA.t[i] /= mx;
  }
  double T = A.temperature;
  int noiseAbove = 0; for (int64_t i = 0; i < noiseA.n; ++i) if (noiseA.v[i] > A.throwaway) noiseAbove = 1;
  int amplBelow = 0; for (int64_t i = 0; i < amplA.n; ++i) if (amplA.v[i] < -A.throwaway) amplBelow = 1;
  int wiggleNoise = T > 0 && noiseA.n > 0 && noiseAbove;
  int wiggleAmpl = T > 0 && amplA.n > 0 && amplBelow;
  sg_harm_params HP; or_default_harm_params(&HP);
  HP.attackLen = A.attackLen; HP.jitterDep = A.jitterDep; HP.jitterLen = A.jitterLen; HP.vibratoFreq = A.vibratoFreq;
  HP.vibratoDep = A.vibratoDep; HP.shimmerDep = A.shimmerDep; HP.creakyBreathy = A.creakyBreathy; HP.rolloff = A.rolloff;
  HP.rolloffOct = A.rolloffOct; HP.rolloffKHz = A.rolloffKHz; HP.rolloffParab = A.rolloffParab; HP.rolloffParabHarm = A.rolloffParabHarm;
  HP.temperature = T; HP.pitchDriftDep = A.tempEffects[3]; HP.pitchDriftFreq = A.tempEffects[4]; HP.shortestEpoch = A.shortestEpoch;
  HP.subFreq = A.subFreq; HP.subDep = A.subDep; HP.rolloffLip = A.rolloffLip; HP.amDep = A.amDep; HP.amFreq = A.amFreq;
  HP.nonlinBalance = A.nonlinBalance; HP.nonlinDep = A.nonlinDep; HP.pitchFloor = A.pitchFloor; HP.pitchCeiling = A.pitchCeiling;
  HP.pitchSamplingRate = A.pitchSamplingRate; HP.throwaway = A.throwaway; HP.samplingRate = sr; HP.overlap = A.overlap;
  static const double PV_VARY[9][2] = {{0,100},{0,200},{0,24},{0,100},{-60,0},{-30,10},{50,500},{10,1000},{0,500}};
  unvoiced = (dv*)calloc(nS > 0 ? nS : 1, sizeof(dv));
  for (int64_t b = 0; b < nB; ++b) {
    double sylDur, pauseDur;
    {
      double sd = (PV_SYLLEN_HIGH - PV_SYLLEN_LOW) * T * A.tempEffects[0], lo = PV_SYLLEN_LOW, hi = PV_SYLLEN_HIGH;
      if (A.sylLen >= lo && A.sylLen <= hi) TRY(rnorm_bounded(&R, 1, &A.sylLen, 1, &sd, 1, &lo, &hi, 0, &sylDur));
      else sylDur = A.sylLen;
      double sd2 = (PV_PAUSE_HIGH - PV_PAUSE_LOW) * T * A.tempEffects[0], lo2 = PV_PAUSE_LOW, hi2 = PV_PAUSE_HIGH;
      TRY(rnorm_bounded(&R, 1, &A.pauseLen, 1, &sd2, 1, &lo2, &hi2, 0, &pauseDur));
    }
    double* sst = (double*)malloc(nS * sizeof(double)); double* sen = (double*)malloc(nS * sizeof(double));
    rc = divide_into_syllables(&R, nS, sylDur, pauseDur, T * A.tempEffects[0], sst, sen);
    if (rc) { free(sst); free(sen); goto done; }
    double* ssi = (double*)malloc(nS * sizeof(double));
    for (int64_t s = 0; s < nS; ++s) ssi[s] = r_round(sst[s] * sr / 1000);
    ssi[0] = 1;
    if (noiseA.n > 0 && noiseA.t[0] != 0) {
      double shift = -r_round(noiseA.t[0] * sr / 1000);
      if (noiseA.t[0] < 0) ssi[0] = ssi[0] - shift;
      else for (int64_t s = 0; s < nS; ++s) ssi[s] -= shift;
    }
    dv_free(&voiced); voiced = dv_new(0);
    for (int64_t s = 0; s < nUnv; ++s) dv_free(&unvoiced[s]);
    nUnv = 0;
    sg_harm_params HPs = HP;
    for (int64_t s = 0; s < nS; ++s) {
      anc_t pA = anc_from(anc_view(&pitchA)), aA = anc_from(anc_view(&amplA));
      if (T > 0) {
        double* slots[9] = {&HPs.nonlinDep, &HPs.attackLen, &HPs.jitterDep, &HPs.shimmerDep, &HPs.rolloff, &HPs.rolloffOct, &HPs.shortestEpoch, &HPs.subFreq, &HPs.subDep};
        double base[9] = {HP.nonlinDep, HP.attackLen, HP.jitterDep, HP.shimmerDep, HP.rolloff, HP.rolloffOct, HP.shortestEpoch, HP.subFreq, HP.subDep};
        int rnd_[9] = {0, 1, 0, 0, 0, 0, 0, 1, 1};
        for (int p = 0; p < 9; ++p) {
          double l = PV_VARY[p][0], h = PV_VARY[p][1], sd = (h - l) * T / 10, v;
          rc = rnorm_bounded(&R, 1, &base[p], 1, &sd, 1, &l, &h, rnd_[p], &v);
          if (rc) { anc_free(&pA); anc_free(&aA); free(sst); free(sen); free(ssi); goto done; }
          *slots[p] = v;
        }
        if (pA.n > 0) { double lo[2] = {0, 25}, hi[2] = {1, 3500}; rc = wiggle_anchors(&R, &pA, T, A.tempEffects[5], lo, hi, 0); }
        if (!rc && wiggleNoise) { anc_t tmp = anc_from(anc_view(&noiseA)); double lo[2] = {-INFINITY, -120}, hi[2] = {INFINITY, 40}; rc = wiggle_anchors(&R, &tmp, T, A.tempEffects[6], lo, hi, 1); anc_free(&tmp); }
        if (!rc && wiggleAmpl) { double lo[2] = {0, 0}, hi[2] = {1, -A.throwaway}; rc = wiggle_anchors(&R, &aA, T, A.tempEffects[7], lo, hi, 0); }
        if (rc) { anc_free(&pA); anc_free(&aA); free(sst); free(sen); free(ssi); goto done; }
      }
      double dur = sen[s] - sst[s];
      dv pc = {0};
      if (pA.n > 0) {
        rc = get_smooth_contour(anc_view(&pA), (int64_t)r_round(dur * A.pitchSamplingRate / 1000), 1, 0, 1, A.pitchFloor, 1, A.pitchCeiling, A.pitchSamplingRate, &pc);
        if (rc) { anc_free(&pA); anc_free(&aA); free(sst); free(sen); free(ssi); goto done; }
        for (int64_t i = 0; i < pc.n; ++i) pc.v[i] *= pitchDeltas[s];
      }
      double minNoise = INFINITY; for (int64_t i = 0; i < noiseA.n; ++i) if (noiseA.v[i] < minNoise) minNoise = noiseA.v[i];
      dv syl = {0};
      if (dur < PV_SYLLEN_LOW || (noiseA.n > 0 && minNoise >= 40) || pA.n == 0) {
        syl = dv_new((int64_t)r_round(dur * sr / 1000));
      } else {
        double* w; int64_t wn;
        rc = gen_harm(pc.v, pc.n, &HPs, anc_view(&aA), &R, &w, &wn);
        if (rc) { dv_free(&pc); anc_free(&pA); anc_free(&aA); free(sst); free(sen); free(ssi); goto done; }
        syl.v = w; syl.n = wn;
      }
      dv_free(&pc);
      dv_append(&voiced, syl.v, syl.n); dv_free(&syl);
      if (s < nS - 1) dv_append_zeros(&voiced, (int64_t)floor((sst[s + 1] - sen[s]) * sr / 1000));
      if (noiseA.n > 0 && noiseAbove) {
        anc_t ns = anc_from(anc_view(&noiseA));
        for (int64_t i = 0; i < ns.n; ++i) if (ns.t[i] > 0) ns.t[i] = ns.t[i] * dur / A.sylLen;
        int64_t uvDur = (int64_t)r_round((r_max(ns.t, ns.n) - r_min(ns.t, ns.n)) * sr / 1000);
        double* envN = NULL; int64_t nInt = 0;
        if (nFN > 0) {
          {  /* R/soundgen.R:662-666: max(lengths(formantsNoise)) > 1 | mouth moves */
            int moving = A.formantsNoise_rlen == 0 || A.formantsNoise_rlen > 1;
            for (int64_t q = 0; q < mouthA.n; ++q) if (mouthA.v[q] != .5) moving = 1;
            nInt = moving ? (int64_t)r_round((r_max(ns.t, ns.n) - r_min(ns.t, ns.n)) / 10) : 1;
          }
          envN = (double*)malloc((size_t)(wlp / 2) * (nInt > 0 ? nInt : 1) * sizeof(double));
          rc = spectral_envelope(&R, wlp / 2, nInt, &A.formantsNoise, A.formantDep, A.rolloffLip, anc_view(&mouthA), 0, 0,
                                 A.vocalTract, T, A.tempEffects[1], A.tempEffects[2], A.formantDepStoch, 1, sr, 35400, envN);
          if (rc) { free(envN); anc_free(&ns); anc_free(&pA); anc_free(&aA); free(sst); free(sen); free(ssi); goto done; }
        }
        rc = generate_noise(&R, uvDur, anc_view(&ns), A.rolloffNoise, HPs.attackLen, (int64_t)wlp, sr, A.overlap, A.throwaway, envN, nInt, &unvoiced[s]);
        free(envN); anc_free(&ns);
        if (rc) { anc_free(&pA); anc_free(&aA); free(sst); free(sen); free(ssi); goto done; }
        nUnv = s + 1;
      }
      anc_free(&pA); anc_free(&aA);
    }
    dv_free(&sound); sound = dv_copy(voiced.v, voiced.n);
    if (nUnv > 0 && nFN == 0)
      for (int64_t s = 0; s < nUnv; ++s) { dv t = add_vectors(sound, unvoiced[s], ssi[s]); dv_free(&sound); sound = t; }
    {
      int below = 0; for (int64_t i = 0; i < amplG.n; ++i) if (amplG.v[i] < -A.throwaway) below = 1;
      if (amplG.n > 0 && below) {
        anc_t g2 = anc_from(anc_view(&amplG)); for (int64_t i = 0; i < g2.n; ++i) g2.v[i] = pow(2.0, g2.v[i] / 10);
        dv env; rc = get_smooth_contour(anc_view(&g2), sound.n, 0, 0, 1, 0, 1, -A.throwaway, sr, &env);
        anc_free(&g2);
        if (rc) { free(sst); free(sen); free(ssi); goto done; }
        for (int64_t i = 0; i < sound.n; ++i) sound.v[i] *= env.v[i];
        dv_free(&env);
      }
    }
    dv_free(&filtered);
    if (r_sum(sound.v, sound.n) == 0) filtered = dv_copy(sound.v, sound.n);
    else {
      double fl = floor((double)sound.n / 2); if (fl < wlp) wlp = fl;
      int64_t wl = (int64_t)wlp;
      dv step = r_seq_by(1, (double)(sound.n - wl > 1 ? sound.n - wl : 1), (double)wl - (A.overlap * (double)wl / 100));
      int64_t nc = step.n, nr = wl / 2; dv_free(&step);
      int moving = formants_moving(&Fm);
      int mouthMoves = 0; for (int64_t i = 0; i < mouthA.n; ++i) if (mouthA.v[i] != .5) mouthMoves = 1;
      if (mouthA.n > 0 && mouthMoves) moving = 1;
      int64_t nInt = moving ? nc : 1;
      double* env = (double*)malloc(nr * nInt * sizeof(double));
      rc = spectral_envelope(&R, (double)wl / 2, nInt, &Fm, A.formantDep, A.rolloffLip, anc_view(&mouthA), 0, 0, A.vocalTract, T,
                             A.tempEffects[1], A.tempEffects[2], A.formantDepStoch, 1, sr, 35400, env);
      if (!rc) rc = formant_filter(sound.v, sound.n, env, nInt, wl, A.overlap, &filtered);
      free(env);
      if (rc) { free(sst); free(sen); free(ssi); goto done; }
    }
    if (nUnv > 0 && nFN > 0)
      for (int64_t s = 0; s < nUnv; ++s) { dv t = add_vectors(filtered, unvoiced[s], ssi[s]); dv_free(&filtered); filtered = t; }
    if (A.amDep > 0) {
      dv sig = get_sigmoid(filtered.n, sr, A.amFreq, A.amShape, 1);
      for (int64_t i = 0; i < filtered.n; ++i) filtered.v[i] *= 1 - sig.v[i] * A.amDep / 100;
      dv_free(&sig);
    }
    if (b == 0) { dv_free(&bout); bout = dv_copy(filtered.v, filtered.n); }
    else { dv_append_zeros(&bout, (int64_t)(A.pauseLen * sr / 1000)); dv_append(&bout, filtered.v, filtered.n); }
    free(sst); free(sen); free(ssi);
  }
  if (!isnan(A.addSilence)) {
    int64_t n = (int64_t)r_round(sr / 1000 * A.addSilence);
    dv o = dv_new(n); dv_append(&o, bout.v, bout.n); dv_append_zeros(&o, n); dv_free(&bout); bout = o;
  }
  *out = bout.v; *out_len = bout.n; bout.v = NULL;
done:
  free(ffreq);
  anc_free(&pitchA); anc_free(&pitchG); anc_free(&noiseA); anc_free(&amplA); anc_free(&amplG); anc_free(&mouthA);
  dv_free(&bout); dv_free(&voiced); dv_free(&sound); dv_free(&filtered);
  if (unvoiced) { for (int64_t s = 0; s < nUnv; ++s) dv_free(&unvoiced[s]); free(unvoiced); }
  free(pitchDeltas);
  (void)totFN;
  return rc;
}

/* defaults (R/source.R:173-205, R/soundgen.R:208-277); the oracle defines
 * its own copy so it does not link the product library. */
static void or_default_harm_params(sg_harm_params* p) {
  p->attackLen = 50; p->nonlinBalance = 0; p->nonlinDep = 0; p->jitterDep = 0; p->jitterLen = 1;
  p->vibratoFreq = 100; p->vibratoDep = 0; p->shimmerDep = 0; p->creakyBreathy = 0;
  p->rolloff = -18; p->rolloffOct = -2; p->rolloffKHz = -6; p->rolloffParab = 0; p->rolloffParabHarm = 3;
  p->rolloffLip = 6; p->rolloff_perAmpl = 12; p->temperature = 0; p->pitchDriftDep = .5; p->pitchDriftFreq = .125;
  p->randomWalk_trendStrength = .5; p->shortestEpoch = 300; p->subFreq = 100; p->subDep = 0; p->amDep = 0;
  p->amFreq = 30; p->overlap = 75; p->samplingRate = 16000; p->pitchFloor = 75; p->pitchCeiling = 3500;
  p->pitchSamplingRate = 3500; p->throwaway = -120;
}
