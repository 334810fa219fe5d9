// sg_loess.cpp — see sg_loess.h. Host-side (planner) code.
#include "sg_loess.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <numeric>

#include "sg_plan.h"

namespace sg {

namespace {

// thin SVD of a tall m x 3 matrix (columns a[j]) by one-sided Jacobi:
// on return a[j] = sigma_j u_j, V holds the right singular vectors
void jacobi_svd3(std::vector<double> (&a)[3], double V[3][3]) {
  const size_t m = a[0].size();
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) V[i][j] = i == j ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 60; ++sweep) {
    double worst = 0;
    for (int p = 0; p < 2; ++p)
      for (int q = p + 1; q < 3; ++q) {
        double app = 0, aqq = 0, apq = 0;
        for (size_t i = 0; i < m; ++i) {
          app += a[p][i] * a[p][i];
          aqq += a[q][i] * a[q][i];
          apq += a[p][i] * a[q][i];
        }
        if (apq == 0) continue;
        worst = std::max(worst, std::fabs(apq) / std::sqrt(app * aqq));
        const double zeta = (aqq - app) / (2 * apq);
        const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1 + zeta * zeta));
        const double c = 1 / std::sqrt(1 + t * t), s = c * t;
        for (size_t i = 0; i < m; ++i) {
          const double ap = a[p][i], aq = a[q][i];
          a[p][i] = c * ap - s * aq;
          a[q][i] = s * ap + c * aq;
        }
        for (int i = 0; i < 3; ++i) {
          const double vp = V[i][p], vq = V[i][q];
          V[i][p] = c * vp - s * vq;
          V[i][q] = s * vp + c * vq;
        }
      }
    if (worst < 1e-15) break;
  }
}

// local quadratic at vertex v over the nf nearest points: value and slope.
// Returns false for a zero-width neighbourhood (rho = 0: a vertex on a data
// point with floor(n f) = 1), where R's tricube weights are 0/0 and the vertex
// value is NaN.
bool vertex_fit(const double* x, const double* y, int n, int nf, double f, double v, double& val, double& slope) {
  std::vector<double> d2(n);
  std::vector<int> ord(n);
  for (int i = 0; i < n; ++i) d2[i] = (x[i] - v) * (x[i] - v);
  std::iota(ord.begin(), ord.end(), 0);
  std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return d2[a] < d2[b]; });
  const double rho = d2[ord[nf - 1]] * std::max(1.0, f);
  if (!(rho > 0)) {
    val = slope = std::nan("");
    return false;
  }
  const size_t m = (size_t)std::max(nf, 3);
  std::vector<double> cols[3];
  for (auto& c : cols) c.assign(m, 0.0);
  std::vector<double> eta(m, 0.0);
  for (int i = 0; i < nf; ++i) {
    const int k = ord[i];
    const double r = std::sqrt(d2[k] / rho);
    const double tc = 1 - r * r * r;
    const double w = std::sqrt(tc * tc * tc);  // sqrt of the tricube weight (row scaling)
    const double dx = x[k] - v;
    cols[0][i] = w;
    cols[1][i] = w * dx;
    cols[2][i] = w * dx * dx;
    eta[i] = w * y[k];
  }
  double colnor[3];
  for (int j = 0; j < 3; ++j) {  // equilibrate columns
    double sc = 0;
    for (double e : cols[j]) sc += e * e;
    sc = std::sqrt(sc);
    if (sc > 0) {
      for (double& e : cols[j]) e /= sc;
      colnor[j] = sc;
    } else {
      colnor[j] = 1;
    }
  }
  double V[3][3];
  jacobi_svd3(cols, V);
  double sigma[3];
  for (int j = 0; j < 3; ++j) {
    double s2 = 0;
    for (double e : cols[j]) s2 += e * e;
    sigma[j] = std::sqrt(s2);
  }
  const double tol = std::max({sigma[0], sigma[1], sigma[2]}) * (100 * DBL_EPSILON);
  double gam[3];
  for (int j = 0; j < 3; ++j) {  // pseudo-inverse: gamma_j = u_j . eta / sigma_j above the tolerance
    if (sigma[j] > tol) {
      double ue = 0;
      for (size_t i = 0; i < m; ++i) ue += cols[j][i] / sigma[j] * eta[i];
      gam[j] = ue / sigma[j];
    } else {
      gam[j] = 0;
    }
  }
  double s0 = 0, s1 = 0;
  for (int j = 0; j < 3; ++j) {
    s0 += V[0][j] * gam[j];
    s1 += V[1][j] * gam[j];
  }
  val = s0 / colnor[0];
  slope = s1 / colnor[1];
  return true;
}

}  // namespace

double LoessFit::eval(double z) const {
  int p = 0;
  while (split[p]) p = z <= xi[p] ? son_lo[p] : son_hi[p];
  return hermite(p, z);
}

double LoessFit::eval_seq(double z, int& p) const {
  // z non-decreasing over the calls: the leaf found for an earlier z holds every
  // z up to its upper vertex (the tree sends z <= split to the low son, and that
  // vertex is the split), or every z when its upper vertex is the outer one (1)
  if (p < 0 || !(cv1[p] == 1 || z <= vx[cv1[p]])) {
    p = 0;
    while (split[p]) p = z <= xi[p] ? son_lo[p] : son_hi[p];
  }
  return hermite(p, z);
}

double LoessFit::hermite(int p, double z) const {
  const int a = cv0[p], b = cv1[p];
  const double v0 = vx[a], v1 = vx[b];
  const double h = (z - v0) / (v1 - v0);
  const double phi0 = (1 - h) * (1 - h) * (1 + 2 * h), phi1 = h * h * (3 - 2 * h);
  const double psi0 = h * (1 - h) * (1 - h), psi1 = -h * h * (1 - h);
  return phi0 * val[a] + phi1 * val[b] + (psi0 * slope[a] + psi1 * slope[b]) * (v1 - v0);
}

namespace {
// Is T(u) < thr for some u = 1..len (the valueFloor test of the refit loop)?
// On a leaf cell the Hermite cubic's minimum over its part of [1, len]
// (endpoints and stationary points, power basis) bounds its values at the
// integers there; only a cell whose bound comes within a rounding margin of
// thr has its integers evaluated one by one, as are integers outside the
// vertex range. Same answer as evaluating all len points.
bool dips_below(const LoessFit& T, int64_t len, double thr) {
  double vmin = INFINITY, vmax = -INFINITY;
  for (double v : T.vx) {
    vmin = std::min(vmin, v);
    vmax = std::max(vmax, v);
  }
  auto scan = [&](int64_t z0, int64_t z1) {
    for (int64_t z = std::max<int64_t>(z0, 1); z <= std::min<int64_t>(z1, len); ++z)
      if (T.eval((double)z) < thr) return true;
    return false;
  };
  if (!(vmin <= vmax) || scan(1, (int64_t)std::ceil(vmin) - 1) || scan((int64_t)std::floor(vmax) + 1, len)) return true;
  for (size_t p = 0; p < T.split.size(); ++p) {
    if (T.split[p]) continue;
    const int a = T.cv0[p], b = T.cv1[p];
    const double v0 = T.vx[a], v1 = T.vx[b];
    const double lo = std::max(std::min(v0, v1), 1.0), hi = std::min(std::max(v0, v1), (double)len);
    if (!(lo <= hi) || std::ceil(lo) > std::floor(hi)) continue;
    const double D = v1 - v0, y0 = T.val[a], y1 = T.val[b], m0 = T.slope[a] * D, m1 = T.slope[b] * D;
    const double c1 = m0, c2 = 3 * (y1 - y0) - 2 * m0 - m1, c3 = 2 * (y0 - y1) + m0 + m1;
    auto f = [&](double h) { return y0 + h * (c1 + h * (c2 + h * c3)); };
    const double hlo = std::min((lo - v0) / D, (hi - v0) / D), hhi = std::max((lo - v0) / D, (hi - v0) / D);
    double fmin = std::min(f(hlo), f(hhi));
    // stationary points: qa h^2 + qb h + qc = 0 (the cancellation-free pair of roots;
    // qa may be a rounding residue of a quadratic piece)
    const double qa = 3 * c3, qb = 2 * c2, qc = c1;
    const double disc = qb * qb - 4 * qa * qc;
    if (disc >= 0) {
      const double q = -0.5 * (qb + std::copysign(std::sqrt(disc), qb));
      for (double r : {q != 0 ? qc / q : NAN, qa != 0 ? q / qa : NAN})
        if (r > hlo && r < hhi) fmin = std::min(fmin, f(r));
    }
    const double margin = 1e-9 * (std::fabs(y0) + std::fabs(y1) + std::fabs(m0) + std::fabs(m1) + 1);
    if (!(fmin >= thr + margin) && scan((int64_t)std::ceil(lo), (int64_t)std::floor(hi))) return true;
  }
  return false;
}
}  // namespace

bool loess_fit(const double* x, const double* y, int n, double f, LoessFit& T) {
  if (n < 1) throw SgError(SG_E_DOMAIN, "loess: no data");
  if (std::floor(n * f + 1e-5) <= 0) throw SgError(SG_E_DOMAIN, "loess: span is too small");
  const int nf = (int)std::min<double>(n, std::floor(n * f));
  if (nf <= 0) throw SgError(SG_E_DOMAIN, "loess: span is too small");
  const int fc = (int)std::floor(n * (f * 0.2));
  double lo = x[0], hi = x[0];
  for (int i = 1; i < n; ++i) {
    lo = std::min(lo, x[i]);
    hi = std::max(hi, x[i]);
  }
  const double mu = 0.005 * std::max(hi - lo, 1e-10 * std::max(std::fabs(lo), std::fabs(hi)) + 1e-30);
  T = LoessFit{};
  T.xmin = lo;
  T.xmax = hi;
  T.vx = {lo - mu, hi + mu};
  std::vector<int> cl{1}, cu{n};
  T.cv0 = {0};
  T.cv1 = {1};
  // k-d tree, cells in breadth-first order (cell p: sorted points l..u, 1-based)
  for (size_t p = 0; p < cl.size(); ++p) {
    const int l = cl[p], u = cu[p];
    bool leaf = (u - l + 1) <= fc || (T.vx[T.cv1[p]] - T.vx[T.cv0[p]]) <= 0;
    int m = (l + u) / 2;
    if (!leaf) {
      int off = 0;  // ties go with the high son
      while (!(m + off >= u || m + off < l)) {
        if (x[m + off - 1] == x[m + off]) {
          off = -off;
          if (off >= 0) ++off;
        } else {
          m += off;
          break;
        }
      }
      leaf = T.vx[T.cv0[p]] == x[m - 1] || T.vx[T.cv1[p]] == x[m - 1];
    }
    T.split.push_back(leaf ? 0 : 1);
    T.xi.push_back(leaf ? 0.0 : x[m - 1]);
    T.son_lo.push_back(-1);
    T.son_hi.push_back(-1);
    if (leaf) continue;
    const int vn = (int)T.vx.size();
    T.vx.push_back(x[m - 1]);
    const int a = (int)cl.size(), b = a + 1;
    T.son_lo[p] = a;
    T.son_hi[p] = b;
    cl.push_back(l);
    cu.push_back(m);
    T.cv0.push_back(T.cv0[p]);
    T.cv1.push_back(vn);
    cl.push_back(m + 1);
    cu.push_back(u);
    T.cv0.push_back(vn);
    T.cv1.push_back(T.cv1[p]);
  }
  T.val.resize(T.vx.size());
  T.slope.resize(T.vx.size());
  bool finite = true;
  for (size_t v = 0; v < T.vx.size(); ++v) finite &= vertex_fit(x, y, n, nf, f, T.vx[v], T.val[v], T.slope[v]);
  return finite;
}

LoessFit smooth_loess(const double* t, const double* v, int64_t n, int64_t len, double duration_ms, bool has_floor,
                      double vfloor) {
  // anchors_long[anchor_time_points] = value (R/smoothContours.R:121-125):
  // positions truncate, 0 drops, a repeated position keeps the last value
  std::vector<double> xs, ys;
  for (int64_t i = 0; i < n; ++i) {
    double tp = t[i] / 1.0 * (double)len;
    if (tp == 0) tp = 1;
    const int64_t idx = (int64_t)tp;
    if (idx < 1 || idx > len) continue;
    auto it = std::find(xs.begin(), xs.end(), (double)idx);
    if (it == xs.end()) {
      xs.push_back((double)idx);
      ys.push_back(v[i]);
    } else {
      ys[it - xs.begin()] = v[i];
    }
  }
  std::vector<int> ord(xs.size());
  std::iota(ord.begin(), ord.end(), 0);
  std::sort(ord.begin(), ord.end(), [&](int a, int b) { return xs[a] < xs[b]; });
  std::vector<double> x(xs.size()), y(xs.size());
  for (size_t i = 0; i < ord.size(); ++i) {
    x[i] = xs[ord[i]];
    y[i] = ys[ord[i]];
  }
  double span = (1 / (1 + std::exp(duration_ms / 500)) + 0.5) / std::pow(1.1, (double)(n - 3));
  // smoothContour = try(predict(l, time)); while (try-error) span = span + 0.1
  // (R/smoothContours.R:133-143). predict()'s .C(C_loess_ifit, ..., vval) stops
  // on a NaN vertex value (NAOK = FALSE), so a zero-width fit is that error.
  // Restated, unpinned against R output.
  LoessFit T;  // the finite fit found here is the floor loop's first fit
  for (int k = 0;; ++k) {
    T = LoessFit();
    if (loess_fit(x.data(), y.data(), (int)x.size(), span, T)) break;
    if (k == 200) throw SgError(SG_E_DOMAIN, "loess: no span gives a finite fit");
    span = span + 0.1;
  }
  for (int iter = 0; iter < 200; ++iter) {
    // a zero-width fit inside the valueFloor loop leaves R comparing a
    // try-error string with valueFloor: not restated
    if (iter > 0) {
      T = LoessFit();
      if (!loess_fit(x.data(), y.data(), (int)x.size(), span, T))
        throw SgError(SG_E_UNSUPPORTED, "loess: zero-width fit inside the valueFloor refits");
    }
    const bool below = has_floor && dips_below(T, len, vfloor - 1e-6);
    if (!below) return T;
    span = span / 1.1;  // less smoothing while the contour dips below the floor
  }
  throw SgError(SG_E_DOMAIN, "loess: contour stays below valueFloor");
}

}  // namespace sg
