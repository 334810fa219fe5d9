// sg_loess.h — 1-D loess for getSmoothContour() (R/smoothContours.R:119-154).
//
// loess(y ~ x, span = f) + predict(., 1:len) with R 3.4 stats defaults:
// degree 2, family "gaussian", surface "interpolate", cell 0.2. Follows the
// published netlib dloess algorithm carried by R's stats/src/loessf.f and
// loessc.c: bounding box widened by 0.5% (ehg126), k-d tree split at medians
// until a cell holds <= floor(n f cell) points (ehg124), a local quadratic
// fit at every vertex over the floor(n f) nearest points with tricube weights,
// equilibrated columns and an SVD pseudo-inverse (ehg127), cubic Hermite
// interpolation between a cell's vertices (ehg128). Parity vs R is unpinned
// (R is absent from this environment); see DESIGN.md.
#pragma once
#include <cstdint>
#include <vector>

namespace sg {

struct LoessFit {
  std::vector<double> vx, val, slope;  // vertices (creation order) with fitted value and slope
  std::vector<int> cv0, cv1, split, son_lo, son_hi;
  std::vector<double> xi;
  double xmin = 0, xmax = 0;           // data range (predict gives NA outside)
  double eval(double z) const;         // Hermite interpolation in the leaf cell containing z
  // eval() for non-decreasing z: *leaf (start at -1) carries the last leaf between calls
  double eval_seq(double z, int& leaf) const;
  double hermite(int leaf, double z) const;
};

// fit; throws SgError for spans R rejects. Returns false when a vertex value
// is NaN (zero-width neighbourhood), which makes R's predict() stop.
bool loess_fit(const double* x, const double* y, int n, double f, LoessFit& out);

// getSmoothContour's loess branch: anchor times t (already scaled to [0, 1])
// and values -> the fit R evaluates on 1..len (span + 0.1 while predict()
// fails on a NaN vertex, then span / 1.1 while a value falls below
// valueFloor - 1e-6). Returns the final fit.
LoessFit smooth_loess(const double* t, const double* v, int64_t n, int64_t len, double duration_ms, bool has_floor,
                      double vfloor);

}  // namespace sg
