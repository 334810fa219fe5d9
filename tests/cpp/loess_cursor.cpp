// LoessFit::eval_seq (leaf cursor, non-decreasing z) against the k-d tree walk
// LoessFit::eval, bit for bit, over random anchor sets (tests/test_loess_cursor.py).
#include "sg_loess.h"
#include <cstdio>
#include <algorithm>
#include <random>
#include <cstring>
using namespace sg;
int main() {
  std::mt19937_64 g(7);
  std::uniform_real_distribution<double> U(0, 1);
  long bad = 0, tot = 0;
  for (int trial = 0; trial < 400; ++trial) {
    int n = 3 + (int)(U(g) * 10);
    int64_t len = 2 + (int64_t)(U(g) * 3000);
    std::vector<double> t(n), v(n);
    for (int i = 0; i < n; ++i) { t[i] = (i == 0) ? 0 : (trial % 3 == 0 ? (double)i / (n - 1) : U(g)); v[i] = 50 + 400 * U(g); }
    std::sort(t.begin(), t.end());
    LoessFit T;
    try { T = smooth_loess(t.data(), v.data(), n, len, len / 44.1, false, 0); } catch (...) { continue; }
    int leaf = -1;
    for (int64_t k = 0; k < len; ++k) {
      double z = (double)(k + 1), a = T.eval(z), b = T.eval_seq(z, leaf);
      ++tot; if (memcmp(&a, &b, 8) && !(a != a && b != b)) ++bad;
    }
    // also half-steps and repeated z
    leaf = -1;
    for (int64_t k = 0; k < 2 * len; ++k) {
      double z = 0.5 * (double)k, a = T.eval(z), b = T.eval_seq(z, leaf);
      ++tot; if (memcmp(&a, &b, 8) && !(a != a && b != b)) ++bad;
    }
  }
  printf("tot %ld bad %ld\n", tot, bad);
  return bad != 0;
}
