// The host planner's R-base numerics (sg_rmath.h: fmm_spline + Spline::eval,
// approx1) evaluated on cases read from stdin, for the R-pinned checks in
// tests/test_r_pins.py. Input, one case per line:
//   S|L nx x_1..x_nx y_1..y_nx nu u_1..u_nu
// output: one line of nu values (%.17g) per case.
#include "sg_rmath.h"
#include <cstdio>
using namespace sg;
int main() {
  char kind;
  while (std::scanf(" %c", &kind) == 1) {
    long nx, nu;
    if (std::scanf("%ld", &nx) != 1) return 2;
    vec x(nx), y(nx);
    for (auto& v : x) if (std::scanf("%lf", &v) != 1) return 2;
    for (auto& v : y) if (std::scanf("%lf", &v) != 1) return 2;
    if (std::scanf("%ld", &nu) != 1) return 2;
    vec u(nu);
    for (auto& v : u) if (std::scanf("%lf", &v) != 1) return 2;
    if (kind == 'S') {
      Spline s = fmm_spline(x, y);
      int64_t i = 0;
      for (long l = 0; l < nu; ++l) std::printf("%.17g ", s.eval(u[l], i));
    } else {
      for (long l = 0; l < nu; ++l) std::printf("%.17g ", approx1(u[l], x.data(), y.data(), nx));
    }
    std::printf("\n");
  }
  return 0;
}
