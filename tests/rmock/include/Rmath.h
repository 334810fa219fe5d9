/* Test double of Rmath.h (see Rinternals.h here): the draws come from the
 * library's restatement of R's generator (sg_rrng), seeded by rm_set_seed. */
#ifndef RMOCK_RMATH_H
#define RMOCK_RMATH_H
double norm_rand(void);
double unif_rand(void);
double rgamma(double shape, double scale);
#endif
