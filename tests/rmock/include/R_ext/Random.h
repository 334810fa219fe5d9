/* Test double of R_ext/Random.h (see ../Rinternals.h). */
#ifndef RMOCK_RANDOM_H
#define RMOCK_RANDOM_H
void GetRNGstate(void);
void PutRNGstate(void);
double unif_rand(void);
double norm_rand(void);
#endif
