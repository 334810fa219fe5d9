/* Test double of the part of R's C API (R 3.4, Rinternals.h) that
 * r/src/sg_r_shim.c uses, so the shim compiles and runs here without R
 * (tests/test_r_shim.py). Semantics follow R's documented behaviour for these
 * calls; objects are never garbage-collected. NOT part of the product. */
#ifndef RMOCK_RINTERNALS_H
#define RMOCK_RINTERNALS_H
#include <limits.h>
#include <stddef.h>
#include <stdint.h>

typedef ptrdiff_t R_xlen_t;
typedef struct rm_sexp* SEXP;
typedef unsigned int SEXPTYPE;
enum { NILSXP = 0, CHARSXP = 9, LGLSXP = 10, INTSXP = 13, REALSXP = 14, STRSXP = 16, VECSXP = 19 };

extern SEXP R_NilValue;
extern SEXP R_NamesSymbol;
extern SEXP R_DimSymbol;
extern double R_NaReal;
extern int R_NaInt;
#define NA_REAL R_NaReal
#define NA_INTEGER R_NaInt

int TYPEOF(SEXP x);
R_xlen_t Rf_xlength(SEXP x);
double* REAL(SEXP x);
int* INTEGER(SEXP x);
SEXP VECTOR_ELT(SEXP x, R_xlen_t i);
SEXP SET_VECTOR_ELT(SEXP x, R_xlen_t i, SEXP v);
SEXP STRING_ELT(SEXP x, R_xlen_t i);
const char* CHAR(SEXP x);
SEXP Rf_getAttrib(SEXP x, SEXP name);
int Rf_isNull(SEXP x);
int Rf_isNewList(SEXP x);
int Rf_isMatrix(SEXP x);
int Rf_nrows(SEXP x);
int Rf_ncols(SEXP x);
double Rf_asReal(SEXP x);
int Rf_asInteger(SEXP x);
SEXP Rf_allocVector(SEXPTYPE type, R_xlen_t n);
SEXP Rf_allocMatrix(SEXPTYPE type, int nrow, int ncol);
SEXP Rf_xlengthgets(SEXP x, R_xlen_t n);
SEXP Rf_protect(SEXP x);
void Rf_unprotect(int n);
#define PROTECT(x) Rf_protect(x)
#define UNPROTECT(n) Rf_unprotect(n)
void Rf_error(const char* fmt, ...) __attribute__((noreturn, format(printf, 1, 2)));
void Rf_warning(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
char* R_alloc(size_t n, int size);
#endif
