/* rmock.c — a test double of the R runtime pieces r/src/sg_r_shim.c calls
 * (see include/Rinternals.h), plus a small driver API for
 * tests/test_r_shim.py: build R objects, call a routine by the name the shim
 * registered (R_registerRoutines) with R's error semantics (Rf_error unwinds
 * to the caller, as R's longjmp does), read results back. R's RNG is the
 * library's restatement (sg_rrng: Mersenne-Twister + Inversion, pinned to
 * R's printed draws in tests/test_rrng.py). Test infrastructure only. */
#include <math.h>
#include <setjmp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "R.h"
#include "R_ext/Rdynload.h"
#include "Rmath.h"
#include "soundgen_hip.h"

struct rm_sexp {
  int type;
  R_xlen_t len;
  void* data;     /* double / int / SEXP / char* per type */
  SEXP names;     /* STRSXP or NULL */
  int nrow, ncol; /* dim attribute (matrices); 0 = none */
};

static struct rm_sexp nil = {NILSXP, 0, NULL, NULL, 0, 0};
static struct rm_sexp names_sym = {NILSXP, 0, NULL, NULL, 0, 0};
static struct rm_sexp dim_sym = {NILSXP, 0, NULL, NULL, 0, 0};
SEXP R_NilValue = &nil;
SEXP R_NamesSymbol = &names_sym;
SEXP R_DimSymbol = &dim_sym;
double R_NaReal;
int R_NaInt = INT_MIN;

static jmp_buf* g_jmp;
static char g_err[1024];
static int g_protect;
static sg_rrng* g_rng;

__attribute__((constructor)) static void rm_init_na(void) {
  /* R's NA_real_: a NaN whose low word is 1954 */
  uint64_t bits = 0x7FF00000000007A2ull;
  memcpy(&R_NaReal, &bits, sizeof bits);
}

static SEXP mk(int type, R_xlen_t n) {
  SEXP x = (SEXP)calloc(1, sizeof *x);
  size_t el = type == REALSXP ? sizeof(double) : (type == INTSXP || type == LGLSXP) ? sizeof(int) : sizeof(SEXP);
  x->type = type;
  x->len = n;
  x->data = calloc((size_t)(n > 0 ? n : 1), el);
  if (type == VECSXP || type == STRSXP)
    for (R_xlen_t i = 0; i < n; ++i) ((SEXP*)x->data)[i] = R_NilValue;
  return x;
}

int TYPEOF(SEXP x) { return x->type; }
R_xlen_t Rf_xlength(SEXP x) { return x->len; }
double* REAL(SEXP x) {
  if (x->type != REALSXP) Rf_error("REAL() can only be applied to a 'numeric', not a '%d'", x->type);
  return (double*)x->data;
}
int* INTEGER(SEXP x) {
  if (x->type != INTSXP && x->type != LGLSXP) Rf_error("INTEGER() can only be applied to an 'integer'");
  return (int*)x->data;
}
SEXP VECTOR_ELT(SEXP x, R_xlen_t i) {
  if (x->type != VECSXP || i < 0 || i >= x->len) Rf_error("VECTOR_ELT: bad access");
  return ((SEXP*)x->data)[i];
}
SEXP SET_VECTOR_ELT(SEXP x, R_xlen_t i, SEXP v) {
  if (x->type != VECSXP || i < 0 || i >= x->len) Rf_error("SET_VECTOR_ELT: bad access");
  return ((SEXP*)x->data)[i] = v;
}
SEXP STRING_ELT(SEXP x, R_xlen_t i) {
  if (x->type != STRSXP || i < 0 || i >= x->len) Rf_error("STRING_ELT: bad access");
  return ((SEXP*)x->data)[i];
}
const char* CHAR(SEXP x) {
  if (x->type != CHARSXP) Rf_error("CHAR() on a non-CHARSXP");
  return (const char*)x->data;
}
SEXP Rf_getAttrib(SEXP x, SEXP name) {
  if (name == R_NamesSymbol) return x->names ? x->names : R_NilValue;
  if (name == R_DimSymbol && x->nrow) {
    SEXP d = mk(INTSXP, 2);
    ((int*)d->data)[0] = x->nrow;
    ((int*)d->data)[1] = x->ncol;
    return d;
  }
  return R_NilValue;
}
int Rf_isNull(SEXP x) { return x->type == NILSXP; }
int Rf_isNewList(SEXP x) { return x->type == NILSXP || x->type == VECSXP; }
int Rf_isMatrix(SEXP x) { return x->nrow > 0 || (x->ncol > 0); }
int Rf_nrows(SEXP x) { return x->nrow ? x->nrow : (int)x->len; }
int Rf_ncols(SEXP x) { return x->nrow ? x->ncol : 1; }
double Rf_asReal(SEXP x) {
  if (x->len >= 1) {
    if (x->type == REALSXP) return ((double*)x->data)[0];
    if (x->type == INTSXP || x->type == LGLSXP) {
      int v = ((int*)x->data)[0];
      return v == NA_INTEGER ? NA_REAL : (double)v;
    }
  }
  return NA_REAL;
}
int Rf_asInteger(SEXP x) {
  if (x->len >= 1) {
    if (x->type == INTSXP || x->type == LGLSXP) return ((int*)x->data)[0];
    if (x->type == REALSXP) {
      double v = ((double*)x->data)[0];
      return (isnan(v) || v >= 2147483648.0 || v <= -2147483649.0) ? NA_INTEGER : (int)v;
    }
  }
  return NA_INTEGER;
}
SEXP Rf_allocVector(SEXPTYPE type, R_xlen_t n) {
  if (n < 0) Rf_error("negative length vectors are not allowed");
  return mk((int)type, n);
}
SEXP Rf_allocMatrix(SEXPTYPE type, int nrow, int ncol) {
  SEXP x = mk((int)type, (R_xlen_t)nrow * ncol);
  x->nrow = nrow;
  x->ncol = ncol;
  return x;
}
SEXP Rf_xlengthgets(SEXP x, R_xlen_t n) {
  if (n > x->len) Rf_error("xlengthgets: growing is not mocked");
  x->len = n;
  x->nrow = x->ncol = 0;
  return x;
}
SEXP Rf_protect(SEXP x) {
  ++g_protect;
  return x;
}
void Rf_unprotect(int n) {
  if (n > g_protect) Rf_error("unprotect(): only %d protected items", g_protect);
  g_protect -= n;
}
void Rf_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  if (!g_jmp) {
    fprintf(stderr, "rmock: Rf_error outside rm_call: %s\n", g_err);
    abort();
  }
  longjmp(*g_jmp, 1);
}
void Rf_warning(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
}
char* R_alloc(size_t n, int size) { return (char*)calloc(n ? n : 1, (size_t)size); }

/* R's RNG: GetRNGstate/PutRNGstate bracket the draws; the state lives in g_rng */
static int g_rng_open;
void GetRNGstate(void) { g_rng_open = 1; }
void PutRNGstate(void) { g_rng_open = 0; }
static sg_rrng* rng(void) {
  if (!g_rng_open) Rf_error("rmock: a draw outside GetRNGstate()/PutRNGstate()");
  if (!g_rng && sg_rrng_create(1, &g_rng) != 0) Rf_error("rmock: sg_rrng_create failed");
  return g_rng;
}
double unif_rand(void) { return sg_rrng_unif(rng()); }
double norm_rand(void) { return sg_rrng_norm(rng()); }
double rgamma(double shape, double scale) { return sg_rrng_gamma(rng(), shape, scale); }

/* routine registration */
struct rm_dll {
  const R_CallMethodDef* calls;
};
static struct rm_dll g_dll;
static int g_dynamic = 1;
int R_registerRoutines(DllInfo* info, const void* c, const R_CallMethodDef* call, const void* f, const void* e) {
  (void)c; (void)f; (void)e;
  info->calls = call;
  return 1;
}
Rboolean R_useDynamicSymbols(DllInfo* info, Rboolean value) {
  (void)info;
  g_dynamic = value;
  return TRUE;
}

/* ---- driver API (tests/test_r_shim.py) -------------------------------- */
void R_init_soundgen(DllInfo* dll);
void R_unload_soundgen(DllInfo* dll);

int rm_init(void) {
  R_init_soundgen(&g_dll);
  return g_dynamic;
}
void rm_unload(void) { R_unload_soundgen(&g_dll); }
int rm_n_routines(void) {
  int n = 0;
  while (g_dll.calls && g_dll.calls[n].name) ++n;
  return n;
}
const char* rm_routine(int i, int* nargs) {
  *nargs = g_dll.calls[i].numArgs;
  return g_dll.calls[i].name;
}
void rm_set_seed(int seed) {
  if (!g_rng) sg_rrng_create(seed, &g_rng);
  else sg_rrng_set_seed(g_rng, seed);
}
double rm_unif(void) {  /* the next runif(1) of the stream (tests: stream position) */
  g_rng_open = 1;
  double u = sg_rrng_unif(rng());
  g_rng_open = 0;
  return u;
}
const char* rm_error(void) { return g_err; }
int rm_protect_depth(void) { return g_protect; }

typedef SEXP (*F0)(void);
typedef SEXP (*F1)(SEXP);
typedef SEXP (*F2)(SEXP, SEXP);
typedef SEXP (*F3)(SEXP, SEXP, SEXP);
typedef SEXP (*F4)(SEXP, SEXP, SEXP, SEXP);
typedef SEXP (*F5)(SEXP, SEXP, SEXP, SEXP, SEXP);

/* .Call(name, args...): 0 and *out on success; -1 with rm_error() when the
 * routine called Rf_error (R's longjmp), -2 unknown name, -3 wrong arity */
int rm_call(const char* name, int nargs, SEXP* args, SEXP* out) {
  const R_CallMethodDef* volatile d = NULL;
  for (int i = 0; g_dll.calls && g_dll.calls[i].name; ++i)
    if (!strcmp(g_dll.calls[i].name, name)) d = &g_dll.calls[i];
  if (!d) return -2;
  if (d->numArgs != nargs) return -3;
  jmp_buf jb;
  jmp_buf* volatile prev = g_jmp;
  g_jmp = &jb;
  g_err[0] = 0;
  volatile int depth = g_protect;
  if (setjmp(jb)) {
    g_jmp = prev;
    g_protect = depth;  /* R resets the protect stack on error */
    g_rng_open = 0;
    return -1;
  }
  SEXP r = R_NilValue;
  switch (nargs) {
    case 0: r = ((F0)d->fun)(); break;
    case 1: r = ((F1)d->fun)(args[0]); break;
    case 2: r = ((F2)d->fun)(args[0], args[1]); break;
    case 3: r = ((F3)d->fun)(args[0], args[1], args[2]); break;
    case 4: r = ((F4)d->fun)(args[0], args[1], args[2], args[3]); break;
    case 5: r = ((F5)d->fun)(args[0], args[1], args[2], args[3], args[4]); break;
    default: g_jmp = prev; return -3;
  }
  g_jmp = prev;
  *out = r;
  return 0;
}

SEXP rm_null(void) { return R_NilValue; }
SEXP rm_real(R_xlen_t n, const double* v) {
  SEXP x = mk(REALSXP, n);
  if (n) memcpy(x->data, v, (size_t)n * sizeof(double));
  return x;
}
SEXP rm_int(R_xlen_t n, const int* v) {
  SEXP x = mk(INTSXP, n);
  if (n) memcpy(x->data, v, (size_t)n * sizeof(int));
  return x;
}
SEXP rm_lgl_na(void) {  /* the logical NA of a formal such as amplAnchors = NA */
  SEXP x = mk(LGLSXP, 1);
  ((int*)x->data)[0] = NA_INTEGER;
  return x;
}
SEXP rm_matrix(int nrow, int ncol, const double* v) {  /* column-major, as R stores it */
  SEXP x = Rf_allocMatrix(REALSXP, nrow, ncol);
  memcpy(x->data, v, (size_t)nrow * ncol * sizeof(double));
  return x;
}
static SEXP mkchar(const char* s) {
  SEXP c = (SEXP)calloc(1, sizeof *c);
  c->type = CHARSXP;
  c->len = (R_xlen_t)strlen(s);
  c->data = strdup(s);
  return c;
}
/* list(...) with names (NULL: unnamed) */
SEXP rm_list(int n, SEXP* elts, const char** names) {
  SEXP x = mk(VECSXP, n);
  for (int i = 0; i < n; ++i) ((SEXP*)x->data)[i] = elts[i];
  if (names) {
    SEXP nm = mk(STRSXP, n);
    for (int i = 0; i < n; ++i) ((SEXP*)nm->data)[i] = mkchar(names[i]);
    x->names = nm;
  }
  return x;
}
int rm_type(SEXP x) { return x->type; }
R_xlen_t rm_length(SEXP x) { return x->len; }
double* rm_real_ptr(SEXP x) { return x->type == REALSXP ? (double*)x->data : NULL; }
int rm_nrow(SEXP x) { return x->nrow; }
int rm_ncol(SEXP x) { return x->ncol; }
SEXP rm_elt(SEXP x, R_xlen_t i) { return x->type == VECSXP && i >= 0 && i < x->len ? ((SEXP*)x->data)[i] : NULL; }
