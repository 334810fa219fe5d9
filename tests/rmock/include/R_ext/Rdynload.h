/* Test double of R_ext/Rdynload.h (see ../Rinternals.h). */
#ifndef RMOCK_RDYNLOAD_H
#define RMOCK_RDYNLOAD_H
typedef void* (*DL_FUNC)(void);
typedef enum { FALSE = 0, TRUE } Rboolean;
typedef struct {
  const char* name;
  DL_FUNC fun;
  int numArgs;
} R_CallMethodDef;
typedef struct rm_dll DllInfo;
int R_registerRoutines(DllInfo* info, const void* c, const R_CallMethodDef* call, const void* f, const void* e);
Rboolean R_useDynamicSymbols(DllInfo* info, Rboolean value);
#endif
