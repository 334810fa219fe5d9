/* Test double of R.h (see Rinternals.h here). */
#ifndef RMOCK_R_H
#define RMOCK_R_H
#include <stdio.h>
#include <stdlib.h>
#include "Rinternals.h"
#include "R_ext/Random.h"
#endif
