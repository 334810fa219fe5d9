#!/bin/bash
# Runs CPU tests against the ASan + UBSan builds (tests/sanitize/Makefile):
#   bash tests/sanitize/run.sh [pytest args]     (default: the planner / oracle CPU tests)
# libasan (and libstdc++, so ASan's __cxa_throw interceptor resolves: python is
# not a C++ program) are preloaded into the pytest process only; the product
# and oracle libraries are swapped for the sanitized ones by SG_HIP_LIB /
# SG_ORACLE_LIB. Reports go to tests/sanitize/_build/report.* and fail the run.
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
make -s -C "$ROOT/soundgen_beta_amd/csrc"
make -s -j8 -C "$HERE"
rm -f "$HERE"/_build/report.*
ASAN_LIB=$(gcc -print-file-name=libasan.so)
CXX_LIB=$(gcc -print-file-name=libstdc++.so.6)
[ $# -gt 0 ] || set -- tests/test_planner.py tests/test_amp_build.py tests/test_oracle.py tests/test_loess_cursor.py \
  tests/test_api_helpers.py tests/test_rrng.py tests/test_dist.py tests/test_node.py -m "not gpu"
cd "$ROOT"
rc=0
env LD_PRELOAD="$ASAN_LIB $CXX_LIB" \
  ASAN_OPTIONS=detect_leaks=0:abort_on_error=0:log_path="$HERE/_build/report" \
  UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1:log_path="$HERE/_build/report" \
  SG_HIP_LIB="$HERE/_build/libsoundgen_hip_san.so" SG_ORACLE_LIB="$HERE/_build/libsg_oracle_san.so" \
  python -m pytest -q -p no:cacheprovider -x "$@" || rc=$?
if ls "$HERE"/_build/report.* > /dev/null 2>&1; then
  echo "sanitizer reports:"; head -40 "$HERE"/_build/report.*
  exit 1
fi
exit $rc
