#!/bin/bash
# round-5 GPU check: decode tests on a variant library, then a same-box A/B of decode library
# builds (tools/lib_ab.py).  env: TAG, VTESTS (test files), VLIB (variant for the tests), LIBS, ROUNDS
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r5}
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$VTESTS" ]; then
  SLATE_LIB_VARIANT=${VLIB:-libslatecodec.so} timeout -k 10 600 python -u -m pytest $VTESTS -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
if [ -n "$LIBS" ]; then
  timeout -k 10 900 python -u tools/lib_ab.py ${BLOCKS:-1000000} ${ROUNDS:-3} $LIBS > $OUT/ab.log 2>&1 || { echo AB_FAILED; tail -30 $OUT/ab.log; exit 1; }
  tail -1 $OUT/ab.log
fi
