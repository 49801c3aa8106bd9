#!/bin/bash
# round-4 GPU check: decode tests + same-box A/B of decode library builds (tools/lib_ab.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${R4TAG:-r4}
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$R4TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $R4TESTS -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
timeout -k 10 600 python -u tools/lib_ab.py 1000000 ${R4ROUNDS:-3} $R4LIBS > $OUT/ab.log 2>&1 || { echo AB_FAILED; tail -30 $OUT/ab.log; exit 1; }
tail -1 $OUT/ab.log
if [ -n "$R4NONE" ]; then
  SLATE_AB_CODEC=none timeout -k 10 400 python -u tools/lib_ab.py 1000000 3 $R4NONE > $OUT/ab_none.log 2>&1 || { echo AB_NONE_FAILED; tail -30 $OUT/ab_none.log; exit 1; }
  tail -1 $OUT/ab_none.log
fi
if [ -n "$R4ABLATE" ]; then
  SLATE_LIB_VARIANT=libslatecodec_prof.so timeout -k 10 400 python -u tools/ablate.py 1000000 $R4ABLATE > $OUT/ablate.json 2> $OUT/ablate.err || { echo ABLATE_FAILED; tail -30 $OUT/ablate.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/ablate.json'));print({k:v['ms_median'] for k,v in d['modes'].items()})"
fi
