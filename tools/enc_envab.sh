#!/bin/bash
# encode A/B of one library under two environments (ENV_A / ENV_B, e.g. "SLATE_FILTER_FIRST=0"),
# alternating twice, after the encode GPU suites; then a kernel trace of the A side
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${OUT:-gpurun_out/encenv}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$ENC_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $ENC_TESTS -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || { echo TESTS_FAILED; tail -30 "$OUT/tests.log"; exit 1; }
  tail -1 "$OUT/tests.log"
fi
for r in 1 2; do
  env $ENV_A timeout -k 10 300 python -u tools/enc_ab.py 10000000 snappy >> "$OUT/ab_a.log" 2>&1 || { echo A_FAILED; tail -20 "$OUT/ab_a.log"; exit 1; }
  echo "A($ENV_A) $(tail -1 $OUT/ab_a.log)"
  env $ENV_B timeout -k 10 300 python -u tools/enc_ab.py 10000000 snappy >> "$OUT/ab_b.log" 2>&1 || { echo B_FAILED; tail -20 "$OUT/ab_b.log"; exit 1; }
  echo "B($ENV_B) $(tail -1 $OUT/ab_b.log)"
done
if [ -n "$ENC_TRACE" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$OUT/trace" -o run -- python3 tools/enc_ab.py 10000000 snappy > "$OUT/trace.log" 2>&1 || { echo TRACE_FAILED; exit 1; }
fi
