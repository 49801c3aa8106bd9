#!/bin/bash
# encode A/B on the box: the encode GPU suites on the current library, then configs[2] Snappy builds
# alternating between the libraries named in ENC_LIBS (tools/enc_ab.py, bit-exact checked each run)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${OUT:-gpurun_out/encab}
mkdir -p "$OUT"
if [ -n "$ENC_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $ENC_TESTS -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || { echo TESTS_FAILED; tail -30 "$OUT/tests.log"; exit 1; }
  tail -1 "$OUT/tests.log"
fi
for r in 1 2; do
  for lib in $ENC_LIBS; do
    SLATE_LIB_VARIANT=$lib timeout -k 10 300 python -u tools/enc_ab.py 10000000 ${ENC_CODEC:-snappy} >> "$OUT/ab.log" 2>&1 || { echo AB_FAILED $lib; tail -20 "$OUT/ab.log"; exit 1; }
    tail -1 "$OUT/ab.log"
  done
done
