#!/bin/bash
# Snappy encoder A/B: the encode GPU tests on the library as built, then configs[2] Snappy builds
# (tools/enc_ab.py, bit-exact at 10 M KV) under a kernel trace for each variant in $VARIANTS.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${OUT:-gpurun_out/snapdpp}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_encode_gpu.py tests/test_encode_codecs_gpu.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 \
  || { echo TESTS_FAILED; tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
for v in ${VARIANTS:-base dpp cum}; do
  SLATE_LIB_VARIANT=libslatecodec_$v.so timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/$v" -o run -- python3 tools/enc_ab.py 10000000 snappy > "$OUT/$v.log" 2>&1 \
    || { echo RUN_FAILED $v; tail -20 "$OUT/$v.log"; exit 1; }
  tail -1 "$OUT/$v.log"
  grep -E "snappy_chunks|enc_pack_snappy" "$OUT/$v/run_kernel_stats.csv" | cut -d, -f1-4 | cut -c1-140
done
