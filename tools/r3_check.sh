#!/bin/bash
# Round-3 checkpoint: the new Zlib block-parallel inflate and the copy-thread pools (their GPU
# tests).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=${OUT:-gpurun_out/r3c}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_zstd_par_gpu.py tests/test_zlib_par_gpu.py tests/test_shard_gpu.py -m gpu -x -v -s --timeout 120 --timeout-method thread > $OUT/zlib_tests.log 2>&1 || { echo PAR_TESTS_FAILED; tail -60 $OUT/zlib_tests.log; exit 1; }
grep -E "PASS|FAIL|zlib-6|zstd-3|slate z|passed|failed" $OUT/zlib_tests.log | tail -30

