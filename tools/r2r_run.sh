#!/bin/bash
# r2r: LZ4 / Zlib / Zstd encode, then the whole GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2r
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_encode_codecs_gpu.py -x -v --timeout 300 --timeout-method thread --durations=8 > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -70 $OUT/tests.log; exit 1; }
tail -14 $OUT/tests.log
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo SUITE_FAILED; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
