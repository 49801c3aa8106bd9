#!/bin/bash
# r2g: seek kernels (a7) and the whole GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2g
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_seek_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/seek_tests.log 2>&1 || { echo SEEK_FAILED; tail -50 $OUT/seek_tests.log; exit 1; }
tail -2 $OUT/seek_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
