#!/bin/bash
# r2h: every-codec SST open (index / filter payload kernel) and the whole GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2h
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_sst_codecs_gpu.py -x -v --timeout 300 --timeout-method thread --durations=10 > $OUT/codec_tests.log 2>&1 || { echo CODEC_FAILED; tail -60 $OUT/codec_tests.log; exit 1; }
tail -15 $OUT/codec_tests.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
