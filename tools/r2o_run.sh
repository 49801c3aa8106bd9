#!/bin/bash
# r2o: device-resident SST builder: builder / encode / compaction tests, then the whole GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2o
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_builder_device_gpu.py tests/test_encode_gpu.py tests/test_compaction_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -60 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo SUITE_FAILED; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
