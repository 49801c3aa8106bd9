#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2l
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_shard_gpu.py tests/test_sst_codecs_gpu.py tests/test_encode_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
SLATE_HOST_TRACE=1 timeout -k 10 300 python -u tools/host_probe.py > $OUT/probe.log 2>&1 || { echo PROBE_FAILED; tail -30 $OUT/probe.log; exit 1; }
cat $OUT/probe.log | grep -v "wait decode" | tail -12
