#!/bin/bash
# r3p2: LZ4 payloads with blocks above 64 KiB / linked blocks through the tag-parallel passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3p2
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_lz4_par_gpu.py tests/test_sst_codecs_gpu.py tests/test_stream_gpu.py tests/test_lz4_gpu.py -x -v -s --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -60 $OUT/tests.log; exit 1; }
grep -E "passed|failed|4 M KV" $OUT/tests.log | tail -5
