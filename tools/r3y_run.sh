#!/bin/bash
# r3y: XXH32 / XXH64 content checksums taken from registers by v_readlane (no LDS staging):
# the payload tests, then SST open times (this builder's 10 M-KV SSTs, every codec).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3y
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_lz4_par_gpu.py tests/test_sst_codecs_gpu.py tests/test_encode_codecs_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 400 python -u tools/payload_probe.py 10000000 lz4,zstd,zlib > $OUT/open_times.log 2>&1 || { echo PROBE_FAILED; tail -20 $OUT/open_times.log; exit 1; }
cat $OUT/open_times.log
