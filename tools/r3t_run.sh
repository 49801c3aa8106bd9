#!/bin/bash
# r3t: LZ4 and Zstd payloads split by block: SST codec suite, LZ4 suite, open times.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3t
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_sst_codecs_gpu.py tests/test_lz4_gpu.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -60 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 500 python3 -u tools/payload_probe.py 10000000 lz4,zstd,zlib,snappy > $OUT/probe.log 2>&1 || { echo PROBE_FAILED; tail -20 $OUT/probe.log; exit 1; }
grep -v amdgpu.ids $OUT/probe.log
