#!/bin/bash
# r2d: decode_lpb3 iteration: Snappy parity tests, then the P/M probe on the profiling variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2d
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py tests/test_decode_lpb_gpu.py tests/test_shard_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/snappy_tests.log 2>&1 || { echo SNAPPY_TESTS_FAILED; tail -60 $OUT/snappy_tests.log; exit 1; }
tail -2 $OUT/snappy_tests.log
SLATE_LIB_VARIANT=libslatecodec_prof.so timeout -k 10 200 python3 tools/lpb3_probe.py 262144 ${PROBE_MODES:-0,512,0x400000,0x800000,32} 2>&1 | grep -v amdgpu.ids | tee $OUT/probe.txt
