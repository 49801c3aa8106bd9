#!/bin/bash
# r3b: CodecLz4 lane-per-block fast path: LZ4 + Snappy parity tests, LZ4 timing (fast vs exact
# path), Snappy A/B of the templated kernel (prof = new tree, base = before).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3b
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_lz4_gpu.py tests/test_decode_lpb_gpu.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -60 $OUT/tests.log; exit 1; }
tail -4 $OUT/tests.log
SLATE_ABLATE_CODEC=3 SLATE_LIB_VARIANT=libslatecodec_prof.so timeout -k 10 300 python3 tools/ablate.py 1000000 0,16 > $OUT/lz4.json 2> $OUT/lz4.err || { echo LZ4_FAILED; tail -20 $OUT/lz4.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/lz4.json')); print('lz4', {m: (round(v['ms_median'],3), round(v['GiBps'],1)) for m, v in d['modes'].items()})"
bash tools/r2ab_run.sh r3b/ab "base prof" 0
