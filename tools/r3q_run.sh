#!/bin/bash
# r3q: A/B of SLATE_CRC_SPLIT (CodecSnappy CRC in its own kernel on another stream) vs the default.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3q
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-io > $OUT/base_$i.json 2> $OUT/base_$i.err || { echo BENCH_FAILED; tail -20 $OUT/base_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/base_$i.json')); print('base', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['verified'])"
  SLATE_LIB_VARIANT=libslatecodec_crcsplit.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-io --allow-variant > $OUT/split_$i.json 2> $OUT/split_$i.err || { echo BENCH_FAILED; tail -20 $OUT/split_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/split_$i.json')); print('split', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['verified'])"
done
SLATE_LIB_VARIANT=libslatecodec_crcsplit.so timeout -k 10 400 python -u -m pytest tests/test_decode_gpu.py tests/test_decode_lpb_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
