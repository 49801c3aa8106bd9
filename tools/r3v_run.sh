#!/bin/bash
# r3v: index flatbuffer built during the filter encode: encode + compaction
# parity, configs[2] encode timing (host trace) for None and Snappy.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3v
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_encode_gpu.py tests/test_encode_codecs_gpu.py tests/test_compaction_gpu.py tests/test_sst_codecs_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for c in none snappy; do
SLATE_HOST_TRACE=1 timeout -k 10 300 python -u tools/bench_encode.py --codec $c --steps 3 --check > $OUT/enc_$c.json 2> $OUT/enc_$c.err || { echo ENC_FAILED $c; tail -20 $OUT/enc_$c.err; exit 1; }
grep "slate build\] flush" $OUT/enc_$c.err | tail -2
cut -c1-900 $OUT/enc_$c.json
done
