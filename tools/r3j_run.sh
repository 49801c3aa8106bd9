#!/bin/bash
# r3j: LZ4 bench line (1 M V-half blocks, liblz4 frames as pierrec's writer defaults) + shard tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3j
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_shard_gpu.py -x -v --timeout 200 --timeout-method thread > $OUT/shard_tests.log 2>&1 || { echo SHARD_TESTS_FAILED; tail -40 $OUT/shard_tests.log; exit 1; }
tail -3 $OUT/shard_tests.log
timeout -k 10 400 python -u bench.py --codec lz4 --no-host-io > $OUT/bench_lz4.json 2> $OUT/bench_lz4.err || { echo BENCH_LZ4_FAILED; tail -20 $OUT/bench_lz4.err; exit 1; }
cat $OUT/bench_lz4.json
