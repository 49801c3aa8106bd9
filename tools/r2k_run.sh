#!/bin/bash
# r2k: host pipeline overlap: shard/host tests, bench with host_io.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2k
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_shard_gpu.py tests/test_multi.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['host_io'])"
