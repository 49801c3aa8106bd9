#!/bin/bash
# r3z: round-2 checkpoint: whole GPU suite, smoke, bench line, kernel trace, traffic.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3z
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
bash tools/traffic.sh $OUT/traffic > $OUT/traffic.log 2>&1 || { echo TRAFFIC_FAILED; tail -20 $OUT/traffic.log; exit 1; }
tail -5 $OUT/traffic.log
cp profiles/pmc_decode_latest.json $OUT/ 2>/dev/null
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
