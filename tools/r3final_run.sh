#!/bin/bash
# r3final: round-2 final state: whole GPU suite, smoke, PMC traffic (stamped to this build), the
# default bench line, and the kernel trace of the same bench command (default steps).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=${OUT:-gpurun_out/r3final}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
bash tools/traffic.sh $OUT/traffic > $OUT/traffic.log 2>&1 || { echo TRAFFIC_FAILED; tail -20 $OUT/traffic.log; exit 1; }
tail -1 $OUT/traffic.log
cp profiles/pmc_decode_latest.json $OUT/
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline --no-host-io --verify none > $OUT/trace.log 2>&1 || { echo TRACE_FAILED; tail -20 $OUT/trace.log; exit 1; }
grep '^{' $OUT/trace.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('trace bench kernel_ms', d['roofline']['kernel_ms'])"
head -3 $OUT/trace/run_kernel_stats.csv
