#!/bin/bash
# r2f: lpb2 with atomic round dequeue: whole GPU suite, bench line, kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2f
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-io --verify none > $OUT/trace.log 2>&1 || { echo TRACE_FAILED; tail -20 $OUT/trace.log; exit 1; }
head -4 $OUT/trace/run_kernel_stats.csv
