#!/bin/bash
# r2c: first run of the parse/materialize Snappy decoder (decode_lpb3.hip): Snappy parity tests
# first, then the whole GPU suite, the bench line and a kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2c
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_decode_gpu.py tests/test_decode_lpb_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/snappy_tests.log 2>&1 || { echo SNAPPY_TESTS_FAILED; tail -60 $OUT/snappy_tests.log; exit 1; }
tail -2 $OUT/snappy_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-host-io > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-io --verify none > $OUT/trace.log 2>&1 || { echo TRACE_FAILED; tail -20 $OUT/trace.log; exit 1; }
head -12 $OUT/trace/run_kernel_stats.csv
