# r1f: merge GPU parity, merge bench + kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r1f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_merge_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/merge_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/merge_tests.log; exit 1; }
tail -2 $OUT/merge_tests.log
timeout -k 10 300 python -u tools/bench_merge.py > $OUT/bench_merge.json 2> $OUT/bench_merge.err || { echo BENCH_FAILED; tail -20 $OUT/bench_merge.err; exit 1; }
cat $OUT/bench_merge.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace_merge -o run -- python3 tools/bench_merge.py --steps 10 > $OUT/trace_merge.log 2>&1 || { echo TRACE_FAILED; tail -20 $OUT/trace_merge.log; exit 1; }
find $OUT/trace_merge -name "*kernel_stats.csv" | head -1 | xargs cat
