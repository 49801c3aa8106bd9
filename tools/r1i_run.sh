# r1i: full GPU suite, smoke, headline bench, compaction bench + its kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r1i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 python -u tools/bench_compact.py > $OUT/bench_compact.json 2> $OUT/bench_compact.err || { echo CBENCH_FAILED; tail -20 $OUT/bench_compact.err; exit 1; }
cat $OUT/bench_compact.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace_compact -o run -- python3 tools/bench_compact.py --steps 1 > $OUT/trace_compact.log 2>&1 || { echo TRACE_FAILED; tail -20 $OUT/trace_compact.log; exit 1; }
echo done
