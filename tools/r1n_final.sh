# r1n: final state of the round -- full GPU suite, smoke, PMC traffic passes (FETCH/WRITE, each
# its own run) refreshing profiles/pmc_decode_latest.json, the headline bench line, and the
# kernel trace of the same bench command.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r1n
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.log; exit 1; }
bash tools/traffic.sh $OUT/traffic > $OUT/traffic.log 2>&1 || { echo TRAFFIC_FAILED; tail -20 $OUT/traffic.log; exit 1; }
cp profiles/pmc_decode_latest.json $OUT/pmc_decode_latest.json
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace_bench -o run -- python3 bench.py --no-host-io --no-cpu-baseline > $OUT/trace_bench.log 2>&1 || { echo TRACE_FAILED; tail -20 $OUT/trace_bench.log; exit 1; }
echo done
