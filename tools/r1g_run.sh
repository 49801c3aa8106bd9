# r1g: compaction chain GPU parity (+ merge suite again) and the compaction bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r1g
mkdir -p $OUT
export TMPDIR=/tmp
true
true
timeout -k 10 400 python -u tools/bench_compact.py > $OUT/bench_compact.json 2> $OUT/bench_compact.err || { echo BENCH_FAILED; tail -20 $OUT/bench_compact.err; exit 1; }
cat $OUT/bench_compact.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace2 -o run -- python3 tools/bench_compact.py --steps 1 > $OUT/trace.log 2>&1 || { echo TRACE_FAILED; tail -20 $OUT/trace.log; exit 1; }
