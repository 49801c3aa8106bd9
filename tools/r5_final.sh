#!/bin/bash
# Round-5 final checkpoint, in two GPU calls.
#   PART=1: the GPU suite, smoke, the PMC traffic files of the Snappy / CodecNone / Zstd legs
#           (tools/traffic.sh: stamped to this library; copied to $OUT/pmc for profiles/)
#   PART=3: the per-shape traffic attribution of the headline kernel (tools/traffic_shapes.sh)
#   PART=2: the default bench line (reading the PMC files committed from part 1) and the same
#           command under rocprofv3 --kernel-trace --stats
#   PART=4: the headline launches alone (no extra legs) under the kernel trace
# env: TAG, PART
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r5final}
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${PART:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
  for c in snappy none zstd; do
    bash tools/traffic.sh $OUT/traffic_$c $c > $OUT/traffic_$c.log 2>&1 || { echo TRAFFIC_FAILED $c; tail -20 $OUT/traffic_$c.log; exit 1; }
    tail -c 600 $OUT/traffic_$c.log; echo
  done
  mkdir -p $OUT/pmc && cp profiles/pmc_decode_latest.json profiles/pmc_decode_none_latest.json profiles/pmc_decode_zstd_latest.json $OUT/pmc/
elif [ "$PART" = 3 ]; then
  bash tools/traffic_shapes.sh $OUT/shapes > $OUT/shapes.log 2>&1 || { echo SHAPES_FAILED; tail -20 $OUT/shapes.log; exit 1; }
  tail -c 1500 $OUT/shapes.log
elif [ "$PART" = 2 ]; then
  timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -30 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -f csv -d $OUT/benchprof -o bench -- python3 bench.py > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo BENCH_PROF_FAILED; tail -30 $OUT/bench_prof.err; exit 1; }
  f=$(ls $OUT/benchprof/*kernel_stats.csv | head -1)
  head -12 $f | cut -c1-200
fi
if [ "$PART" = 4 ]; then  # the headline launches alone under the kernel trace (the stats file's average is theirs)
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/headprof -o head -- python3 bench.py --no-cpu-baseline --no-host-io --no-extras --verify none > $OUT/head.json 2> $OUT/head.err || { echo HEAD_PROF_FAILED; tail -30 $OUT/head.err; exit 1; }
  cat $OUT/head.json
  head -6 $OUT/headprof/head_kernel_stats.csv | cut -c1-220
fi
