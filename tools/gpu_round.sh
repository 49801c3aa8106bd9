#!/bin/bash
# One GPU checkpoint on the box (run through gpurun): the GPU test suite, smoke, the PMC traffic
# passes stamped to this library build, the default bench line, and the rocprofv3 kernel trace of
# the bench's headline leg.  Every GPU step has its own time limit; the first failure ends the run.
# usage: OUT=gpurun_out/<tag> bash tools/gpu_round.sh [tests|bench|all]   (default: all)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${OUT:-gpurun_out/round}
MODE=${1:-all}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 \
    || { echo TESTS_FAILED; tail -40 "$OUT/gpu_tests.log"; exit 1; }
  tail -2 "$OUT/gpu_tests.log"
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
    || { echo SMOKE_FAILED; tail -20 "$OUT/smoke.log"; exit 1; }
  tail -2 "$OUT/smoke.log"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  bash tools/traffic.sh "$OUT/traffic" > "$OUT/traffic.log" 2>&1 || { echo TRAFFIC_FAILED; tail -20 "$OUT/traffic.log"; exit 1; }
  tail -1 "$OUT/traffic.log" | cut -c1-400
  cp profiles/pmc_decode_latest.json "$OUT/"
  bash tools/traffic.sh "$OUT/traffic_none" none > "$OUT/traffic_none.log" 2>&1 || { echo TRAFFIC_NONE_FAILED; tail -20 "$OUT/traffic_none.log"; exit 1; }
  tail -1 "$OUT/traffic_none.log" | cut -c1-400
  cp profiles/pmc_decode_none_latest.json "$OUT/"
  bash tools/traffic.sh "$OUT/traffic_zstd" zstd > "$OUT/traffic_zstd.log" 2>&1 || { echo TRAFFIC_ZSTD_FAILED; tail -20 "$OUT/traffic_zstd.log"; exit 1; }
  tail -1 "$OUT/traffic_zstd.log" | cut -c1-400
  cp profiles/pmc_decode_zstd_latest.json "$OUT/"
  timeout -k 10 500 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo BENCH_FAILED; tail -30 "$OUT/bench.err"; exit 1; }
  cat "$OUT/bench.json"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 bench.py --no-extras \
    --no-cpu-baseline --no-host-io --verify none > "$OUT/trace.log" 2>&1 || { echo TRACE_FAILED; tail -20 "$OUT/trace.log"; exit 1; }
  head -4 "$OUT/trace/run_kernel_stats.csv"
fi
