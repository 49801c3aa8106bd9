#!/bin/bash
# r2i: fragment-parallel Snappy stream decode: stream tests, timing probe + kernel stats, GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2i
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_stream_gpu.py tests/test_sst_codecs_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/stream_tests.log 2>&1 || { echo STREAM_FAILED; tail -60 $OUT/stream_tests.log; exit 1; }
tail -2 $OUT/stream_tests.log
timeout -k 10 300 python -u tools/stream_probe.py > $OUT/probe.json 2> $OUT/probe.err || { echo PROBE_FAILED; tail -30 $OUT/probe.err; exit 1; }
cat $OUT/probe.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o probe -- python3 tools/stream_probe.py > $OUT/prof.log 2>&1 || { echo PROF_FAILED; tail -30 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats_probe.csv
cut -d, -f1-8 $OUT/kernel_stats_probe.csv | head -20
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
