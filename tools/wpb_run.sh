#!/bin/bash
# A/B of the two-phase Snappy decoder (SLATE_SNAPPY_WPB=1) against the streaming decoder:
# the decode GPU tests under the two-phase decoder, both bench lines, and the kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=${OUT:-gpurun_out/wpb1}
mkdir -p $OUT
export TMPDIR=/tmp
SLATE_SNAPPY_WPB=1 timeout -k 10 600 python -u -m pytest tests/test_decode_gpu.py tests/test_decode_lpb_gpu.py tests/test_workload.py tests/test_devbuf_gpu.py tests/test_shard_gpu.py tests/test_stream_gpu.py tests/test_seek_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -50 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
SLATE_SNAPPY_WPB=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline --no-host-io > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('wpb ',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac'])"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline --no-host-io --verify none > $OUT/bench_lpb2.json 2> $OUT/bench_lpb2.err || { echo BENCH2_FAILED; tail -30 $OUT/bench_lpb2.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_lpb2.json'));print('lpb2',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac'])"
SLATE_SNAPPY_WPB=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 bench.py --steps 5 --warmup 2 --no-extras --no-cpu-baseline --no-host-io --verify none > $OUT/trace.log 2>&1 || { echo TRACE_FAILED; tail -20 $OUT/trace.log; exit 1; }
grep -E "snappy|lpb2|plan_sizes" $OUT/trace/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
