#!/bin/bash
# r2t: CodecZstd fast path (zstd_fast.hip): zstd parity tests, configs[4] bench, kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2t
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 400 python -u -m pytest tests/test_zstd_gpu.py tests/test_sst_codecs_gpu.py tests/test_encode_codecs_gpu.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -60 $OUT/tests.log; exit 1; }
tail -14 $OUT/tests.log
fi
timeout -k 10 300 python -u bench.py --codec zstd --steps 10 --warmup 2 --no-host-io --cache /tmp/wlc > $OUT/bench_zstd.json 2> $OUT/bench_zstd.err || { echo BENCH_FAILED; tail -30 $OUT/bench_zstd.err; exit 1; }
cat $OUT/bench_zstd.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 bench.py --codec zstd --steps 5 --warmup 1 --no-host-io --no-cpu-baseline --verify none --cache /tmp/wlc > $OUT/prof.log 2>&1 || { echo PROF_FAILED; tail -20 $OUT/prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r2t/prof/**/run_kernel_stats.csv', recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')
PY
