#!/bin/bash
# r3k: LZ4 plan skips literal-only chunks: LZ4 parity, LZ4 kernel split.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_lz4_gpu.py tests/test_sst_codecs_gpu.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -60 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
SLATE_ABLATE_CODEC=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 tools/ablate.py 1000000 0 > $OUT/lz4.log 2>&1 || { echo PROF_FAILED; tail -20 $OUT/lz4.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r3k/prof/**/run_kernel_stats.csv', recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:5]:
    print(r['Name'][:80], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')
PY
