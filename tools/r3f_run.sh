#!/bin/bash
# r3f: LZ4 content checksum in the decode loop: whole GPU suite, LZ4 kernel split.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -60 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
SLATE_ABLATE_CODEC=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 tools/ablate.py 1000000 0 > $OUT/lz4.log 2>&1 || { echo PROF_FAILED; tail -20 $OUT/lz4.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r3f/prof/**/run_kernel_stats.csv', recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:5]:
    print(r['Name'][:80], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')
PY
