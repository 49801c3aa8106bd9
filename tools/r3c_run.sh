#!/bin/bash
# r3c: kernel split of the CodecLz4 decode (fast path + checksum pass + exact path) and its plan.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3c
mkdir -p $OUT
export TMPDIR=/tmp
SLATE_ABLATE_CODEC=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 tools/ablate.py 1000000 0 > $OUT/lz4.log 2>&1 || { echo PROF_FAILED; tail -20 $OUT/lz4.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r3c/prof/**/run_kernel_stats.csv', recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]:
    print(r['Name'][:80], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')
PY
