#!/bin/bash
# r3n: per-call durations of the Snappy chunk encoder (filter vs index) in one configs[2] build.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3n
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/prof -o run -- python3 tools/bench_encode.py --codec snappy --steps 1 > $OUT/enc.log 2>&1 || { echo PROF_FAILED; tail -20 $OUT/enc.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r3n/prof/**/run_kernel_trace.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows:
    n = r['Kernel_Name']
    if 'snappy_chunks' in n or 'bloom_build' in n or 'enc_pack_snappy' in n:
        print(n[:40], r.get('Grid_Size', r.get('Grid_Size_X', '')), round((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6, 3), 'ms')
PY
