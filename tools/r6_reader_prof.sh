#!/bin/bash
# The C per-call harness (tools/build/percall: slate_block_decode, slate_block_seek, the read-ahead
# reader) under rocprofv3's kernel and HIP API traces (tooling).  env: OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${OUT:-gpurun_out/reader_prof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/percall_bench.py --dump $OUT/percall_in.bin > $OUT/dump.log 2>&1 || { echo DUMP_FAILED; tail -20 $OUT/dump.log; exit 1; }
timeout -k 10 120 ./tools/build/percall $OUT/percall_in.bin 2000 > $OUT/percall_plain.json || { echo PLAIN_FAILED; exit 1; }
cat $OUT/percall_plain.json
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats -f csv -d $OUT/prof -o pc -- ./tools/build/percall $OUT/percall_in.bin 2000 > $OUT/percall_prof.json 2> $OUT/prof.err || { echo PROF_FAILED; tail -20 $OUT/prof.err; exit 1; }
cat $OUT/percall_prof.json
f=$(ls $OUT/prof/*kernel_stats.csv | head -1); head -12 $f | cut -c1-200
f=$(ls $OUT/prof/*hip_api_stats.csv | head -1); head -14 $f | cut -c1-200
rm -f $OUT/percall_in.bin
