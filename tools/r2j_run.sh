#!/bin/bash
# r2j: kernel stats of the large-stream probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2j
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o probe -- python3 tools/stream_probe.py > $OUT/prof.log 2>&1 || { echo PROF_FAILED; tail -30 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats_probe.csv
cut -d, -f1-8 $OUT/kernel_stats_probe.csv | head -24
