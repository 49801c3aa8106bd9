#!/bin/bash
# r3zp: kernel trace of the zlib exact-path opens (plan kernel vs payload kernel).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3zp
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 tools/zlib_open_probe.py > $OUT/probe.log 2>&1 || { echo PROF_FAILED; tail -20 $OUT/probe.log; exit 1; }
grep zlib $OUT/probe.log
cut -c1-160 $OUT/trace/run_kernel_stats.csv | head -12
