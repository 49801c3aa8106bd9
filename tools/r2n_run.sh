#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2n
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -f csv -d $OUT/prof -o host -- python3 tools/host_probe.py > $OUT/prof.log 2>&1 || { echo PROF_FAILED; tail -30 $OUT/prof.log; exit 1; }
ls -R $OUT/prof | head
