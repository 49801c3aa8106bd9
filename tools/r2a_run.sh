#!/bin/bash
# r2a: baseline SQ/TCC counters of the round-1 decode_lpb2_kernel (262 k blocks), for the redesign.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2a
mkdir -p $OUT
bash tools/pmc.sh $OUT/pmc 262144 0 && python3 tools/pmc_summary.py $OUT/pmc lpb2 262144 > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
