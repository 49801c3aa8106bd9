#!/bin/bash
# r2e: SQ/TCC counters of decode_lpb3 (P + M, and P alone) on the profiling variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2e
mkdir -p $OUT
export SLATE_LIB_VARIANT=libslatecodec_prof.so
bash tools/pmc.sh $OUT/pm 262144 0 && python3 tools/pmc_summary.py $OUT/pm lpb3 262144 > $OUT/summary_pm.txt 2>&1
bash tools/pmc.sh $OUT/p 262144 0x400000 && python3 tools/pmc_summary.py $OUT/p lpb3 262144 > $OUT/summary_p.txt 2>&1
paste $OUT/summary_pm.txt $OUT/summary_p.txt
