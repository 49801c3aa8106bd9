#!/bin/bash
# r3w: lockstep tail per round (finish iteration of each block vs its round's slowest) and what
# grouping similar blocks could recover.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3w
mkdir -p $OUT
SLATE_LIB_VARIANT=libslatecodec_prof.so timeout -k 10 300 python -u tools/finish_probe.py > $OUT/finish.json 2> $OUT/finish.err || { echo PROBE_FAILED; tail -20 $OUT/finish.err; exit 1; }
cat $OUT/finish.json
