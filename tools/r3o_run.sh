#!/bin/bash
# r3o: the Snappy chunk encoder on random / zero / key-like / bloom-like data.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3o
mkdir -p $OUT
timeout -k 10 200 python3 tools/snap_chunk_probe.py > $OUT/probe.log 2>&1 || { echo PROBE_FAILED; tail -20 $OUT/probe.log; exit 1; }
cat $OUT/probe.log
