#!/bin/bash
# Per-call wait A/B (one GPU call): the C per-call harness with hipStreamSynchronize (default) and
# with SLATE_WAIT=query (busy poll of hipStreamQuery), interleaved three times.  env: TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r5}/wait
mkdir -p $OUT
timeout -k 10 120 python3 tools/percall_bench.py --dump $OUT/pc.bin > $OUT/dump.log 2>&1 || { echo DUMP_FAILED; tail -20 $OUT/dump.log; exit 1; }
for r in 1 2 3; do
  for w in sync query; do
    SLATE_WAIT=$w timeout -k 10 60 tools/build/percall $OUT/pc.bin 3000 > $OUT/$w.$r.json 2>&1 || { echo PERCALL_FAILED $w; tail $OUT/$w.$r.json; exit 1; }
    echo "$w $r $(cat $OUT/$w.$r.json)" | tee -a $OUT/summary.txt
  done
done
