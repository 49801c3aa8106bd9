#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2q
mkdir -p $OUT
for c in none snappy; do
SLATE_HOST_TRACE=1 timeout -k 10 300 python -u tools/bench_encode.py --codec $c --steps 1 > $OUT/enc_$c.json 2> $OUT/enc_$c.err || { echo FAILED; tail -20 $OUT/enc_$c.err; exit 1; }
grep "slate build" $OUT/enc_$c.err | tail -8
done
