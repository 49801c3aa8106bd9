#!/bin/bash
# r2p: configs[2] encode end to end (host and device input), kernel stats, bit-exact check.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r2p
mkdir -p $OUT
for c in none snappy; do
  timeout -k 10 400 python -u tools/bench_encode.py --codec $c --check > $OUT/encode_$c.json 2> $OUT/encode_$c.err || { echo ENC_FAILED; tail -20 $OUT/encode_$c.err; exit 1; }
  cat $OUT/encode_$c.json
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_$c -o enc -- python3 tools/bench_encode.py --codec $c --steps 2 > $OUT/prof_$c.log 2>&1 || { echo PROF_FAILED; tail -20 $OUT/prof_$c.log; exit 1; }
  find $OUT/prof_$c -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats_encode_$c.csv
done
