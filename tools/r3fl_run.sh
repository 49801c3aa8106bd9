#!/bin/bash
# r3fl: compiler-flag variants of the decode kernel (profiling builds, tools/variant.sh), A/B
# interleaved twice against a profiling build without extra flags, same box.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3fl
mkdir -p $OUT
for pass in 1 2; do
  for v in base mmc trk nosinkvm; do
    SLATE_LIB_VARIANT=libslatecodec_$v.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-io --verify none --allow-variant > $OUT/${v}_$pass.json 2> $OUT/${v}_$pass.err || { echo BENCH_FAILED $v; tail -20 $OUT/${v}_$pass.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${v}_$pass.json')); print('$v', $pass, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
