#!/bin/bash
# A/B of decode_lpb2 variants (profiling builds from tools/variant.sh), interleaved passes on one box.
# usage: tools/r2ab_run.sh OUTTAG "variant1 variant2 ..." [modes for the first variant]
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/$1
mkdir -p $OUT
VARS="$2"
FIRST_MODES=${3:-0}
for pass in 1 2; do
  first=1
  for v in $VARS; do
    modes=0; [ $first = 1 ] && modes=$FIRST_MODES; first=0
    SLATE_LIB_VARIANT=libslatecodec_$v.so timeout -k 10 120 python3 tools/ablate.py 1000000 $modes > $OUT/$v.$pass.json 2> $OUT/$v.$pass.err || { echo ABLATE_FAILED $v; tail -20 $OUT/$v.$pass.err; exit 1; }
    python3 - $OUT/$v.$pass.json $v $pass <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[3], sys.argv[2], {m: round(v["ms_median"], 4) for m, v in d["modes"].items()})
PY
  done
done
