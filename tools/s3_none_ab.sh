#!/bin/bash
# CodecNone kernel A/B (profiling variants, tools/variant.sh): ablations (1 no CRC, 4 no rows, 8 no
# output stores) for default and sc1 store policy, then the PMC traffic + SQ passes of the library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${OUT:-gpurun_out/none_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in ${VARIANTS:-prof sc1}; do
  SLATE_ABLATE_CODEC=0 SLATE_LIB_VARIANT=libslatecodec_$v.so timeout -k 10 300 python -u tools/ablate.py 1000000 ${MODES:-0,1,4,8,13} \
    > "$OUT/ab_$v.json" 2> "$OUT/ab_$v.err" || { echo AB_FAILED $v; tail -20 "$OUT/ab_$v.err"; exit 1; }
  python3 -c "import json,sys;d=json.load(open('$OUT/ab_$v.json'));print('$v',{m:round(x['ms_median'],3) for m,x in d['modes'].items()})"
done
if [ -z "$NO_PMC" ]; then
  bash tools/traffic.sh "$OUT/traffic" none > "$OUT/traffic.log" 2>&1 || { echo TRAFFIC_FAILED; tail -20 "$OUT/traffic.log"; exit 1; }
  tail -1 "$OUT/traffic.log" | cut -c1-1500
  cp profiles/pmc_decode_none_latest.json "$OUT/"
fi
