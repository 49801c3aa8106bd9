#!/bin/bash
# Phase B' placement and occupancy on BASELINE configs[4] (tooling): the bench's zstd leg with
# SLATE_ZF_HUF_WG (B' workgroups per CU) and SLATE_ZF_SERIAL (B' on the main stream) varied,
# interleaved twice.  env: OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${OUT:-gpurun_out/zstd_ab}
mkdir -p $OUT /tmp/zcache
export TMPDIR=/tmp
for pass in 1 2; do
  for v in "2 side" "3 side" "2 serial" "3 serial"; do
    set -- $v
    if [ "$2" = serial ]; then export SLATE_ZF_SERIAL=1; else unset SLATE_ZF_SERIAL; fi
    SLATE_ZF_HUF_WG=$1 timeout -k 10 300 python -u bench.py --codec zstd --steps 10 --no-cpu-baseline --no-host-io --verify sample --cache /tmp/zcache > $OUT/z_$1_$2_$pass.json 2> $OUT/z_$1_$2_$pass.err || { echo ZSTD_FAILED $v; tail -20 $OUT/z_$1_$2_$pass.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/z_$1_$2_$pass.json')); print('$v pass $pass', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
