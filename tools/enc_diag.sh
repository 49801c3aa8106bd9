#!/bin/bash
# Encode diagnosis: configs[2] Snappy build with the filter after the flush, then beside it
# (host trace on: HIP errors are printed with their call site).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=${OUT:-gpurun_out/encd}
mkdir -p $OUT
export TMPDIR=/tmp
SLATE_SIDE_FILTER=0 SLATE_HOST_TRACE=1 timeout -k 10 300 python -u tools/bench_encode.py --codec snappy --steps 2 > $OUT/seq.json 2> $OUT/seq.trace; echo "seq rc=$?"
grep -E "slate build|slate hip" $OUT/seq.trace | tail -8
SLATE_HOST_TRACE=1 timeout -k 10 300 python -u tools/bench_encode.py --codec snappy --steps 2 > $OUT/side.json 2> $OUT/side.trace; echo "side rc=$?"
grep -E "slate build|slate hip|Error" $OUT/side.trace | tail -12
