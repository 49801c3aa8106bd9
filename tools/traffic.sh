#!/bin/bash
# HBM traffic of the decode kernels on the bench workload (run on the GPU box):
# separate rocprofv3 --pmc passes for FETCH_SIZE and WRITE_SIZE over a short bench.py
# run, then tools/traffic.py folds them into profiles/pmc_decode_latest.json, which
# bench.py reports as roofline.traffic.  usage: tools/traffic.sh OUTDIR
set -e
OUT=${1:-gpurun_out/traffic}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-host-io --verify none"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/fetch" -o run -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/write" -o run -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1
SLATE_COMMIT=${SLATE_COMMIT:-} python3 tools/traffic.py "$OUT"
