#!/bin/bash
# Per-access-shape HBM traffic of the headline decode (run on the GPU box): FETCH_SIZE and
# WRITE_SIZE passes over the bench workload on the profiling build (tools/variant.sh prof ""),
# once as built and once per ablation that removes one access shape (SLATE_DEBUG_MODE bits of
# decode_lpb2.hip: 32768 = no far-copy hole loads, 16384 = no row-descriptor stores, 1024 = no
# output flush stores).  tools/traffic_shapes.py turns the differences into bytes per shape with
# the counters' per-shape factors (profiles/r2s/fetch_calib.txt).
# usage: tools/traffic_shapes.sh OUTDIR [blocks]
set -e
OUT=${1:-gpurun_out/shapes}
BLOCKS=${2:-1000000}
mkdir -p "$OUT"
export TMPDIR=/tmp
export SLATE_LIB_VARIANT=libslatecodec_prof.so
ARGS="--codec snappy --steps 2 --warmup 1 --blocks $BLOCKS --no-cpu-baseline --no-host-io --no-extras --verify none --allow-variant"
for mode in 0 32768 16384 1024; do
  mkdir -p "$OUT/m$mode"
  for c in FETCH_SIZE WRITE_SIZE; do
    SLATE_DEBUG_MODE=$mode timeout -s KILL 240 rocprofv3 --pmc $c -f csv -d "$OUT/m$mode/$c" -o run -- python3 bench.py $ARGS > "$OUT/m$mode/$c.log" 2>&1
  done
done
python3 tools/traffic_shapes.py "$OUT" "$BLOCKS"
