#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the decode kernel under ablation modes (GPU box).
# usage: tools/traffic_ablate.sh OUTDIR mode...
set -e
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for m in "$@"; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/f$m" -o run -- python3 tools/ablate.py 262144 $m > "$OUT/f$m.log" 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/w$m" -o run -- python3 tools/ablate.py 262144 $m > "$OUT/w$m.log" 2>&1
done
echo done
