#!/bin/bash
# Timing + HBM traffic passes for the decode kernel (run on the GPU box).
# usage: tools/pmc_quick.sh OUTDIR [ablate.py args...]
set -e
OUT=${1:-gpurun_out/pmcq}
shift || true
ARGS=${@:-262144 0}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 python3 -u tools/ablate.py $ARGS > "$OUT/ablate.json" 2>"$OUT/ablate.err"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -f csv -d "$OUT/fetch" -o run -- python3 tools/ablate.py 262144 0 > "$OUT/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -f csv -d "$OUT/write" -o run -- python3 tools/ablate.py 262144 0 > "$OUT/write.log" 2>&1
echo done
