#!/bin/bash
# HBM traffic of the decode kernels on the bench workload (run on the GPU box):
# separate rocprofv3 --pmc passes for FETCH_SIZE, WRITE_SIZE and two SQ groups over a short bench.py
# run, then tools/traffic.py folds them into profiles/pmc_decode_latest.json, which
# bench.py reports as roofline.traffic.  usage: tools/traffic.sh OUTDIR [snappy|none|zstd]
# (none: the CodecNone leg's decode_none_kernel -> profiles/pmc_decode_none_latest.json; zstd: the configs[4]
# decode's kernels summed -> profiles/pmc_decode_zstd_latest.json)
set -e
OUT=${1:-gpurun_out/traffic}
CODEC=${2:-snappy}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--codec $CODEC --steps 2 --warmup 1 --no-cpu-baseline --no-host-io --no-extras --verify none"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/fetch" -o run -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/write" -o run -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1
# the SQ instruction / stall counters of the same command, two passes (8 SQ slots each)
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -f csv -d "$OUT/sq1" -o run -- python3 bench.py $ARGS > "$OUT/sq1.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS -f csv -d "$OUT/sq2" -o run -- python3 bench.py $ARGS > "$OUT/sq2.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1
SLATE_COMMIT=${SLATE_COMMIT:-} python3 tools/traffic.py "$OUT" "$CODEC"
