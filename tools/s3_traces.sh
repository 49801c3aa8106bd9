#!/bin/bash
# Kernel traces of the secondary workloads: configs[2] Snappy / None SST builds (tools/bench_encode.py)
# and the configs[4] Zstd decode (bench.py --codec zstd).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${OUT:-gpurun_out/traces}
mkdir -p "$OUT"
export TMPDIR=/tmp
SLATE_HOST_TRACE=1 timeout -k 10 300 python3 tools/bench_encode.py --codec snappy --steps 2 > "$OUT/enc_host.json" 2> "$OUT/enc_host.trace" || { echo ENC_HOST_FAILED; tail -20 "$OUT/enc_host.trace"; exit 1; }
grep "slate build" "$OUT/enc_host.trace" | tail -14
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/enc" -o run -- python3 tools/bench_encode.py --codec snappy --steps 2 > "$OUT/enc.log" 2>&1 || { echo ENC_FAILED; tail -20 "$OUT/enc.log"; exit 1; }
cut -d, -f1-4 "$OUT/enc/run_kernel_stats.csv" | head -16 | cut -c1-160
ZARGS="--codec zstd --no-extras --no-host-io --no-cpu-baseline --steps 5 --verify none"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/zstd" -o run -- python3 bench.py $ZARGS > "$OUT/zstd.log" 2>&1 || { echo ZSTD_FAILED; tail -20 "$OUT/zstd.log"; exit 1; }
cut -d, -f1-4 "$OUT/zstd/run_kernel_stats.csv" | head -16 | cut -c1-160
