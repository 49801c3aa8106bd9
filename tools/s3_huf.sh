#!/bin/bash
# configs[4] Huffman-literal phase (zs_fast_huf_kernel) ablations, profiling variant: mode 0, no
# tree (1<<30), no streams (1<<29); per-kernel times from rocprofv3 (workload generated first).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${OUT:-gpurun_out/huf}
mkdir -p "$OUT"
export TMPDIR=/tmp
ZARGS="--codec zstd --no-extras --no-host-io --no-cpu-baseline --steps 5 --verify none --cache /tmp/zcache"
timeout -k 10 300 python3 bench.py $ZARGS > "$OUT/gen.log" 2>&1 || { echo GEN_FAILED; tail -20 "$OUT/gen.log"; exit 1; }
for m in ${MODES:-0 1073741824 536870912}; do
  SLATE_DEBUG_MODE=$m SLATE_LIB_VARIANT=libslatecodec_prof.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/m$m" -o run -- python3 bench.py $ZARGS --allow-variant > "$OUT/m$m.log" 2>&1 || { echo RUN_FAILED $m; tail -20 "$OUT/m$m.log"; exit 1; }
  echo "mode $m"; grep -E "zs_fast|decode_list|decode_large" "$OUT/m$m/run_kernel_stats.csv" | cut -d, -f1-4 | cut -c1-120
done
