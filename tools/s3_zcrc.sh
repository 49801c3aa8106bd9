#!/bin/bash
# Zstd fast path phase A2: the zstd GPU tests on the new library, then the configs[4] kernel trace
# with the wave-per-block CRC kernel (mode 0) and the lane-per-block one (1<<19), profiling variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${OUT:-gpurun_out/zcrc}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_zstd_gpu.py tests/test_zstd_par_gpu.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 \
  || { echo TESTS_FAILED; tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
ZARGS="--codec zstd --no-extras --no-host-io --no-cpu-baseline --steps 10 --cache /tmp/zcache"
timeout -k 10 300 python3 bench.py $ZARGS > "$OUT/new.json" 2> "$OUT/new.err" || { echo GEN_FAILED; tail -20 "$OUT/new.err"; exit 1; }
cat "$OUT/new.json"
for m in 0 524288; do
  SLATE_DEBUG_MODE=$m SLATE_LIB_VARIANT=libslatecodec_prof.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/m$m" -o run -- python3 bench.py $ZARGS --verify none --allow-variant > "$OUT/m$m.log" 2>&1 || { echo RUN_FAILED $m; tail -20 "$OUT/m$m.log"; exit 1; }
  echo "mode $m"; grep -E "zs_|decode_list|decode_large" "$OUT/m$m/run_kernel_stats.csv" | cut -d, -f1-4 | cut -c1-120
done
