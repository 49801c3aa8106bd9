#!/bin/bash
# round-5 kernel-time breakdowns (one GPU call): the kv100 Zstd / Zlib legs under the kernel trace,
# and the per-call C harness under the kernel + HIP runtime trace.  env: TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r5prof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/zstd -o z -- python3 tools/leg_probe.py kv100_zstd --blocks 262144 --extra-steps 3 > $OUT/zstd.log 2>&1 || { echo ZSTD_FAILED; tail -20 $OUT/zstd.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/zlib -o z -- python3 tools/leg_probe.py kv100_zlib --blocks 65536 --extra-steps 2 > $OUT/zlib.log 2>&1 || { echo ZLIB_FAILED; tail -20 $OUT/zlib.log; exit 1; }
timeout -k 10 120 python3 tools/percall_bench.py --dump $OUT/pc.bin > $OUT/dump.log 2>&1 || { echo DUMP_FAILED; tail -20 $OUT/dump.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --hip-runtime-trace --stats -f csv -d $OUT/pc -o pc -- tools/build/percall $OUT/pc.bin 1000 > $OUT/pc.log 2>&1 || { echo PC_FAILED; tail -20 $OUT/pc.log; exit 1; }
for d in zstd zlib pc; do f=$(ls $OUT/$d/*kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && head -12 $f | cut -c1-220; done
