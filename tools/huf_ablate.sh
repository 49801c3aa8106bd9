#!/bin/bash
# Phase B' (zs_fast_huf_kernel) split on the configs[4] Zstd leg, profiling build under the kernel
# trace: as built, without the Huffman tree (SLATE_DEBUG_MODE 1<<30: a flat 8-bit table), without
# the literal streams (1<<29), without both; SLATE_ZF_SERIAL=1 puts B' on the main stream alone
# (before B) so its own time is seen.  env: TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r5}/huf
mkdir -p $OUT
export TMPDIR=/tmp
for m in 0 1073741824 536870912 1610612736; do
  SLATE_ZF_SERIAL=1 SLATE_LIB_VARIANT=libslatecodec_prof.so SLATE_DEBUG_MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/m$m -o z -- python3 tools/leg_probe.py configs4_zstd --blocks 1000000 --extra-steps 3 > $OUT/m$m.log 2>&1 || { echo HUF_ABLATE_FAILED $m; tail -20 $OUT/m$m.log; exit 1; }
  f=$(ls $OUT/m$m/*kernel_stats.csv | head -1)
  echo "mode $m"; grep -E "zs_" $f | cut -d, -f1-4,6,7 | sed 's/(slate::DecodeArgs, slate::ZsFastArgs)//'
done
