#!/bin/bash
# Per-phase time of the single-block Snappy kernel (decode_one_par_kernel, slate_block_decode):
# the C per-call harness on the profiling library with SLATE_ONE_STOP=k (the kernel ends after
# phase k; 0 = whole).  Differences between successive k price the phases.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r5}/onestop
mkdir -p $OUT /tmp/onestop_lib
cp slatedb-go_amd/lib/libslatecodec_prof.so /tmp/onestop_lib/libslatecodec.so
timeout -k 10 120 python3 tools/percall_bench.py --dump $OUT/pc.bin > $OUT/dump.log 2>&1 || { echo DUMP_FAILED; tail -20 $OUT/dump.log; exit 1; }
for r in 1 2; do
  for k in 0 1 2 3 4 5 6; do
    SLATE_ONE_STOP=$k PERCALL_DECODE_ONLY=1 LD_LIBRARY_PATH=/tmp/onestop_lib timeout -k 10 60 tools/build/percall $OUT/pc.bin 3000 > $OUT/stop$k.log 2>&1 || { echo STOP_FAILED $k; tail $OUT/stop$k.log; exit 1; }
    echo "pass $r stop $k $(cat $OUT/stop$k.log)" | tee -a $OUT/summary.txt
  done
done
