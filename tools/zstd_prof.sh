#!/bin/bash
# Per-kernel times of the Zstd legs (configs4_zstd, kv100_zstd) for each library in LIBS, under the
# rocprofv3 kernel trace (one GPU call).  env: TAG, LIBS
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r5}/zprof
mkdir -p $OUT
export TMPDIR=/tmp
for lib in ${LIBS:-libslatecodec.so}; do
  for L in configs4_zstd:1000000 kv100_zstd:262144; do
    name=${L%%:*}; blocks=${L#*:}
    SLATE_LIB_VARIANT=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/$lib/$name -o z -- python3 tools/leg_probe.py $name --blocks $blocks --extra-steps 3 > $OUT/$lib.$name.log 2>&1 || { echo PROF_FAILED $lib $name; tail -20 $OUT/$lib.$name.log; exit 1; }
    f=$(ls $OUT/$lib/$name/*kernel_stats.csv | head -1)
    echo "== $lib $name"; grep -E "zs_|zl_" $f | cut -d, -f1-4,6,7 | sed 's/(slate::DecodeArgs, slate::ZsFastArgs)//'
  done
done
