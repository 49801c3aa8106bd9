#!/bin/bash
# Phase A' (zs_fse_parse_kernel) split on the kv100 Zstd leg: the profiling library in full
# (mode 0) and with the sequence loop cut (mode 1<<18: the tables only, every block then handed
# to the exact path, so the leg stays correct); the kernel traces give A' per launch.  env: TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r5}/fse
mkdir -p $OUT
export TMPDIR=/tmp
for m in 0 262144; do
  SLATE_LIB_VARIANT=libslatecodec_prof.so SLATE_DEBUG_MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/m$m -o z -- python3 tools/leg_probe.py kv100_zstd --blocks 262144 --extra-steps 3 > $OUT/m$m.log 2>&1 || { echo FSE_ABLATE_FAILED $m; tail -20 $OUT/m$m.log; exit 1; }
  f=$(ls $OUT/m$m/*kernel_stats.csv | head -1)
  echo "mode $m"; grep -E "zs_|zl_" $f | cut -d, -f1-4
done
