#!/bin/bash
# Kernel trace of the configs[4] Zstd leg (tooling): per-phase average durations.  env: OUT
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${OUT:-gpurun_out/zstd_trace}
mkdir -p $OUT /tmp/zcache
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o z -- python3 bench.py --codec zstd --steps 10 --no-cpu-baseline --no-host-io --verify none --cache /tmp/zcache > $OUT/z.json 2> $OUT/z.err || { echo ZTRACE_FAILED; tail -20 $OUT/z.err; exit 1; }
cat $OUT/z.json | cut -c1-400
f=$(ls $OUT/prof/*kernel_stats.csv | head -1); head -14 $f | cut -c1-180
python3 tools/trace_timeline.py $(ls $OUT/prof/*kernel_trace.csv | head -1) zs_fast_parse zs_fast_sum 2
