#!/bin/bash
# r3h: CodecZstd Huffman-literal phase (zs_fast_huf_kernel) on configs[4]: kernel times with the
# tree (1<<30) or the streams (1<<29) switched off (profiling variant; timing only).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/zstd_ablate.py gen /tmp/zab.npz 1000000 || { echo GEN_FAILED; exit 1; }
for m in 0 $((1<<29)) $((1<<30)) $(((1<<29)|(1<<30))); do
  SLATE_LIB_VARIANT=libslatecodec_prof.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $OUT/m$m -o run -- python3 tools/zstd_ablate.py run /tmp/zab.npz $m > $OUT/m$m.log 2>&1 || { echo RUN_FAILED $m; tail -5 $OUT/m$m.log; exit 1; }
  python3 - $m <<'PY'
import csv, glob, sys
f = glob.glob(f'gpurun_out/r3h/m{sys.argv[1]}/**/run_kernel_stats.csv', recursive=True)[0]
print(sys.argv[1], {r['Name'].split('(')[0].replace('slate::',''): round(float(r['AverageNs'])/1e3) for r in list(csv.DictReader(open(f)))[:6]})
PY
done
