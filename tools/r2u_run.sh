#!/bin/bash
# r2u: CodecZstd fast path ablations (profiling variant): per-kernel times per mode.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2u
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/zstd_ablate.py gen /tmp/zab.npz 1000000 || { echo GEN_FAILED; exit 1; }
for m in ${MODES:-0}; do
  SLATE_LIB_VARIANT=libslatecodec_prof.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $OUT/m$m -o run -- python3 tools/zstd_ablate.py run /tmp/zab.npz $m > $OUT/m$m.log 2>&1 || { echo PROF_FAILED $m; tail -5 $OUT/m$m.log; exit 1; }
  python3 - $m <<'PY'
import csv, glob, sys
m = sys.argv[1]
f = glob.glob(f'gpurun_out/r2u/m{m}/**/run_kernel_stats.csv', recursive=True)[0]
rows = {r['Name'].split('(')[0].replace('slate::', '').replace('void ', ''): float(r['AverageNs']) / 1e3 for r in csv.DictReader(open(f))}
keep = ['zs_fast_parse_kernel', 'zs_fast_build_kernel', 'zs_fast_huf_kernel', 'zs_fast_sum_kernel', 'decode_list_kernel<2>']
print(m, {k: round(rows.get(k, 0), 1) for k in keep})
PY
done
