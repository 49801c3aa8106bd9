#!/bin/bash
# r2x: VALU / SALU / LDS instruction counts of phase B under ablations (profiling variant).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2x
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/zstd_ablate.py gen /tmp/zab.npz 1000000 || { echo GEN_FAILED; exit 1; }
for m in 0 $((1<<20)) $((1<<21)) $((1<<22)) $(((1<<20)|(1<<21)|(1<<22))); do
  SLATE_LIB_VARIANT=libslatecodec_prof.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES -f csv -d $OUT/m$m -o run -- python3 tools/zstd_ablate.py run /tmp/zab.npz $m > $OUT/m$m.log 2>&1 || { echo PMC_FAILED $m; tail -5 $OUT/m$m.log; exit 1; }
  mkdir -p $OUT/s$m && mv $OUT/m$m $OUT/s$m/
  echo "== mode $m"; python3 tools/pmc_summary.py $OUT/s$m zs_fast_build 1000000 | grep -v "^avg"
done
