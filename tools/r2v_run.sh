#!/bin/bash
# r2v: SQ counters of the CodecZstd fast-path kernels (configs[4], 1 M blocks).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2v
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/zstd_ablate.py gen /tmp/zab.npz 1000000 || { echo GEN_FAILED; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY -f csv -d $OUT/p1 -o run -- python3 tools/zstd_ablate.py run /tmp/zab.npz 0 > $OUT/p1.log 2>&1 || { echo P1_FAILED; tail -5 $OUT/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU -f csv -d $OUT/p2 -o run -- python3 tools/zstd_ablate.py run /tmp/zab.npz 0 > $OUT/p2.log 2>&1 || { echo P2_FAILED; tail -5 $OUT/p2.log; exit 1; }
for k in zs_fast_build zs_fast_huf zs_fast_sum zs_fast_crc zs_fast_parse; do
  echo "== $k"
  mkdir -p $OUT/sum_$k && cp -r $OUT/p1 $OUT/p2 $OUT/sum_$k/ 2>/dev/null
  python3 tools/pmc_summary.py $OUT/sum_$k $k 1000000 | grep -v "^avg"
done
