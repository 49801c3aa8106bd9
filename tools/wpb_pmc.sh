#!/bin/bash
# SQ counters of the two-phase Snappy decoder's kernels over a short bench run (two passes).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=${OUT:-gpurun_out/wpb_pmc}
mkdir -p $OUT
export TMPDIR=/tmp
export SLATE_SNAPPY_WPB=1
ARGS="--steps 2 --warmup 1 --no-extras --no-cpu-baseline --no-host-io --verify none --blocks ${BLOCKS:-262144}"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -f csv -d $OUT/pmc1 -o run -- python3 bench.py $ARGS > $OUT/pmc1.log 2>&1 || { echo PMC1_FAILED; tail -5 $OUT/pmc1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU -f csv -d $OUT/pmc2 -o run -- python3 bench.py $ARGS > $OUT/pmc2.log 2>&1 || { echo PMC2_FAILED; tail -5 $OUT/pmc2.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || { echo TRACE_FAILED; exit 1; }
for k in snappy_build snappy_walk decode_lpb2; do python3 tools/pmc_summary.py $OUT $k ${BLOCKS:-262144}; echo; done
