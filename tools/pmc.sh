#!/bin/bash
# PMC passes over the decode kernel (one counter group per rocprofv3 run, as the
# gfx950 slot limits require), plus a kernel-trace --stats pass.
# usage: tools/pmc.sh OUTDIR [ablate.py args...]   (run on the GPU box)
set -e
OUT=${1:-gpurun_out/pmc}
shift || true
ARGS=${@:-262144 0}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 tools/ablate.py $ARGS > "$OUT/trace.log" 2>&1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT" \
           "WRITE_SIZE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_WAIT_INST_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -f csv -d "$OUT/pmc$i" -o run -- python3 tools/ablate.py $ARGS > "$OUT/pmc$i.log" 2>&1 || echo "pass $i failed"
done
echo pmc done
