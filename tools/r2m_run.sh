#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2m
mkdir -p $OUT
timeout -k 10 120 python -u tools/dma_probe.py > $OUT/dma.log 2>&1 || { echo FAILED; tail -20 $OUT/dma.log; exit 1; }
cat $OUT/dma.log | grep -v amdgpu.ids
HSA_ENABLE_SDMA=0 timeout -k 10 120 python -u tools/dma_probe.py > $OUT/dma_nosdma.log 2>&1 || { echo FAILED2; tail -20 $OUT/dma_nosdma.log; exit 1; }
echo "--- HSA_ENABLE_SDMA=0"; cat $OUT/dma_nosdma.log | grep -v amdgpu.ids
