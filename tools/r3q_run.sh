#!/bin/bash
# r3q: opening a configs[2]-sized SST's index and filter per codec (slate_decode_index, slate_bloom_decode).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3q
mkdir -p $OUT
timeout -k 10 500 python3 -u tools/payload_probe.py 10000000 > $OUT/probe.log 2>&1 || { echo PROBE_FAILED; tail -20 $OUT/probe.log; exit 1; }
grep -v amdgpu.ids $OUT/probe.log
