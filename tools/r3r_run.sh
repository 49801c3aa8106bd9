#!/bin/bash
# r3r: LZ4 SST open (index, filter) with and without the content checksum (profiling variants).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3r
mkdir -p $OUT
for v in prof noxxh; do
SLATE_LIB_VARIANT=libslatecodec_$v.so timeout -k 10 300 python3 -u tools/payload_probe.py 10000000 lz4 > $OUT/$v.log 2>&1 || { echo PROBE_FAILED; tail -20 $OUT/$v.log; exit 1; }
echo $v; grep -v amdgpu.ids $OUT/$v.log
done
