#!/bin/bash
# r2z: ablation sweep of decode_lpb2_kernel on 1 M V-half blocks (profiling variant; timing only).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2z
mkdir -p $OUT
SLATE_LIB_VARIANT=libslatecodec_prof.so timeout -k 10 300 python3 tools/ablate.py 1000000 0,64,128,65536,8192,32768,1024,16384,192,512 > $OUT/ablate.json 2> $OUT/ablate.err || { echo ABLATE_FAILED; tail -20 $OUT/ablate.err; exit 1; }
cat $OUT/ablate.json
