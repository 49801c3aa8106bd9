#!/bin/bash
# Round 2: FETCH_SIZE / WRITE_SIZE calibration against known byte counts (tools/fetch_calib.hip)
set -e
OUT=gpurun_out/r2s
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/fetch -o run -- ./tools/build/fetch_calib > $OUT/fetch.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/write -o run -- ./tools/build/fetch_calib > $OUT/write.log 2>&1
timeout -k 10 60 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- ./tools/build/fetch_calib > $OUT/trace.log 2>&1
python3 tools/fetch_calib.py $OUT > $OUT/fetch_calib.txt
cat $OUT/fetch_calib.txt
