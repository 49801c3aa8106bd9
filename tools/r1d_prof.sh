# r1d profiles: kernel trace of the Zstd configs[4] bench (the workload is generated
# outside the profiler: see bench.py --cache) and the Zstd bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r1d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python3 -u bench.py --codec zstd --steps 10 --warmup 2 --no-host-io --cpu-seconds 6 --cache /tmp/wlc > $OUT/bench_zstd.json 2> $OUT/bench_zstd.err || { echo ZB_FAILED; tail -5 $OUT/bench_zstd.err; exit 1; }
cat $OUT/bench_zstd.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace_zstd -o run -- python3 $R/bench.py --codec zstd --steps 10 --warmup 2 --no-host-io --no-cpu-baseline --cache /tmp/wlc > $OUT/trace_zstd.log 2>&1 || { echo TRACE2_FAILED; tail -20 $OUT/trace_zstd.log; exit 1; }
echo done
