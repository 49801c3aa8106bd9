#!/bin/bash
# r2b: full GPU suite (sharded/pipeline tests added), smoke, default bench (configs1, per-block
# set, every block verified), configs[3] slice on one GPU, HBM traffic passes stamped with the build.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2b
mkdir -p $OUT
echo "nproc=$(nproc) affinity=$(python3 -c 'import os;print(len(os.sched_getaffinity(0)))') cpu.max=$(cat /sys/fs/cgroup/cpu.max 2>/dev/null)" > $OUT/host.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 600 python -u bench.py --workload configs3 --steps 5 --warmup 1 --no-cpu-baseline --no-host-io > $OUT/bench_configs3.json 2> $OUT/bench_configs3.err || { echo C3_FAILED; tail -20 $OUT/bench_configs3.err; exit 1; }
cat $OUT/bench_configs3.json
bash tools/traffic.sh $OUT/traffic > $OUT/traffic.log 2>&1 || { echo TRAFFIC_FAILED; tail -20 $OUT/traffic.log; exit 1; }
cp profiles/pmc_decode_latest.json $OUT/
tail -1 $OUT/traffic.log
