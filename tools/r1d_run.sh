set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r1d
timeout -k 10 300 python -u -m pytest tests/test_zstd_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r1d/zstd_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r1d/zstd_tests.log; exit 1; }
tail -2 gpurun_out/r1d/zstd_tests.log
timeout -k 10 400 python -u bench.py --codec zstd --steps 10 --warmup 2 --no-host-io --no-cpu-baseline > gpurun_out/r1d/bench_zstd2.json 2> gpurun_out/r1d/bench_zstd2.err || { echo ZSTD_BENCH_FAILED; tail -20 gpurun_out/r1d/bench_zstd2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r1d/bench_zstd2.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'])"
