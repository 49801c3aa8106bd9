#!/bin/bash
# Snappy encode checkpoint: the encode GPU suites, then configs[2] through the builder with the
# host trace (kernel phases) and the full-size bit-exact check, and the kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=${OUT:-gpurun_out/enc}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_encode_gpu.py tests/test_encode_codecs_gpu.py tests/test_sst_codecs_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
SLATE_HOST_TRACE=1 timeout -k 10 300 python -u tools/bench_encode.py --codec snappy --check > $OUT/enc_snappy.json 2> $OUT/enc_snappy.trace || { echo ENC_FAILED; tail -20 $OUT/enc_snappy.trace; exit 1; }
grep "slate build" $OUT/enc_snappy.trace | tail -5
python3 -c "import json;d=json.load(open('$OUT/enc_snappy.json'));print('e2e host',d['host_input']['end_to_end_s'],'device',d['device_input']['end_to_end_s'],'bit_exact',d['bit_exact'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 tools/bench_encode.py --codec snappy --steps 2 > $OUT/trace.log 2>&1 || { echo TRACE_FAILED; tail -20 $OUT/trace.log; exit 1; }
cut -d, -f1-4 $OUT/trace/run_kernel_stats.csv | head -12 | cut -c1-160
# opening a 10 M-KV SST's index and filter as the reference's zlib / zstd writers shape them
timeout -k 10 300 python -u tools/payload_probe.py 10000000 zlib-ref,zstd-ref,zlib,zstd > $OUT/payload_probe.log 2>&1 || { echo PROBE_FAILED; tail -20 $OUT/payload_probe.log; exit 1; }
cat $OUT/payload_probe.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/ptrace -o run -- python3 tools/payload_probe.py 10000000 zlib-ref,zstd-ref > $OUT/ptrace.log 2>&1 || { echo PTRACE_FAILED; tail -20 $OUT/ptrace.log; exit 1; }
cut -d, -f1-4 $OUT/ptrace/run_kernel_stats.csv | head -24 | cut -c1-140
