#!/bin/bash
# r3p: golang/snappy encoder with one barrier per match: encode parity, chunk probe, configs[2] Snappy.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3p
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_encode_gpu.py tests/test_encode_codecs_gpu.py tests/test_compaction_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python3 tools/snap_chunk_probe.py > $OUT/probe.log 2>&1 || { echo PROBE_FAILED; tail -20 $OUT/probe.log; exit 1; }
grep -v amdgpu.ids $OUT/probe.log
SLATE_HOST_TRACE=1 timeout -k 10 300 python -u tools/bench_encode.py --codec snappy --steps 3 --check > $OUT/enc_snappy.json 2> $OUT/enc_snappy.err || { echo ENC_FAILED; tail -20 $OUT/enc_snappy.err; exit 1; }
grep "slate build\]" $OUT/enc_snappy.err | tail -4
cut -c1-700 $OUT/enc_snappy.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 tools/bench_encode.py --codec snappy --steps 1 > $OUT/prof.log 2>&1 || { echo PROF_FAILED; tail -20 $OUT/prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r3p/prof/**/run_kernel_stats.csv', recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:5]:
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')
PY
