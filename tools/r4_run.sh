#!/bin/bash
# round-4 GPU check: decode tests + same-box A/B of decode library builds (tools/lib_ab.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${R4TAG:-r4}
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$R4TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $R4TESTS -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
timeout -k 10 600 python -u tools/lib_ab.py 1000000 ${R4ROUNDS:-3} $R4LIBS > $OUT/ab.log 2>&1 || { echo AB_FAILED; tail -30 $OUT/ab.log; exit 1; }
tail -1 $OUT/ab.log
if [ -n "$R4NONE" ]; then
  SLATE_AB_CODEC=none timeout -k 10 400 python -u tools/lib_ab.py 1000000 3 $R4NONE > $OUT/ab_none.log 2>&1 || { echo AB_NONE_FAILED; tail -30 $OUT/ab_none.log; exit 1; }
  tail -1 $OUT/ab_none.log
fi
if [ -n "$R4ABLATE" ]; then
  SLATE_LIB_VARIANT=libslatecodec_prof.so timeout -k 10 400 python -u tools/ablate.py 1000000 $R4ABLATE > $OUT/ablate.json 2> $OUT/ablate.err || { echo ABLATE_FAILED; tail -30 $OUT/ablate.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/ablate.json'));print({k:v['ms_median'] for k,v in d['modes'].items()})"
fi
if [ -n "$R4ZSTD" ]; then
  ZA="--codec zstd --no-extras --no-host-io --no-cpu-baseline --steps 10 --verify none --cache /tmp/zc"
  timeout -k 10 300 python -u bench.py $ZA > $OUT/zstd_par.json 2> $OUT/zstd_par.err || { echo ZSTD_FAILED; tail -20 $OUT/zstd_par.err; exit 1; }
  SLATE_ZF_SERIAL=1 timeout -k 10 300 python -u bench.py $ZA > $OUT/zstd_ser.json 2> $OUT/zstd_ser.err || { echo ZSTD_SER_FAILED; tail -20 $OUT/zstd_ser.err; exit 1; }
  timeout -k 10 300 python -u bench.py $ZA > $OUT/zstd_par2.json 2> $OUT/zstd_par2.err || { echo ZSTD_FAILED; tail -20 $OUT/zstd_par2.err; exit 1; }
  for f in zstd_par zstd_ser zstd_par2; do python3 -c "import json;d=json.load(open('$OUT/$f.json'));print('$f',d['roofline']['kernel_ms'],d['roofline']['frac'])"; done
fi
if [ -n "$R4RATIO" ]; then
  timeout -k 10 300 python -u tools/ratio_probe.py > $OUT/ratio.json 2> $OUT/ratio.err || { echo RATIO_FAILED; tail -20 $OUT/ratio.err; exit 1; }
  cat $OUT/ratio.json
fi
if [ -n "$R4PERCALL" ]; then
  timeout -k 10 300 python -u tools/percall_bench.py > $OUT/percall.json 2> $OUT/percall.err || { echo PERCALL_FAILED; tail -20 $OUT/percall.err; exit 1; }
  cat $OUT/percall.json
fi
