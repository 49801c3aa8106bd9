#!/bin/bash
# round-5 development run (one GPU call): new-feature tests, the extra bench legs alone, then a
# same-box A/B of decode library builds.  env: TESTS, LEGS ("kv100_zstd:262144 kv100_zlib:65536"),
# VLIB + VTESTS (tests on a variant library), LIBS, ROUNDS, TAG, PRE (a probe script run first),
# DESELECT (pytest --deselect options), NLIBS (libraries for a CodecNone A/B), PERCALL=1,
# ENCTRACE=1, VLIB2 + VTESTS2, PROF=1 (tools/r5_prof.sh), COPY=1, RATIO=1, ONESTOP=1 (tools/onestop.sh),
# ABLEGS + ABLIBS (each leg on each library, same box, twice interleaved), FSE=1 (tools/fse_ablate.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r5}
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$PRE" ]; then
  timeout -k 10 300 python -u $PRE > $OUT/pre.log 2>&1 || { echo PRE_FAILED; tail -30 $OUT/pre.log; exit 1; }
  cat $OUT/pre.log
fi
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS $DESELECT -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -60 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
for L in $LEGS; do
  name=${L%%:*}; blocks=${L#*:}
  timeout -k 10 300 python -u tools/leg_probe.py $name --blocks $blocks --extra-steps 5 > $OUT/$name.json 2> $OUT/$name.err || { echo LEG_FAILED $name; tail -30 $OUT/$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$name.json'));[print(k,{x:v[x] for x in ('value','ms_per_step','handbacks') if x in v}, v['roofline']['kernel_ms'], v['roofline']['frac']) for k,v in d.items()]"
done
for r in 1 2; do for L in $ABLEGS; do for lib in $ABLIBS; do
  name=${L%%:*}; blocks=${L#*:}
  SLATE_LIB_VARIANT=$lib timeout -k 10 300 python -u tools/leg_probe.py $name --blocks $blocks --extra-steps 5 > $OUT/ab_${name}_${lib}_$r.json 2> $OUT/ab_${name}_$lib.err || { echo ABLEG_FAILED $name $lib; tail -30 $OUT/ab_${name}_$lib.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/ab_${name}_${lib}_$r.json'));[print('$lib', k,{x:v[x] for x in ('value','ms_per_step','handbacks') if x in v}, v['roofline']['kernel_ms'], v['roofline']['frac']) for k,v in d.items()]"
done; done; done
if [ -n "$FSE" ]; then TAG=${TAG:-r5} tools/fse_ablate.sh || exit 1; fi
if [ -n "$VTESTS" ]; then
  SLATE_LIB_VARIANT=${VLIB:-libslatecodec.so} timeout -k 10 600 python -u -m pytest $VTESTS -x -q --timeout 120 --timeout-method thread > $OUT/vtests.log 2>&1 || { echo VTESTS_FAILED; tail -40 $OUT/vtests.log; exit 1; }
  tail -1 $OUT/vtests.log
fi
if [ -n "$VTESTS2" ]; then
  SLATE_LIB_VARIANT=$VLIB2 timeout -k 10 600 python -u -m pytest $VTESTS2 -x -q --timeout 120 --timeout-method thread > $OUT/vtests2.log 2>&1 || { echo VTESTS2_FAILED; tail -40 $OUT/vtests2.log; exit 1; }
  tail -1 $OUT/vtests2.log
fi
if [ -n "$LIBS" ]; then
  timeout -k 10 900 python -u tools/lib_ab.py ${BLOCKS:-1000000} ${ROUNDS:-3} $LIBS > $OUT/ab.log 2>&1 || { echo AB_FAILED; tail -30 $OUT/ab.log; exit 1; }
  tail -1 $OUT/ab.log
fi
if [ -n "$NLIBS" ]; then  # a second A/B on the CodecNone workload
  SLATE_AB_CODEC=none timeout -k 10 900 python -u tools/lib_ab.py ${BLOCKS:-1000000} ${ROUNDS:-3} $NLIBS > $OUT/ab_none.log 2>&1 || { echo AB_NONE_FAILED; tail -30 $OUT/ab_none.log; exit 1; }
  tail -1 $OUT/ab_none.log
fi
if [ -n "$PERCALL" ]; then  # per-call latency (C harness + Python)
  timeout -k 10 300 python -u tools/percall_bench.py > $OUT/percall.json 2> $OUT/percall.err || { echo PERCALL_FAILED; tail -20 $OUT/percall.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/percall.json'));print({k:v for k,v in d.items() if 'us' in k}, d.get('c_abi'))"
fi
if [ -n "$ENCTRACE" ]; then  # configs[2] host-input split, with the builder's host trace
  for c in none snappy; do
    SLATE_HOST_TRACE=1 timeout -k 10 300 python -u tools/bench_encode.py --codec $c --steps 3 > $OUT/enc_$c.json 2> $OUT/enc_$c.trace || { echo ENC_FAILED; tail -20 $OUT/enc_$c.trace; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/enc_$c.json'));print('$c', d['host_input'], d['device_input'])"
  done
fi

if [ -n "$PROF" ]; then  # kernel traces of the kv100 legs and the per-call harness
  TAG=${TAG:-r5}/prof tools/r5_prof.sh || exit 1
fi
if [ -n "$ONESTOP" ]; then  # per-phase time of the single-block kernel
  TAG=${TAG:-r5} tools/onestop.sh || exit 1
fi
if [ -n "$COPY" ]; then  # the streaming-copy shapes (bench.py measured_copy_gbps)
  timeout -k 10 300 python3 -c "import json,torch,bench;print(json.dumps(bench.measured_copy_gbps(torch.device('cuda',0))))" > $OUT/copy.json 2> $OUT/copy.err || { echo COPY_FAILED; tail -20 $OUT/copy.err; exit 1; }
  cat $OUT/copy.json
fi
if [ -n "$RATIO" ]; then  # the codecs' compression ratio against the libraries
  timeout -k 10 600 python3 tools/codec_ratio.py > $OUT/ratio.json 2> $OUT/ratio.err || { echo RATIO_FAILED; tail -20 $OUT/ratio.err; exit 1; }
  tail -3 $OUT/ratio.json
fi

