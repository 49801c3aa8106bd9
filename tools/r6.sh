#!/bin/bash
# Round-6 GPU runner (one gpurun call per invocation).  env: TAG (output dir under gpurun_out/),
# STEPS (space-separated, run in order, the first failure ends the call):
#   tests       the GPU suite (pytest -m gpu)
#   testsk      a subset: TESTK = pytest -k expression
#   smoke       __graft_entry__.smoke()
#   bench       the default bench line
#   head        the headline leg alone under rocprofv3 --kernel-trace --stats
#   percall     tools/percall_bench.py (per-call decode / seek / reader from C)
#   ab          tools/lib_ab.py AB_BLOCKS (1048576) blocks, AB_ROUNDS (3) rounds over LIBS (file names
#               under slatedb-go_amd/lib/); SLATE_AB_CODEC picks the codec
#   traffic     tools/traffic.sh for CODECS (default "snappy none zstd"), stamped PMC files
#   cmd         an arbitrary command in CMD
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${TAG:-r6}
mkdir -p $OUT
export TMPDIR=/tmp
for s in ${STEPS:-tests}; do
  echo "== $s $(date +%T)"
  case $s in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/tests.log; exit 1; }
    tail -1 $OUT/tests.log ;;
  testsk)
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$TESTK" > $OUT/testsk.log 2>&1 || { echo TESTSK_FAILED; tail -40 $OUT/testsk.log; exit 1; }
    tail -3 $OUT/testsk.log ;;
  smoke)
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.log; exit 1; }
    tail -1 $OUT/smoke.log ;;
  bench)
    timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { echo BENCH_FAILED; tail -30 $OUT/bench.err; exit 1; }
    cat $OUT/bench.json ;;
  head)
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $OUT/headprof -o head -- python3 bench.py --no-cpu-baseline --no-host-io --no-extras --verify none > $OUT/head.json 2> $OUT/head.err || { echo HEAD_PROF_FAILED; tail -30 $OUT/head.err; exit 1; }
    cat $OUT/head.json
    head -6 $OUT/headprof/head_kernel_stats.csv | cut -c1-220 ;;
  percall)
    timeout -k 10 300 python -u tools/percall_bench.py > $OUT/percall.json 2> $OUT/percall.err || { echo PERCALL_FAILED; tail -30 $OUT/percall.err; exit 1; }
    cat $OUT/percall.json ;;
  ab)
    timeout -k 10 900 python -u tools/lib_ab.py ${AB_BLOCKS:-1048576} ${AB_ROUNDS:-3} $LIBS > $OUT/ab_${SLATE_AB_CODEC:-snappy}.log 2>&1 || { echo AB_FAILED; tail -30 $OUT/ab_${SLATE_AB_CODEC:-snappy}.log; exit 1; }
    tail -15 $OUT/ab_${SLATE_AB_CODEC:-snappy}.log ;;
  traffic)
    for c in ${CODECS:-snappy none zstd}; do
      bash tools/traffic.sh $OUT/traffic_$c $c > $OUT/traffic_$c.log 2>&1 || { echo TRAFFIC_FAILED $c; tail -20 $OUT/traffic_$c.log; exit 1; }
      tail -c 600 $OUT/traffic_$c.log; echo
    done
    mkdir -p $OUT/pmc && cp profiles/pmc_decode_*latest.json $OUT/pmc/ ;;
  cmd)
    timeout -k 10 ${CMD_TIMEOUT:-600} bash -c "$CMD" > $OUT/cmd.log 2>&1 || { echo CMD_FAILED; tail -40 $OUT/cmd.log; exit 1; }
    tail -40 $OUT/cmd.log ;;
  *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
