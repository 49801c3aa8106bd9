#!/bin/bash
# r3p3: LZ4 large-block payload times (pierrec-shaped frames), exact path vs the parallel passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3p3
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_lz4_par_gpu.py -x -v -s --durations=0 --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -60 $OUT/tests.log; exit 1; }
grep -E "passed|failed|4 M KV|s call" $OUT/tests.log | tail -12
