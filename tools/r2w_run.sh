#!/bin/bash
# r2w: the whole GPU suite + smoke on the current tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r2w
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo SUITE_FAILED; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
