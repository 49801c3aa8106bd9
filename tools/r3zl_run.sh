#!/bin/bash
# r3zl: Huffman table values hoisted into registers (zsym): GPU suite, then zlib exact-path opens,
# old vs new library on the same box.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r3zl
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
SLATE_LIB_VARIANT=libslatecodec_old.so timeout -k 10 300 python -u tools/zlib_open_probe.py > $OUT/old.log 2>&1 || { echo OLD_FAILED; tail -20 $OUT/old.log; exit 1; }
timeout -k 10 300 python -u tools/zlib_open_probe.py > $OUT/new.log 2>&1 || { echo NEW_FAILED; tail -20 $OUT/new.log; exit 1; }
echo old; grep zlib $OUT/old.log; echo new; grep zlib $OUT/new.log
