#!/bin/bash
# Runs one GPU test file under several -k selections in turn (bisecting an order-dependent
# failure); stops at the first timeout / crash.  usage: tools/kselect.sh FILE "expr1" "expr2" ...
cd "${GRAFT_REPO_ROOT:-.}"
f=$1; shift
for k in "$@"; do
  timeout -k 10 200 python -u -m pytest "$f" -x -q --timeout 120 --timeout-method thread -k "$k" > /tmp/ks.log 2>&1
  rc=$?
  echo "== -k '$k' rc=$rc: $(tail -1 /tmp/ks.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 /tmp/ks.log; exit $rc; fi
done
