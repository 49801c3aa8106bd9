#!/bin/bash
# The headline bench line five times on one box (run-to-run spread of value / kernel ms / frac).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r5var
for i in 1 2 3 4 5; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-io --no-extras --verify none > gpurun_out/r5var/head_$i.json 2> gpurun_out/r5var/head_$i.err || { echo FAIL $i; tail -20 gpurun_out/r5var/head_$i.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r5var/head_$i.json').read().strip().splitlines()[-1]);print($i, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
