#!/bin/bash
# Round-3 CodecNone checkpoint: the GPU suite on the new library, then the CodecNone bench leg on the
# previous library (variant libslatecodec_old.so, wave-per-block decode_fast_kernel<0>) and on the
# new one (decode_none_kernel), same box, and the kernel trace of the new one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${OUT:-gpurun_out/none}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 \
  || { echo TESTS_FAILED; tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
ARGS="--codec none --no-extras --no-host-io --no-cpu-baseline --steps 20"
SLATE_LIB_VARIANT=libslatecodec_old.so timeout -k 10 300 python -u bench.py $ARGS --allow-variant > "$OUT/none_old.json" 2> "$OUT/none_old.err" \
  || { echo OLD_FAILED; tail -20 "$OUT/none_old.err"; exit 1; }
timeout -k 10 300 python -u bench.py $ARGS > "$OUT/none_new.json" 2> "$OUT/none_new.err" || { echo NEW_FAILED; tail -20 "$OUT/none_new.err"; exit 1; }
python3 - "$OUT" <<'EOF'
import json, sys
for k in ("old", "new"):
    d = json.load(open(f"{sys.argv[1]}/none_{k}.json"))
    r = d["roofline"]
    print(k, d["value"], "GiB/s", d["ms_per_step"], "ms/step kernel", r["kernel_ms"], "frac", r["frac"], "verified", d["verified"]["blocks"])
EOF
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 bench.py $ARGS --verify none > "$OUT/trace.log" 2>&1 \
  || { echo TRACE_FAILED; tail -20 "$OUT/trace.log"; exit 1; }
cut -d, -f1-4 "$OUT/trace/run_kernel_stats.csv" | head -8 | cut -c1-150
