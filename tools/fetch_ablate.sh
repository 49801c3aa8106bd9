#!/bin/bash
# HBM bytes of decode_lpb2_kernel with parts switched off (profiling variant, tools/ablate.py modes):
# separate --pmc FETCH_SIZE and WRITE_SIZE passes per mode; prints per-launch GB (FETCH x2, gfx950).
# usage: OUT=... tools/fetch_ablate.sh "0 1024 16384 65536"
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${OUT:-gpurun_out/fetchab}
mkdir -p "$OUT"
export TMPDIR=/tmp
for m in $1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    SLATE_LIB_VARIANT=libslatecodec_prof.so timeout -s KILL 200 rocprofv3 --pmc $c -f csv -d "$OUT/m${m}_$c" -o run -- python3 tools/ablate.py 1000000 $m > "$OUT/m${m}_$c.log" 2>&1 || { echo FAILED $m $c; exit 1; }
  done
done
python3 - "$OUT" $1 <<'PY'
import csv, glob, sys
out = sys.argv[1]
for m in sys.argv[2:]:
    res = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = []
        for f in glob.glob(f"{out}/m{m}_{c}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "decode_lpb2_kernel" in r["Kernel_Name"]:
                    vals.append(float(r["Counter_Value"]))
        res[c] = (sum(vals) / len(vals) if vals else 0.0, len(vals))
    f, w = res["FETCH_SIZE"][0] * 1024 * 2 / 1e9, res["WRITE_SIZE"][0] * 1024 / 1e9
    print(f"mode {m}: fetch {f:.2f} GB (x2), write {w:.2f} GB per launch ({res['FETCH_SIZE'][1]} launches)")
PY
