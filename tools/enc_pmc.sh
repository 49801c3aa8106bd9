#!/bin/bash
# SQ instruction / wait counters of the Snappy encode kernels (configs[2] build, one step), two
# --pmc passes of their own, summed per kernel by tools/pmc_summary.py.  usage: OUT=... tools/enc_pmc.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${OUT:-gpurun_out/encpmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--codec snappy --steps 1"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -f csv -d "$OUT/sq1" -o run -- python3 tools/bench_encode.py $ARGS > "$OUT/sq1.log" 2>&1 || { echo SQ1_FAILED; tail -20 "$OUT/sq1.log"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA -f csv -d "$OUT/sq2" -o run -- python3 tools/bench_encode.py $ARGS > "$OUT/sq2.log" 2>&1 || { echo SQ2_FAILED; tail -20 "$OUT/sq2.log"; exit 1; }
python3 - "$OUT" <<'EOF'
import csv, glob, sys, collections, json
out = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.defaultdict(set)
for f in glob.glob(out + "/sq*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if "snappy" not in k and "enc_" not in k:
            continue
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[k].add((f, r["Dispatch_Id"]))
res = {k: {c: v for c, v in sorted(d.items())} for k, d in tot.items()}
print(json.dumps(res, indent=1))
json.dump(res, open(out + "/enc_pmc.json", "w"), indent=1)
EOF
