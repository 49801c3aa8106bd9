"""Fold tools/traffic_shapes.sh's passes into per-shape HBM bytes of the headline decode (tooling).

The counters count access shapes differently (profiles/r2s/fetch_calib.txt, tools/fetch_calib.py on
gfx950): FETCH_SIZE = 0.5 x the bytes of wide streaming reads (64-byte runs and up), 2.85 x the
bytes of scattered 16-byte reads; WRITE_SIZE = 1.0 x 64-byte-run writes, 2.0 x scattered 16-byte
writes.  Each ablation removes one shape, so its difference to the full run is that shape's
counted bytes; dividing by the shape's factor gives the bytes that crossed to HBM:
  * far-copy hole sources (16-byte loads, one per lane): F(0) - F(32768), / 2.85;
  * input refills and the rest of the reads (64-byte transposed runs): F(32768), / 0.5;
  * row descriptors (16 bytes per lane, blocks' rows scattered over the wave): W(0) - W(16384), / 2.0;
  * decoded output (128-byte flush runs): W(0) - W(1024), / 1.0;
  * the rest of the writes (meta): what is left, counted as written.
Writes profiles/pmc_shapes_latest.json.  usage: python tools/traffic_shapes.py OUTDIR BLOCKS"""
import csv
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "decode_lpb2_kernel"


def per_launch_kib(path, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return max(vals.values()) if vals else None  # the launches are identical; the max skips a partial one


def main():
    out, blocks = sys.argv[1], int(sys.argv[2])
    c = {}
    for mode in (0, 32768, 16384, 1024):
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            c[(mode, ctr)] = per_launch_kib(os.path.join(out, f"m{mode}", ctr, "run_counter_collection.csv"), ctr)
    kib = 1024.0
    F0, W0 = c[(0, "FETCH_SIZE")], c[(0, "WRITE_SIZE")]
    hole_counted = F0 - c[(32768, "FETCH_SIZE")]
    stream_counted = c[(32768, "FETCH_SIZE")]
    rows_counted = W0 - c[(16384, "WRITE_SIZE")]
    out_counted = W0 - c[(1024, "WRITE_SIZE")]
    other_counted = W0 - rows_counted - out_counted
    shapes = {
        "hole_sources": {"counted_bytes": hole_counted * kib, "factor": 2.85, "bytes": hole_counted * kib / 2.85},
        "input_and_other_reads": {"counted_bytes": stream_counted * kib, "factor": 0.5,
                                  "bytes": stream_counted * kib / 0.5},
        "row_descriptors": {"counted_bytes": rows_counted * kib, "factor": 2.0, "bytes": rows_counted * kib / 2.0},
        "decoded_output": {"counted_bytes": out_counted * kib, "factor": 1.0, "bytes": out_counted * kib},
        "other_writes": {"counted_bytes": other_counted * kib, "factor": 1.0, "bytes": other_counted * kib},
    }
    total = sum(s["bytes"] for s in shapes.values())
    for s in shapes.values():
        s["bytes_per_block"] = round(s["bytes"] / blocks, 1)
        s["counted_bytes"] = int(s["counted_bytes"])
        s["bytes"] = int(s["bytes"])
    lib = os.path.join(REPO, "slatedb-go_amd", "lib", "libslatecodec_prof.so")
    res = {"kernel": KERNEL, "blocks": blocks, "lib": os.path.basename(lib),
           "lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest() if os.path.exists(lib) else None,
           "counters_kib": {f"{m}:{k}": v for (m, k), v in c.items()},
           "shapes": shapes, "hbm_bytes_per_launch_by_shape": int(total),
           "flat_x2_estimate": int((2 * F0 + W0) * kib),
           "note": "profiling build (SLATE_PROFILING_BUILD) of the shipped kernel source; the ablations change "
                   "the kernel's results and exist only in that build"}
    json.dump(res, open(os.path.join(REPO, "profiles", "pmc_shapes_latest.json"), "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
