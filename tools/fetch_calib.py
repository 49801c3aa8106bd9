"""Fold tools/fetch_calib.hip's rocprofv3 passes (tooling): for each access shape, the counter's
bytes per launch against the 1 GiB the launch really reads or writes.  Usage:
fetch_calib.py <dir with fetch/ and write/ rocprofv3 outputs> > profiles/.../fetch_calib.txt"""
import csv
import glob
import os
import sys

REAL = 1 << 30


def per_kernel(root, counter):
    out = {}
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0]
            key = (name, r["Dispatch_Id"])
            out[key] = out.get(key, 0.0) + float(r["Counter_Value"])
    by = {}
    for (name, _), v in out.items():
        by.setdefault(name, []).append(v)
    return by


def main():
    root = sys.argv[1]
    for counter, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        for name, vals in sorted(per_kernel(os.path.join(root, sub), counter).items()):
            kib = sorted(vals)[len(vals) // 2]
            print(f"{counter:10s} {name:40s} {kib * 1024 / 2**30:7.3f} GiB counted per launch "
                  f"(median of {len(vals)}), counter / real = {kib * 1024 / REAL:5.3f}")


if __name__ == "__main__":
    main()
