"""Summarise tools/pmc.sh output: per-launch counter values for kernels matching a
substring, plus derived per-block figures.  usage: pmc_summary.py DIR [substr] [blocks]"""
import collections
import csv
import os
import sys


def main():
    d = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "lpb"
    blocks = float(sys.argv[3]) if len(sys.argv) > 3 else 262144.0
    tot = collections.defaultdict(float)
    for p in sorted(os.listdir(d)):
        f = os.path.join(d, p, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        agg = collections.defaultdict(float)
        disp = set()
        for r in csv.DictReader(open(f)):
            if sub not in r["Kernel_Name"]:
                continue
            disp.add(r["Dispatch_Id"])
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
        nd = max(1, len(disp))
        for k, v in agg.items():
            tot[k] = v / nd
    for k in sorted(tot):
        print(f"{k:28s} {tot[k]:14.4g}  per block {tot[k] / blocks:10.2f}")
    st = os.path.join(d, "trace", "run_kernel_stats.csv")
    if os.path.exists(st):
        for r in csv.DictReader(open(st)):
            if sub in r["Name"]:
                print(f"avg duration {float(r['AverageNs']) / 1e6:.4f} ms over {r['Calls']} calls: {r['Name'][:60]}")
    if "SQ_WAVE_CYCLES" in tot:
        wc = tot["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in tot:
                print(f"{k} / WAVE_CYCLES = {tot[k] / wc:.3f}")
    if "GRBM_GUI_ACTIVE" in tot and os.path.exists(st):
        pass


if __name__ == "__main__":
    main()
