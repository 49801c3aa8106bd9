"""Kernel timeline of a rocprofv3 --kernel-trace CSV (tooling): per kernel launch its start and end
relative to the first kernel of each build window, and the build's critical path -- which kernels
ran alone and which overlapped.  usage: python tools/timeline.py TRACE_CSV [--match NAME_SUBSTR]"""
import csv
import sys


def main():
    path = sys.argv[1]
    rows = list(csv.DictReader(open(path)))
    ev = []
    for r in rows:
        name = r.get("Kernel_Name", "")
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        ev.append((s, e, name.split("(")[0].replace("void ", ""), r.get("Stream_Id", r.get("Queue_Id", ""))))
    ev.sort()
    # builds: windows that start at an enc_kv_kernel
    starts = [i for i, x in enumerate(ev) if "enc_kv_kernel" in x[2]]
    for bi, i0 in enumerate(starts):
        i1 = starts[bi + 1] if bi + 1 < len(starts) else len(ev)
        win = ev[i0:i1]
        t0 = win[0][0]
        end = max(x[1] for x in win)
        print(f"== build {bi}: {(end - t0) / 1e6:.2f} ms from enc_kv_kernel to the last kernel end")
        busy = 0
        cur_s = cur_e = None
        for s, e, n, q in win:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        print(f"   busy (union of kernel intervals) {busy / 1e6:.2f} ms")
        for s, e, n, q in win:
            d = (e - s) / 1e6
            if d > 0.2:
                print(f"   {(s - t0) / 1e6:8.2f} .. {(e - t0) / 1e6:8.2f}  {d:7.2f} ms  q{q}  {n[:60]}")


if __name__ == "__main__":
    main()
