"""One step's kernel timeline from a rocprofv3 kernel trace (tooling): the launches from the
last occurrence of a start kernel through the next end kernel, with start / end in µs from the
step's first start, duration and queue.
usage: python tools/trace_timeline.py KERNEL_TRACE.csv START_SUBSTR END_SUBSTR [STEP_FROM_END=1]"""
import csv
import sys


def main():
    path, first, last = sys.argv[1], sys.argv[2], sys.argv[3]
    back = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    rows = list(csv.DictReader(open(path)))
    name_k = next(k for k in rows[0] if k.lower() in ("kernel_name", "name"))
    s_k = next(k for k in rows[0] if "start" in k.lower())
    e_k = next(k for k in rows[0] if "end" in k.lower())
    q_k = next((k for k in rows[0] if "queue" in k.lower() or "stream" in k.lower()), None)
    rows.sort(key=lambda r: int(r[s_k]))
    starts = [i for i, r in enumerate(rows) if first in r[name_k]]
    i0 = starts[-back]
    t0 = int(rows[i0][s_k])
    for r in rows[i0:]:
        nm = r[name_k].split("(")[0].replace("slate::", "").replace("(anonymous namespace)::", "")
        s, e = (int(r[s_k]) - t0) / 1e3, (int(r[e_k]) - t0) / 1e3
        print(f"{s:9.1f} {e:9.1f} {e - s:8.1f}  q={r[q_k] if q_k else '?'}  {nm}")
        if last in r[name_k]:
            break


if __name__ == "__main__":
    main()
