"""Static instruction mix of the lane-per-block decode loop (tooling): compiles
decode_lpb2.hip with SLATE_FORCE_DBG=<mask> (ablation bits folded at compile time) and the
walker's general phases compiled out (SLATE_COUNT_FAST_ONLY: the bench's rows never take them), and reports VALU/SALU/DS/VMEM counts of the main step loop (4 steps)."""
import collections
import os
import re
import subprocess
import sys
import tempfile

SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "slatedb-go_amd", "csrc", "decode_lpb2.hip")


def mix(dbg):
    with tempfile.TemporaryDirectory() as d:
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-S", "--cuda-device-only",
               f"-DSLATE_FORCE_DBG={dbg}", "-DSLATE_COUNT_FAST_ONLY", SRC, "-o", os.path.join(d, "k.s")]
        subprocess.run(cmd, check=True, capture_output=True)
        text = open(os.path.join(d, "k.s")).read()
    start = text.index("_ZN5slate18decode_lpb2_kernelILb0E")
    lines = text[start:].split("\n")
    labels = {m.group(1): i for i, l in enumerate(lines) for m in [re.match(r"^(\.LBB\d+_\d+):", l)] if m}
    best = None
    for i, l in enumerate(lines):
        m = re.search(r"s_(cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            body = [x.strip() for x in lines[labels[m.group(2)]:i] if x.strip() and x.strip()[0] not in ";." and not x.strip().endswith(":")]
            nd = sum(1 for x in body if x.startswith("ds_"))
            nb = sum(1 for x in body if x.startswith("buffer_"))
            npm = sum(1 for x in body if x.startswith("ds_bpermute"))
            if nb >= 8 and nd >= 20 and npm >= 8 and (best is None or len(body) < len(best)):
                best = body
    c = collections.Counter(x.split()[0] for x in best)
    return {k: sum(v for op, v in c.items() if op.startswith(p)) for k, p in
            (("VALU", "v_"), ("SALU", "s_"), ("DS", "ds_"), ("VMEM", "buffer_"))}


if __name__ == "__main__":
    for dbg in [int(x, 0) for x in (sys.argv[1:] or ["0"])]:
        print(dbg, mix(dbg))
