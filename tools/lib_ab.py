"""Same-box A/B of decode library builds (tooling): one workload generated once, then each
library (slatedb-go_amd/lib/<name>) timed in its own process, interleaved over rounds, and
every block of the first round's output verified against the generator.

usage: python tools/lib_ab.py BLOCKS ROUNDS LIB [LIB ...]   (LIB: file name under lib/)
env: SLATE_AB_CODEC=snappy|none|lz4, SLATE_AB_STEPS (20)"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "slatedb-go_amd")]


def child(wdir, steps, verify):
    import torch

    import bench
    import slatecodec as sc
    from tools import workload as wl
    codec = {"snappy": sc.SNAPPY, "none": sc.NONE, "lz4": sc.LZ4}[os.environ.get("SLATE_AB_CODEC", "snappy")]
    blob, in_off = np.load(os.path.join(wdir, "blob.npy")), np.load(os.path.join(wdir, "in_off.npy"))
    dev = torch.device("cuda", 0)
    ctx = sc.Context(0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    leg = bench.DecodeLeg(sc, ctx, codec, blob, in_off)
    kern_ms, wall_ms = leg.timed(torch, stream, steps, 3)
    meta = leg.d_meta.download().view(sc.META_DTYPE)
    bad_status = int((meta["status"] != 0).sum())
    verified = 0
    if verify and bad_status == 0:
        verified = leg.verify_against_generator(wl, (0, 1, leg.n), "all", meta, 16, True)
    print(json.dumps({"lib": os.environ.get("SLATE_LIB_VARIANT", "libslatecodec.so"), "kernel_ms": round(kern_ms, 4),
                      "wall_ms": round(wall_ms, 4), "bad_status": bad_status, "verified": verified}), flush=True)


def main():
    if sys.argv[1] == "--child":
        child(sys.argv[2], int(sys.argv[3]), sys.argv[4] == "1")
        return
    n, rounds, libs = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3:]
    import slatecodec as sc
    from tools import workload as wl
    codec = {"snappy": sc.SNAPPY, "none": sc.NONE, "lz4": sc.LZ4}[os.environ.get("SLATE_AB_CODEC", "snappy")]
    steps = os.environ.get("SLATE_AB_STEPS", "20")
    wdir = tempfile.mkdtemp(prefix="lib_ab_")
    blob, in_off = wl.block_set(codec, 0, 1, n, threads=16)
    np.save(os.path.join(wdir, "blob.npy"), blob)
    np.save(os.path.join(wdir, "in_off.npy"), in_off)
    res = {lib: [] for lib in libs}
    for r in range(rounds):
        for lib in libs:
            env = dict(os.environ, SLATE_LIB_VARIANT=lib)
            out = subprocess.run([sys.executable, __file__, "--child", wdir, steps, "1" if r == 0 else "0"], env=env,
                                 capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(out.stdout[-2000:], out.stderr[-4000:], file=sys.stderr)
                sys.exit(f"lib_ab: {lib} failed ({out.returncode})")
            line = json.loads(out.stdout.strip().splitlines()[-1])
            print(json.dumps(line), flush=True)
            if line["bad_status"]:
                sys.exit(f"lib_ab: {lib}: {line['bad_status']} blocks with a bad status")
            res[lib].append(line["kernel_ms"])
    print(json.dumps({"blocks": n, "codec": os.environ.get("SLATE_AB_CODEC", "snappy"),
                      "kernel_ms_median": {k: float(np.median(v)) for k, v in res.items()},
                      "kernel_ms_min": {k: float(np.min(v)) for k, v in res.items()}}))


if __name__ == "__main__":
    main()
