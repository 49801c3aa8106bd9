"""Same-process A/B of the staged CodecZlib plan (the plan is phase Z, kept for the decode) against
the unstaged one (SLATE_ZL_NO_STAGE: a sizes-only inflate in the plan, phase Z again in the decode),
on bench.py's kv100_zlib workload (configs[1]'s 1 M x 4 KiB V-half blocks, Go-shaped zlib level 6).
A step = plan + decode, timed with HIP events on the context's stream, rounds alternating.
usage: python tools/zlib_ab.py [BLOCKS] [ROUNDS] [STEPS]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    import slatecodec as sc
    from tools import workload as wl
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    t0 = time.time()
    dec, dec_off = wl.decoded_blocks(n, seed=bench.SEED, half=True)
    blob, in_off = wl.encode_blocks(sc.ZLIB, dec, dec_off, threads=16)
    print(f"workload {n} blocks, {int(in_off[-1])} B encoded, {time.time() - t0:.1f} s", flush=True)
    ctx = sc.Context(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    leg = bench.DecodeLeg(sc, ctx, sc.ZLIB, blob, in_off, time_plan=True)
    res = {"staged": [], "unstaged": []}
    for r in range(rounds):
        for name in ("staged", "unstaged"):
            if name == "unstaged":
                os.environ["SLATE_ZL_NO_STAGE"] = "1"
            else:
                os.environ.pop("SLATE_ZL_NO_STAGE", None)
            ctx.handbacks(reset=True)
            kern, wall = leg.timed(torch, stream, steps, 1)
            hb = ctx.handbacks(reset=True)
            meta = leg.d_meta.download().view(sc.META_DTYPE)
            ok = bool((meta["status"] == 0).all())
            res[name].append(kern)
            print(json.dumps({"round": r, "mode": name, "step_ms": round(kern, 4), "wall_ms": round(wall, 4),
                              "handbacks": int(hb), "all_ok": ok}), flush=True)
    os.environ.pop("SLATE_ZL_NO_STAGE", None)
    verified = leg.verify_against_decoded((dec, dec_off), leg.d_meta.download().view(sc.META_DTYPE))
    dec_bytes = int(dec_off[-1])
    print(json.dumps({"blocks": n, "staged_ms": round(float(np.median(res["staged"])), 4),
                      "unstaged_ms": round(float(np.median(res["unstaged"])), 4),
                      "staged_gib_s": round(dec_bytes / (np.median(res["staged"]) * 1e-3) / 2**30, 1),
                      "verified_blocks": verified}), flush=True)
    leg.free()


if __name__ == "__main__":
    main()
