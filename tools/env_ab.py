"""Same-process A/B of a per-call library switch (an environment variable the library reads on
every call: SLATE_ZL_NO_STAGE, SLATE_ZF_NO_H) on one of bench.py's decode workloads, rounds
alternating, a step = plan + decode timed with HIP events on the context's stream.
usage: python tools/env_ab.py WORKLOAD ENVVAR [BLOCKS] [ROUNDS] [STEPS]
  WORKLOAD: kv100_zlib | kv100_zstd (configs[1]'s V-half blocks) | configs4_zstd (bench --codec zstd)"""
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
    wk, var = sys.argv[1], sys.argv[2]
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 1_000_000
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    steps = int(sys.argv[5]) if len(sys.argv) > 5 else 5
    t0 = time.time()
    if wk == "configs4_zstd":
        codec = sc.ZSTD
        dec, dec_off = wl.mixed_blocks(n, seed=bench.SEED)
    else:
        codec = {"kv100_zlib": sc.ZLIB, "kv100_zstd": sc.ZSTD}[wk]
        dec, dec_off = wl.decoded_blocks(n, seed=bench.SEED, half=True)
    blob, in_off = wl.encode_blocks(codec, dec, dec_off, threads=16)
    print(f"{wk}: {n} blocks, {int(in_off[-1])} B encoded, {time.time() - t0:.1f} s", flush=True)
    ctx = sc.Context(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    leg = bench.DecodeLeg(sc, ctx, codec, blob, in_off, time_plan=True)
    res = {"on": [], "off": []}
    for r in range(rounds):
        for name in ("on", "off"):
            if name == "off":
                os.environ[var] = "1"
            else:
                os.environ.pop(var, None)
            ctx.handbacks(reset=True)
            kern, wall = leg.timed(torch, stream, steps, 1)
            hb = ctx.handbacks(reset=True)
            meta = leg.d_meta.download().view(sc.META_DTYPE)
            res[name].append(kern)
            print(json.dumps({"round": r, var: name == "off", "step_ms": round(kern, 4), "wall_ms": round(wall, 4),
                              "handbacks": int(hb), "all_ok": bool((meta["status"] == 0).all())}), flush=True)
        verified = leg.verify_against_decoded((dec, dec_off), leg.d_meta.download().view(sc.META_DTYPE))
        print(json.dumps({"round": r, "verified_blocks_last_off": verified}), flush=True)
    os.environ.pop(var, None)
    leg.step()
    torch.cuda.synchronize()
    verified = leg.verify_against_decoded((dec, dec_off), leg.d_meta.download().view(sc.META_DTYPE))
    dec_bytes = int(dec_off[-1])
    on, off = float(np.median(res["on"])), float(np.median(res["off"]))
    print(json.dumps({"workload": wk, "blocks": n, "switch": var, "on_ms": round(on, 4), "off_ms": round(off, 4),
                      "on_gib_s": round(dec_bytes / (on * 1e-3) / 2**30, 1), "verified_blocks_on": verified}), flush=True)
    leg.free()


if __name__ == "__main__":
    main()
