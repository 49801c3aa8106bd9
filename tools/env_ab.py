"""Same-process A/B of per-call library switches (environment variables the library reads on every
call: SLATE_ZL_NO_STAGE, SLATE_ZF_NO_H, SLATE_ZF_H_SERIAL, SLATE_ZF_CRC_WG) on one of bench.py's
decode workloads, rounds alternating, a step = plan + decode timed with HIP events on the
context's stream.
usage: python tools/env_ab.py WORKLOAD ENVVAR [BLOCKS] [ROUNDS] [STEPS]   (on = unset, off = ENVVAR=1)
       python tools/env_ab.py WORKLOAD MODE1 MODE2 ... --blocks N --rounds R --steps S
         MODE = name:VAR=VAL,VAR=VAL (name: alone = no variables set)
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
    argv = sys.argv[1:]
    opts = {"--blocks": 1_000_000, "--rounds": 3, "--steps": 5}
    for k in list(opts):
        if k in argv:
            i = argv.index(k)
            opts[k] = int(argv[i + 1])
            del argv[i:i + 2]
    wk = argv[0]
    if ":" in argv[1]:
        modes = []
        for spec in argv[1:]:
            name, _, body = spec.partition(":")
            modes.append((name, dict(kv.split("=", 1) for kv in body.split(",") if kv)))
        n, rounds, steps = opts["--blocks"], opts["--rounds"], opts["--steps"]
    else:
        var = argv[1]
        modes = [("on", {}), ("off", {var: "1"})]
        n = int(argv[2]) if len(argv) > 2 else 1_000_000
        rounds = int(argv[3]) if len(argv) > 3 else 3
        steps = int(argv[4]) if len(argv) > 4 else 5
    allvars = sorted({v for _, m in modes for v in m})
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
    res = {name: [] for name, _ in modes}
    dec_bytes = int(dec_off[-1])
    for r in range(rounds):
        for name, env in modes:
            for v in allvars:
                os.environ.pop(v, None)
            os.environ.update(env)
            ctx.handbacks(reset=True)
            kern, wall = leg.timed(torch, stream, steps, 1)
            hb = ctx.handbacks(reset=True)
            meta = leg.d_meta.download().view(sc.META_DTYPE)
            res[name].append(kern)
            verified = leg.verify_against_decoded((dec, dec_off), meta) if r == rounds - 1 else 0
            print(json.dumps({"round": r, "mode": name, "env": env, "step_ms": round(kern, 4), "wall_ms": round(wall, 4),
                              "handbacks": int(hb), "all_ok": bool((meta["status"] == 0).all()),
                              "verified_blocks": verified}), flush=True)
    for v in allvars:
        os.environ.pop(v, None)
    print(json.dumps({"workload": wk, "blocks": n, "median_ms": {k: round(float(np.median(x)), 4) for k, x in res.items()},
                      "median_gib_s": {k: round(dec_bytes / (float(np.median(x)) * 1e-3) / 2**30, 1)
                                       for k, x in res.items()}}), flush=True)
    leg.free()


if __name__ == "__main__":
    main()
