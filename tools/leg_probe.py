"""Runs one of bench.py's extra legs alone (tooling, for development runs on the GPU box).
usage: python tools/leg_probe.py LEG [--blocks N] [--extra-steps K]   LEG: kv100_zstd | kv100_zlib | configs4_zstd | codec_none"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "slatedb-go_amd")]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("leg")
    p.add_argument("--blocks", type=int, default=1_000_000)
    p.add_argument("--extra-steps", type=int, default=10)
    p.add_argument("--cpu-seconds", type=float, default=4.0)
    a = p.parse_args()
    import torch
    import bench
    import slatecodec as sc
    from tools import workload as wl
    torch.cuda.init()
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = sc.Context(0)
    ctx.set_stream(stream.cuda_stream)
    args = argparse.Namespace(blocks=a.blocks, extra_steps=a.extra_steps, no_cpu_baseline=True,
                              cpu_seconds=a.cpu_seconds)
    if a.leg == "kv100_zstd":
        r = bench.kv100_leg(sc, ctx, stream, wl, args, 16, sc.ZSTD)
    elif a.leg == "kv100_zlib":
        r = bench.kv100_leg(sc, ctx, stream, wl, args, 16, sc.ZLIB)
    elif a.leg == "configs4_zstd":
        r = bench.zstd_leg(sc, ctx, stream, wl, args, 16)
    elif a.leg == "codec_none":
        r = bench.codec_none_leg(sc, ctx, stream, wl, args, 16)
    else:
        sys.exit(f"unknown leg {a.leg}")
    print(json.dumps({a.leg: r}), flush=True)


if __name__ == "__main__":
    main()
