"""Which configs[1]-shaped Zstd block does the fast path hand back, and is phase B's output wrong
(the frame without checksum then decodes wrong) or phase C's XXH64?  GPU development probe."""
import os
import struct
import sys
import zlib

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "slatedb-go_amd"))
from oracle import binding as ob  # noqa: E402
from tests import blockgen as bg  # noqa: E402
from tests import zstdgen  # noqa: E402
import slatecodec as sc  # noqa: E402


def crc(s):
    return s + struct.pack(">I", zlib.crc32(s))


def run(ctx, blocks, misalign=9):
    blob, off = bg.pack(blocks, misalign)
    ctx.handbacks(reset=True)
    g_out, g_off, g_meta, _, _ = ctx.decode_batch(ob.ZSTD, blob, off)
    hb = ctx.handbacks()
    return hb, g_out, g_off, g_meta


def main():
    ctx = sc.Context(0)
    kvs = bg.kv_synthetic(38 * 3000, seed=7, half=True)
    bodies = [b[:-4] for b in bg.sst_blocks(kvs, 4096, ob.NONE)]
    ck = [crc(zstdgen.frame(d, 3, True, True, 0, 0)) for d in bodies]
    nock = [crc(zstdgen.frame(d, 3, False, True, 0, 0)) for d in bodies]
    for rep in range(3):
        hb, *_ = run(ctx, ck)
        print("full batch checksum frames: handbacks", hb, flush=True)
    hb, g_out, g_off, g_meta = run(ctx, nock)
    bad = [i for i, d in enumerate(bodies) if bytes(g_out[g_off[i]:g_off[i] + len(d)]) != d]
    print("full batch no-checksum frames: handbacks", hb, "wrong outputs", bad[:20], flush=True)
    for misalign in (0, 3):
        hb, *_ = run(ctx, ck, misalign)
        print("misalign", misalign, "handbacks", hb, flush=True)
    step = 250
    for lo in range(0, len(ck), step):
        hb, *_ = run(ctx, ck[lo:lo + step])
        if hb:
            print("chunk", lo, "handbacks", hb, flush=True)
            for i in range(lo, min(lo + step, len(ck))):
                h1, *_ = run(ctx, [ck[i]])
                if h1:
                    print("  single", i, "handbacks", h1, "len", len(bodies[i]), flush=True)
    print("done", flush=True)


if __name__ == "__main__":
    main()
