"""Zstd frame shapes against the decode fast path (tooling; DESIGN §4 Zstd):
configs[4]-like blocks compressed by libzstd at several levels and block sizes (tests/zstdgen.py,
checksum and content size on), each frame classified on the host by the fast path's shape rule
(zstd_fast.hip zs_fast_parse: one frame of one compressed block, raw / RLE / Huffman literals,
at most 16 sequences, predefined or RLE sequence tables -- FSE_Compressed or repeat tables go to the
exact path), then decoded on the GPU device-resident (plan + decode, HIP events), every block's
status and bytes checked against the input.  Reports per variant the hand-back rate by reason and
the decode rate.  usage: python tools/zstd_shapes.py [--mb DECODED_MB_PER_VARIANT]   (one JSON line per variant)"""
import collections
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "slatedb-go_amd")]


def shape(f: bytes) -> str:
    """The fast path's shape test on one frame: 'fast' or the first reason it is handed back."""
    if f[:4] != b"\x28\xb5\x2f\xfd":
        return "magic"
    fhd = f[4]
    single = (fhd >> 5) & 1
    p = 5 + (0 if single else 1) + [0, 1, 2, 4][fhd & 3] + [1 if single else 0, 2, 4, 8][fhd >> 6]
    bh = int.from_bytes(f[p:p + 3], "little")
    p += 3
    if not bh & 1:
        return "multi-block frame"
    if (bh >> 1) & 3 != 2:
        return "raw / RLE block"
    b0 = f[p]
    lt, sf = b0 & 3, (b0 >> 2) & 3
    if lt == 3:
        return "treeless literals"
    if lt <= 1:
        hs = 1 if sf in (0, 2) else (2 if sf == 1 else 3)
        nl = (b0 >> 3) if sf in (0, 2) else ((b0 >> 4) + (f[p + 1] << 4) if sf == 1 else
                                              (b0 >> 4) + (f[p + 1] << 4) + (f[p + 2] << 12))
        q = p + hs + (nl if lt == 0 else 1)
    else:  # Huffman: sizes in 3, 4 or 5 header bytes
        hs = 3 if sf <= 1 else (4 if sf == 2 else 5)
        v = int.from_bytes(f[p:p + hs], "little")
        bits = {3: 10, 4: 14, 5: 18}[hs]
        cs = (v >> (4 + bits)) & ((1 << bits) - 1)
        q = p + hs + cs
    c0 = f[q]
    ns = c0 if c0 < 128 else (((c0 - 128) << 8) + f[q + 1] if c0 < 255 else f[q + 1] + (f[q + 2] << 8) + 0x7F00)
    if ns == 0:
        return "fast"
    modes = f[q + (1 if c0 < 128 else 2 if c0 < 255 else 3)]
    m = [(modes >> 6) & 3, (modes >> 4) & 3, (modes >> 2) & 3]
    why = ([">16 sequences"] if ns > 16 else []) + (["FSE_Compressed tables"] if 2 in m else []) + \
          (["repeat tables"] if 3 in m else [])
    return " + ".join(why) if why else "fast"


def main():
    import slatecodec as sc
    from tests import sstgen, zstdgen
    from tools import workload as wl
    sys.path.insert(0, REPO)
    import bench
    mb = int(sys.argv[sys.argv.index("--mb") + 1]) if "--mb" in sys.argv else 80  # decoded MB per variant
    torch.cuda.init()
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = sc.Context(0)
    ctx.set_stream(stream.cuda_stream)
    for bs, level in ((4096, 3), (4096, 9), (4096, 19), (8192, 3), (16384, 3), (16384, 19)):
        n = mb * 2 ** 20 // bs
        dec, doff = wl.mixed_blocks(n, block_size=bs)
        frames = [zstdgen.frame(dec[int(doff[i]):int(doff[i + 1])].tobytes(), level=level) for i in range(n)]
        why = collections.Counter(shape(f) for f in frames)
        blocks = [sstgen.crc(f) for f in frames]
        off = np.zeros(n + 1, np.uint64)
        off[1:] = np.cumsum([len(b) for b in blocks])
        blob = np.frombuffer(b"".join(blocks) + bytes(16), np.uint8)
        leg = bench.DecodeLeg(sc, ctx, sc.ZSTD, blob, off)
        ms, _ = leg.timed(torch, stream, 5, 2)
        meta = np.frombuffer(leg.d_meta.download(), dtype=sc.META_DTYPE)
        oo = leg.d_out_off.download(dtype=np.uint64)
        out = leg.d_out.download(int(oo[n]))
        bad = int((meta["status"] != 0).sum())
        for i in range(0, n, max(1, n // 2000)):  # bytes of 2000 spread blocks against the input
            a, l = int(oo[i]), int(doff[i + 1] - doff[i])
            if out[a:a + l].tobytes() != dec[int(doff[i]):int(doff[i + 1])].tobytes():
                bad += 1
        res = {"block_size": bs, "zstd_level": level, "blocks": n, "fast_shape": why.get("fast", 0),
               "handed_back": {k: v for k, v in why.items() if k != "fast"},
               "hand_back_rate": round(1 - why.get("fast", 0) / n, 4), "decode_ms": round(ms, 3),
               "decoded_GiBps": round(int(doff[n]) / (ms * 1e-3) / 2 ** 30, 1), "bad_blocks": bad}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
