"""Profiling aid (tooling): opening an SST's index and filter (slate_decode_index,
slate_bloom_decode) per codec, for a configs[2]-sized SST (10 M KV: ~11 MB index, 12.5 MB filter),
built by the GPU builder.  Times are wall clock of the C-ABI calls (host buffer in).
"zlib-ref" / "zstd-ref": the CodecNone SST's raw index and filter compressed the way the reference's
writers shape them (zlib level 6 without flush points; libzstd level 3 streaming-style frames without
a content size), the payloads of an SST the Go DB wrote."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "slatedb-go_amd")]
import torch  # noqa: E402,F401  (torch's HIP runtime first)
import slatecodec as sc  # noqa: E402
from tools.bench_encode import kv_arrays  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    codecs = sys.argv[2].split(",") if len(sys.argv) > 2 else ["snappy", "lz4", "zstd", "zlib", "none"]
    torch.cuda.init()
    ctx = sc.Context(0)
    keys, key_off, vals, val_off = kv_arrays(n)
    for name in codecs:
        ref = name.endswith("-ref")
        base = name[:-4] if ref else name
        codec = {"none": sc.NONE, "snappy": sc.SNAPPY, "lz4": sc.LZ4, "zstd": sc.ZSTD, "zlib": sc.ZLIB}[base]
        b = sc.SstBuilder(ctx, 4096, 0, 10, sc.NONE if ref else codec)
        assert b.add_batch(keys, key_off, vals, val_off) == 0
        sst = b.build().encode()
        st, info, _ = sc.read_info(sst)
        assert st == sc.OK, st
        ib = sst[info.index_offset:info.index_offset + info.index_len]
        fb = sst[info.filter_offset:info.filter_offset + info.filter_len]
        if ref:
            import zlib
            from tests import sstgen, zstdgen
            if base == "zlib":
                comp = lambda raw: zlib.compress(raw, 6)  # noqa: E731
            else:
                comp = lambda raw: zstdgen.frame(raw, level=3, content_size=False)  # noqa: E731
            ib, fb = sstgen.crc(comp(ib[:-4])), sstgen.crc(comp(fb[:-4]))
        res = {}
        for what, fn in (("index", lambda: ctx.decode_index(ib, codec)), ("filter", lambda: ctx.bloom_decode(fb, codec))):
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                r = fn()
                ts.append(time.perf_counter() - t0)
                assert r[0] == sc.OK, (what, r[0])
            res[what] = round(min(ts) * 1e3, 2)
        print(f"{name:6s} index {len(ib) / 1e6:.2f} MB {res['index']} ms, filter {len(fb) / 1e6:.2f} MB {res['filter']} ms",
              flush=True)


if __name__ == "__main__":
    main()
