"""Profiling aid (tooling): opening an SST's index and filter (slate_decode_index,
slate_bloom_decode) per codec, for a configs[2]-sized SST (10 M KV: ~11 MB index, 12.5 MB filter),
built by the GPU builder.  Times are wall clock of the C-ABI calls (host buffer in)."""
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
        codec = {"none": sc.NONE, "snappy": sc.SNAPPY, "lz4": sc.LZ4, "zstd": sc.ZSTD, "zlib": sc.ZLIB}[name]
        b = sc.SstBuilder(ctx, 4096, 0, 10, codec)
        assert b.add_batch(keys, key_off, vals, val_off) == 0
        sst = b.build().encode()
        st, info, _ = sc.read_info(sst)
        assert st == sc.OK, st
        ib = sst[info.index_offset:info.index_offset + info.index_len]
        fb = sst[info.filter_offset:info.filter_offset + info.filter_len]
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
