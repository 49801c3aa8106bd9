"""Timing probe (tooling) for large single-stream Snappy payloads: a compaction-sized bloom
filter and SST index decoded through slate_bloom_decode / slate_decode_index, checked against
the oracle, wall time per call (PCIe copies and CRC included); run under rocprofv3 --stats for
the kernel split (sp_* fragment-parallel kernels vs snappy_stream_kernel)."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "slatedb-go_amd")]

import slatecodec as sc  # noqa: E402
from oracle import binding as ob  # noqa: E402


def timeit(f, reps=10):
    f()
    t = time.perf_counter()
    for _ in range(reps):
        r = f()
    return (time.perf_counter() - t) / reps * 1e3, r


def main():
    ctx = sc.Context(0)
    res = {}
    keys = [b"k%015d" % i for i in range(2_000_000)]
    npr, bits = ob.bloom_build(keys, 10)
    filt = ob.bloom_encode(npr, bits, ob.SNAPPY)
    ms, g = timeit(lambda: ctx.bloom_decode(filt, ob.SNAPPY))
    o = ob.bloom_decode(filt, ob.SNAPPY)
    assert g[0] == 0 and g[1:] == o[1:]
    res["filter"] = {"keys": len(keys), "encoded_bytes": len(filt), "decoded_bytes": len(bits) + 2, "ms_per_call": ms}
    # an index of 60 k blocks with 40-byte first keys (~3 MB decoded)
    metas = [(i * 4096, b"key-%036d" % (i * 37)) for i in range(60_000)]
    idx = ob.encode_index(metas, ob.SNAPPY)
    ms, (st, index) = timeit(lambda: ctx.decode_index(idx, ob.SNAPPY))
    assert st == 0 and index.block_metas() == metas
    res["index"] = {"blocks": len(metas), "encoded_bytes": len(idx), "ms_per_call": ms}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
