"""Profiling aid (tooling): configs[2] Snappy / None SST builds from HBM-resident KVs on the library
named by SLATE_LIB_VARIANT, the builder's summed GPU pass time (slate_ctx_gpu_time) and wall per build,
and the SST bytes against the oracle's builder once (bit-exact at full size)."""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "slatedb-go_amd")]
import slatecodec as sc  # noqa: E402
from oracle import binding as ob  # noqa: E402
from tools import bench_encode as be  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    codec = {"snappy": sc.SNAPPY, "none": sc.NONE}[sys.argv[2] if len(sys.argv) > 2 else "snappy"]
    torch.cuda.init()
    ctx = sc.Context(0)
    keys, key_off, vals, val_off = be.kv_arrays(n)
    d = [sc.devbuf_from(ctx, x) for x in (keys, key_off, vals, val_off)]
    gpu, wall, enc = [], [], None
    for k in range(4):
        ctx.set_timing(True)
        ctx.gpu_busy_ms(reset=True)
        t0 = time.perf_counter()
        b = sc.SstBuilder(ctx, 4096, 0, 10, codec)
        assert b.add_batch_device(d[0].ptr, d[1].ptr, d[2].ptr, d[3].ptr, n) == 0
        t = b.build()
        t1 = time.perf_counter()
        if k:
            gpu.append(ctx.gpu_busy_ms(reset=True))
            wall.append((t1 - t0) * 1e3)
        enc = t.encode()
        del t, b
    o = ob.SstBuilder(4096, 0, 10, ob.SNAPPY if codec == sc.SNAPPY else ob.NONE)
    assert o.add_batch(keys, key_off, vals, val_off) == 0
    assert o.build() == 0
    exact = o.encode_table() == enc
    print(json.dumps({"variant": os.environ.get("SLATE_LIB_VARIANT", "libslatecodec.so"), "kv": n,
                      "gpu_busy_ms": round(float(np.median([g[0] for g in gpu])), 2),
                      "gpu_summed_ms": round(float(np.median([g[1] for g in gpu])), 2), "wall_ms": round(float(np.median(wall)), 2),
                      "bit_exact": exact}))
    assert exact


if __name__ == "__main__":
    main()
