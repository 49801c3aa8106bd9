"""Debug helper (tooling): LZ4 / Zlib / Zstd SST builds of growing size, reporting the first failure."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "slatedb-go_amd")]
import slatecodec as sc  # noqa: E402
from oracle import binding as ob  # noqa: E402
from tests import blockgen as bg  # noqa: E402

ctx = sc.Context(0)
for codec in (ob.LZ4, ob.ZLIB, ob.ZSTD):
    for n in (3000, 5000, 8000, 12000, 20000, 40000, 60000):
        kvs = bg.kv_synthetic(n)
        b = sc.SstBuilder(ctx, 4096, 0, 10, codec)
        for k, v in kvs:
            assert b.add_value(k, v) == 0
        try:
            t = b.build()
            print(codec, n, "ok", len(t.encode()), flush=True)
        except Exception as e:  # noqa: BLE001
            print(codec, n, "FAIL", e, flush=True)
            break
