"""The bench workload generator (tools/) builds exactly the blocks the reference
builder (restated by the oracle) would cut for the SURVEY 8d synthetic KVs."""
import numpy as np

from oracle import binding as ob
from tests import blockgen as bg


def test_workload_blocks_match_builder():
    from tools import workload as wl
    n = 60
    dec, off = wl.decoded_blocks(n, half=True)
    rng = np.random.default_rng(20250307)
    rv = rng.integers(0, 256, (n * 40 + 64, 42), dtype=np.uint8)
    kvs = [(b"k%015d" % i, (rv[i].tobytes() * 2)) for i in range(n * 40)]
    blocks = bg.sst_blocks(kvs, 4096, ob.NONE)
    for i in range(n):
        meta, buf, rows = ob.block_decode(blocks[i], ob.NONE)
        assert buf == dec[int(off[i]):int(off[i + 1])].tobytes(), i
    rows_per_block = [ob.block_decode(blocks[i], ob.NONE)[0]["n_rows"] for i in range(n)]
    assert set(rows_per_block) <= {37, 38, 39}


def test_workload_snappy_roundtrip():
    from tools import workload as wl
    blob, off, dec_bytes = wl.snappy_vhalf(50, codec=1)
    out, o_off, meta, rows, rb = ob.block_decode_batch(1, blob, off)
    assert (meta["status"] == 0).all()
    ratio = (off[-1]) / dec_bytes
    assert 0.45 < ratio < 0.6, ratio  # Snappy ~0.53 on V-half
