"""Debug aid: test_single_block_api_matrix's block sequence through slate_block_decode, metas
compared with the oracle (prints the mismatches)."""
import os
import random
import sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "slatedb-go_amd")]
import slatecodec as sc
from tests import blockgen as bg
from oracle import binding as ob

ctx = sc.Context(0)
if "--warm" in sys.argv:  # test_vhalf_workload's batches first
    for c in (ob.NONE, ob.SNAPPY):
        kvs = bg.kv_synthetic(38 * 2000, half=True, tomb_every=20)
        g = ctx.decode_batch(c, *bg.pack(bg.sst_blocks(kvs, 4096, c)))
        print("warm", c, (g[2]["status"] == 0).all(), flush=True)
for codec in (ob.NONE, ob.SNAPPY):
    rng = random.Random(31 + codec)
    blocks = []
    for bs in (64, 512, 4096, 32768):
        kvs = bg.random_kvs(rng, 300, alphabet=rng.choice([4, 256]))
        blocks += bg.sst_blocks(kvs, bs, codec)[:6]
    blocks += [bg.mutate(rng, b, fix) for b in blocks[:16] for fix in (False, True)]
    blocks += [b"", b"\x00", b"\x00" * 5, bg.recrc(b"\x00\x00"), bg.recrc(b"\x00\x00\x00\x00\x00\x01"),
               bg.recrc(b"\x00"), bg.recrc(b"\x02\x04ab"), bg.recrc(b"\xff" * 11), bg.recrc(b"\x80"),
               bg.recrc(b"\x05\x00a\x01\x01")]
    big = [(b"big%05d" % i, bytes(rng.randrange(3) for _ in range(30000))) for i in range(4)]
    blocks += bg.sst_blocks([(b"one", bytes(rng.randrange(3) for _ in range(70000)))], 4096, codec)
    blocks += bg.sst_blocks(big, 1 << 17, codec)[:1]
    for rep in range(2):
        bad = 0
        for i, blk in enumerate(blocks):
            st, m, data, offs = ctx.block_decode(blk, codec)
            blob, off = bg.pack([blk])
            o = ob.block_decode_batch(codec, blob, off)
            if m.tobytes() != o[2][0].tobytes():
                bad += 1
                print("codec", codec, "rep", rep, "block", i, len(blk), "gpu", m, "oracle", o[2][0], flush=True)
        print("codec", codec, "rep", rep, "blocks", len(blocks), "mismatches", bad, flush=True)
    g = ctx.decode_batch(codec, *bg.pack(blocks[-2:]))
    print("batch of the last two", g[2], flush=True)
