"""world_size-2 coverage of the multi-GPU path on CPU (gloo): BASELINE configs[1]/[3] shard ONE
block set round-robin (block i on rank i mod N) with no data-path collective.  Each
rank builds its shard with the per-block generator, checks it against the C-ABI partitioner
(slate_shard_pack) applied to the whole set, decodes it (with the oracle: this CPU test has no
GPU; the -m gpu tests decode shards on the HIP path) and verifies it block by block against the
generator; rank 0 checks that the union of the shards is the whole set, in order.  The whole-job
time is the max over ranks."""
import hashlib
import os
import socket

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from tools import workload as wl

SET_BLOCKS = 203  # not a multiple of the world size: the shards differ in length


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import slatecodec as sc
        from oracle import binding as ob
        m = sc.shard_blocks(SET_BLOCKS, world, rank)
        blob, off = wl.block_set(sc.SNAPPY, rank, world, m, threads=2)
        # the partitioner over the whole set gives the same shard
        full, full_off = wl.block_set(sc.SNAPPY, 0, 1, SET_BLOCKS, threads=2)
        pb, po = sc.shard_pack(full, full_off, world, rank)
        assert np.array_equal(po, off) and pb.tobytes() == blob[:int(off[-1])].tobytes()
        out, oo, meta, rows, rb = ob.block_decode_batch(sc.SNAPPY, blob[:int(off[-1])], off)
        assert (meta["status"] == 0).all()
        assert wl.verify_set(rank, world, m, out, oo, rows.view(np.uint8), rb, meta.view(np.uint8), threads=2) == 0
        digests = [hashlib.sha1(out[int(oo[k]):int(oo[k]) + int(meta["data_len"][k]) + 2 * int(meta["n_rows"][k]) + 2]
                                .tobytes()).hexdigest() for k in range(m)]
        shards = [None] * world
        dist.all_gather_object(shards, (rank, digests))
        job = bench.max_over_ranks(dist, 0.25 * (rank + 1), "cpu")
        q.put((rank, shards, job))
    finally:
        dist.destroy_process_group()


def test_two_rank_round_robin_shards():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=180) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[2] for r in res] == [0.5, 0.5]  # max over ranks, identical on every rank
    shards = dict(res[0][1])
    # the union of the shards, re-interleaved, is the whole set decoded in order
    from oracle import binding as ob
    import slatecodec as sc
    full, full_off = wl.block_set(sc.SNAPPY, 0, 1, SET_BLOCKS, threads=2)
    out, oo, meta, _, _ = ob.block_decode_batch(sc.SNAPPY, full[:int(full_off[-1])], full_off)
    for i in range(SET_BLOCKS):
        d = hashlib.sha1(out[int(oo[i]):int(oo[i]) + int(meta["data_len"][i]) + 2 * int(meta["n_rows"][i]) + 2]
                         .tobytes()).hexdigest()
        assert shards[i % world][i // world] == d, i
    assert sum(len(v) for v in shards.values()) == SET_BLOCKS


def test_shard_partition_is_round_robin():
    import slatecodec as sc
    for n, g in ((0, 3), (1, 8), (17, 4), (32_505_856, 8), (32_505_856, 3)):
        counts = [sc.shard_blocks(n, g, s) for s in range(g)]
        assert sum(counts) == n and max(counts) - min(counts) <= 1
    assert sc.shard_blocks(10, 4, 4) == 0  # shard out of range
