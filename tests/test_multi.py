"""world_size-2 coverage of the multi-GPU bench path on CPU (gloo): every rank
decodes its own disjoint shard (no data-path collective) and the whole-job time
is the max over ranks."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from tools import workload as wl


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
        n = 8
        spec = bench.shard_spec(rank, n)
        dec, dec_off = wl.decoded_blocks(n, seed=spec["seed"], half=True, kv_begin=spec["kv_begin"])
        first_key = bytes(dec[int(dec_off[0]) + 4:int(dec_off[0]) + 20])
        last = int(dec_off[n - 1])
        elapsed = 0.25 * (rank + 1)
        job = bench.max_over_ranks(dist, elapsed, "cpu")
        q.put((rank, first_key, int(dec_off[-1]), job, last))
    finally:
        dist.destroy_process_group()


def test_two_rank_shards_and_timing():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, k0, b0, j0, _), (r1, k1, b1, j1, _) = res
    assert j0 == j1 == 0.5  # max over ranks, identical on every rank
    assert k0 != k1  # disjoint key ranges: rank 1 starts at kv 320
    assert k0 == b"k%015d" % 0 and k1 == b"k%015d" % (8 * 40)
    assert b0 > 0 and b1 > 0


def test_shard_spec_disjoint():
    n = 1_000_000
    specs = [bench.shard_spec(r, n) for r in range(8)]
    begins = [s["kv_begin"] for s in specs]
    assert begins == sorted(begins) and np.all(np.diff(begins) >= 38 * n)
    assert len({s["seed"] for s in specs}) == 8
