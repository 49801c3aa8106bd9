"""Per-call latency of the unchanged per-block reader path (tooling; bench.py reports the same
figures under "per_call" and "configs0"):
  * sstable.Iterator.nextBlockIter reads and decodes ONE block per call
    (internal/sstable/iterator.go:92-118); the point-read seek does the same (slatedb/db.go:240).
    A cgo shim that keeps that code routes it to slate_block_decode (one 4 KiB block, host in /
    host out) and block.NewIteratorAtKey to slate_block_seek.  Measured: us per call, against the
    oracle's one-thread us per block (the CPU restatement of block.Decode / NewIteratorAtKey);
  * the read-ahead alternative (INTEGRATION.md "Read-ahead iterator"): slate_block_decode_batch
    over 64 blocks per call, us per block;
  * BASELINE configs[0]: one SST of 64 x 4 KiB CodecNone blocks (100 B KV) encoded and decoded,
    us per SST, by the oracle on one thread and by the library.
usage: python tools/percall_bench.py [--calls N] [--dump PATH: write the C harness's input and stop]"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "slatedb-go_amd")]


def _us(fn, calls):
    fn()
    t = time.perf_counter()
    for _ in range(calls):
        fn()
    return (time.perf_counter() - t) * 1e6 / calls


def per_call(ctx, sc, ob, wl, calls=400):
    blob, in_off = wl.block_set(sc.SNAPPY, 0, 1, 256, threads=4)
    blocks = [blob[int(in_off[i]):int(in_off[i + 1])].tobytes() for i in range(256)]
    res = {"blocks": "configs[1] V-half Snappy 4 KiB blocks (100 B KV), one per call"}
    k = [0]

    def gpu_decode():
        st, m, data, offs = ctx.block_decode(blocks[k[0] & 255], sc.SNAPPY)
        assert st == 0
        k[0] += 1

    def cpu_decode():
        m, data, rows = ob.block_decode(blocks[k[0] & 255], ob.SNAPPY)
        assert m["status"] == 0
        k[0] += 1

    res["slate_block_decode_us"] = round(_us(gpu_decode, calls), 1)
    res["oracle_block_decode_us_1thread"] = round(_us(cpu_decode, calls), 1)
    # seek: one (block, key) query per call over one decoded block, a key in the middle of the block
    out, out_off, meta, rows, row_base = ctx.decode_batch(sc.SNAPPY, blob, in_off)
    st, m0, data0, offs0 = ctx.block_decode(blocks[0], sc.SNAPPY)
    o = offs0[len(offs0) // 2]
    sl = (data0[o + 2] << 8) | data0[o + 3]
    pl = (data0[o] << 8) | data0[o + 1]
    fk_sl = (data0[offs0[0] + 2] << 8) | data0[offs0[0] + 3]
    fk = data0[offs0[0] + 4:offs0[0] + 4 + fk_sl]
    key = bytes(fk[:pl]) + bytes(data0[o + 4:o + 4 + sl])
    one_off = np.array([0, out_off[1]], np.uint64)
    one_out = out[: int(out_off[1])]

    def gpu_seek():
        r = ctx.block_seek(one_out, one_off, meta[:1], [0], [key])
        assert r["status"][0] == 0

    def cpu_seek():
        ob.block_seek(data0, offs0, key)

    if "--dump" in sys.argv:  # the C harness's input only (for a rocprofv3 run of tools/build/percall)
        write_harness_input(sys.argv[sys.argv.index("--dump") + 1], blocks, key, reader_sst(ctx, sc))
        return {"dumped": sys.argv[sys.argv.index("--dump") + 1]}
    res["slate_block_seek_us"] = round(_us(gpu_seek, calls), 1)
    res["oracle_block_seek_us_1thread"] = round(_us(cpu_seek, calls), 1)
    # read-ahead: 64 blocks per call
    sub_off = (in_off[:65] - in_off[0]).astype(np.uint64)
    sub = blob[: int(in_off[64])]

    def gpu_batch64():
        ctx.decode_batch(sc.SNAPPY, sub, sub_off)

    res["slate_block_decode_batch64_us_per_block"] = round(_us(gpu_batch64, max(calls // 8, 10)) / 64, 2)
    res["python_binding_overhead_note"] = ("the *_us figures above are per Python call (ctypes, numpy "
                                           "allocations) for both sides; c_abi has the same calls from C")
    res["c_abi"] = c_harness(blocks, key, calls, reader_sst(ctx, sc))
    return res


def write_harness_input(path, blocks, key, sst=None, read_ahead=64):
    """tools/build/percall's input: the blocks, then the seek key, then (optional) one SST for the
    read-ahead reader."""
    import struct
    with open(path, "wb") as f:
        f.write(struct.pack("<I", len(blocks)))
        for b in blocks:
            f.write(struct.pack("<I", len(b)) + b)
        f.write(struct.pack("<I", len(key)) + bytes(key))
        if sst is not None:
            f.write(struct.pack("<Q", len(sst)) + bytes(sst) + struct.pack("<I", read_ahead))


def reader_sst(ctx, sc, n_blocks=2048):
    """A Snappy SST of configs[1]-shaped blocks (k%015d keys, 84 B V-half values, 38 rows per 4 KiB
    block) for the reader leg, built by the library's SstBuilder."""
    rng = np.random.default_rng(20250307)
    b = sc.SstBuilder(ctx, 4096, 0, 10, sc.SNAPPY)
    for i in range(38 * n_blocks):
        r = rng.integers(0, 256, 42, dtype=np.uint8).tobytes()
        assert b.add_value(b"k%015d" % i, r + r) == 0
    return b.build().encode()


def c_harness(blocks, key, calls, sst=None):
    """The same blocks and key through tools/build/percall (C, as a cgo shim calls the library),
    slate_block_decode / slate_block_seek against the oracle's or_block_decode / or_block_seek, and
    the read-ahead reader over every block of `sst` against the oracle's block.Decode per block."""
    import subprocess
    import tempfile
    exe = os.path.join(REPO, "tools", "build", "percall")
    if not os.path.exists(exe):
        return {"skipped": "tools/build/percall not built (make -C tools)"}
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        path = f.name
    write_harness_input(path, blocks, key, sst)
    try:
        r = subprocess.run([exe, path, str(max(calls, 200) * 5)], capture_output=True, text=True, timeout=120)
    finally:
        os.unlink(path)
    if r.returncode != 0:
        return {"failed": r.returncode, "stderr": r.stderr[-400:]}
    return json.loads(r.stdout)


def configs0(ctx, sc, ob, calls=20):
    """BASELINE configs[0]: one SST of 64 x 4 KiB CodecNone blocks, 100 B KV (keys k%015d, 84 B
    V-half values): build it (Builder.Add + Build) and read every block back (ReadInfo, ReadIndex,
    ReadBlocks), us per SST."""
    rng = np.random.default_rng(20250307)
    kvs = []
    i = 0
    while True:  # enough keys for 64 full blocks (38 rows each) and no more
        r = rng.integers(0, 256, 42, dtype=np.uint8).tobytes()
        kvs.append((b"k%015d" % i, r + r))
        i += 1
        if i >= 64 * 38:
            break

    def cpu():
        b = ob.SstBuilder(4096, 0, 10, ob.NONE)
        for kk, v in kvs:
            b.add(kk, v)
        b.build()
        sst = b.encode_table()
        st, info = ob.sst_read_info(sst)
        st, metas = ob.decode_index(sst[info["index_offset"]:info["index_offset"] + info["index_len"]], info["codec"])
        offs = [o for o, _ in metas] + [info["filter_offset"]]
        for a, bb in zip(offs, offs[1:]):
            ob.block_decode(sst[a:bb], ob.NONE)
        return sst, len(offs) - 1

    def gpu():
        b = sc.SstBuilder(ctx, 4096, 0, 10, sc.NONE)
        for kk, v in kvs:
            b.add(kk, v)
        sst = b.build().encode()
        st, info, _ = sc.read_info(sst)
        st, index = ctx.decode_index(sst[info.index_offset:info.index_offset + info.index_len], info.codec)
        nb = len(index.block_offsets())
        st2, failed, outs = ctx.read_blocks(info, index, 0, nb, sst)
        assert st2 == 0
        return sst, nb

    sst_c, nb_c = cpu()
    sst_g, nb_g = gpu()
    assert sst_c == sst_g, "configs[0] SST bytes differ between the oracle and the library"
    return {"sst_bytes": len(sst_c), "blocks": nb_c, "kv": len(kvs), "bit_exact": True,
            "oracle_us_per_sst_1thread": round(_us(cpu, calls), 1), "slate_us_per_sst": round(_us(gpu, calls), 1),
            "what": "encode (Builder.Add x KV + Build) + decode (ReadInfo, ReadIndex, ReadBlocks of every block)"}


def main():
    import slatecodec as sc
    from oracle import binding as ob
    from tools import workload as wl
    calls = int(sys.argv[sys.argv.index("--calls") + 1]) if "--calls" in sys.argv else 400
    ctx = sc.Context(0)
    pc = per_call(ctx, sc, ob, wl, calls)
    if "--dump" in sys.argv:
        print(json.dumps(pc))
        return
    print(json.dumps({"per_call": pc, "configs0": configs0(ctx, sc, ob)}))


if __name__ == "__main__":
    main()
