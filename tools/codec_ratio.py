"""Compression ratio of the GPU builder's codecs against the libraries the Go writers stand for
(tooling).  configs[2]'s KVs (tools/bench_encode.py kv_arrays:
keys k%015d, V-half 84 B values) go through the GPU sstable.Builder once per codec
(slate_sst_builder_add_batch_device + build, BlockSize 4096, 10 bits per key); the SST's data
blocks, filter and index are sized from its info.  The reference-shaped sizes come from the same
decoded blocks (the CodecNone SST's block payloads, builder.go:215-268 cuts blocks on the decoded
size, so every codec sees the same blocks) compressed by:
  Snappy: C++ libsnappy 1.1.8 (golang/snappy v0.0.4 is what the Go DB writes; ours is byte-exact
          to it, so this row shows the C++-vs-Go parse difference only);
  LZ4:    liblz4 1.9.3 LZ4F_compressFrame with pierrec/lz4 v4's writer defaults (4 MiB blocks,
          independent, content checksum, fast level);
  Zstd:   libzstd 1.4.9 level 3 + checksum + content size (klauspost/compress SpeedDefault is
          level-3 class);
  Zlib:   zlib level 6 (compress/zlib's DefaultCompression), plus the 5 bytes of the empty final
          stored block Go's writer closes with.
klauspost/compress, pierrec/lz4 and Go's compress/flate are absent here, so these are the
closest library stand-ins, not the Go bytes (parity unpinned for size).
usage: python tools/codec_ratio.py [--kv N]   (one JSON line per codec, then a summary line)"""
import argparse
import json
import os
import sys
import zlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "slatedb-go_amd")]


def block_layout(ctx, sc, sst: np.ndarray, codec: int):
    """(block offsets uint64[n+1] with the data-blocks end last, filter_len, index_len) of one SST."""
    info = sc.SstInfo()
    fk = np.zeros(1 << 16, np.uint8)
    st = sc.lib().slate_sst_read_info(sc._ptr(sst), sst.size, sc.C.byref(info), sc._ptr(fk), fk.size)
    assert st == sc.OK, st
    io, il, fo, fl = info.index_offset, info.index_len, info.filter_offset, info.filter_len
    st, index = ctx.decode_index(sst[io:io + il].tobytes(), codec)
    assert st == sc.OK, st
    offs = index.block_offsets()
    return np.append(offs, np.uint64(fo if fl else io)), int(fl), int(il)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--kv", type=int, default=10_000_000)
    p.add_argument("--threads", type=int, default=16)
    args = p.parse_args()
    import torch
    import slatecodec as sc
    from tools import workload as wl
    from tools.bench_encode import kv_arrays
    keys, key_off, vals, val_off = kv_arrays(args.kv)
    ctx = sc.Context(0)
    dev = torch.device("cuda", 0)
    d_keys, d_vals = torch.from_numpy(keys).to(dev), torch.from_numpy(vals).to(dev)
    d_ko = torch.from_numpy(key_off.view(np.int64)).to(dev)
    d_vo = torch.from_numpy(val_off.view(np.int64)).to(dev)
    torch.cuda.synchronize()
    names = {sc.NONE: "none", sc.SNAPPY: "snappy", sc.ZLIB: "zlib", sc.LZ4: "lz4", sc.ZSTD: "zstd"}
    ssts = {}
    for codec in names:
        b = sc.SstBuilder(ctx, 4096, 0, 10, codec)
        assert b.add_batch_device(d_keys.data_ptr(), d_ko.data_ptr(), d_vals.data_ptr(), d_vo.data_ptr(),
                                  args.kv) == 0
        ssts[codec] = b.build().encode_array().copy()
        del b
    # the decoded blocks: the CodecNone SST's block payloads without their CRC trailers
    none = ssts[sc.NONE]
    offs, _, _ = block_layout(ctx, sc, none, sc.NONE)
    n = offs.size - 1
    keep = np.ones(int(offs[-1]), bool)
    crc_at = (offs[1:].astype(np.int64) - 4)[:, None] + np.arange(4)
    keep[crc_at.reshape(-1)] = False
    dec = np.ascontiguousarray(none[: int(offs[-1])][keep])
    dec_off = offs - 4 * np.arange(n + 1, dtype=np.uint64)
    decoded = int(dec_off[-1])
    lib_sizes = {sc.NONE: decoded + 4 * n}
    for codec, bg in ((sc.SNAPPY, 1), (sc.LZ4, 3), (sc.ZSTD, 4)):
        blob, off = wl.encode_blocks(bg, dec, dec_off, args.threads)
        lib_sizes[codec] = int(off[-1])
    views = [dec[int(dec_off[i]):int(dec_off[i + 1])].tobytes() for i in range(n)]
    with ThreadPoolExecutor(args.threads) as ex:
        lib_sizes[sc.ZLIB] = sum(ex.map(lambda v: len(zlib.compress(v, 6)) + 5 + 4, views, chunksize=1024))
    lib_name = {sc.NONE: "-", sc.SNAPPY: "libsnappy 1.1.8", sc.LZ4: "liblz4 1.9.3 (pierrec/lz4 v4 defaults)",
                sc.ZSTD: "libzstd 1.4.9 level 3", sc.ZLIB: "zlib level 6 (+ Go's 5-byte final block)"}
    summary = {}
    for codec, name in names.items():
        sst = ssts[codec]
        o, fl, il = block_layout(ctx, sc, sst, codec)
        assert o.size == n + 1, (name, o.size, n + 1)  # same blocks for every codec
        ours = int(o[-1])
        res = {"codec": name, "kv": args.kv, "blocks": n, "decoded_block_bytes": decoded,
               "sst_bytes": int(sst.size), "data_block_bytes": ours, "filter_bytes": fl, "index_bytes": il,
               "ratio_decoded_over_ours": round(decoded / ours, 4),
               "library": lib_name[codec], "library_data_block_bytes": lib_sizes[codec],
               "ratio_decoded_over_library": round(decoded / lib_sizes[codec], 4),
               "ours_over_library": round(ours / lib_sizes[codec], 4)}
        summary[name] = res["ours_over_library"]
        print(json.dumps(res), flush=True)
    print(json.dumps({"summary": "data-block bytes, ours / library", **summary}), flush=True)


if __name__ == "__main__":
    main()
