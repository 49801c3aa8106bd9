"""Compression ratio of the library's non-Snappy block encoders against the writers Go uses
(tooling).  compress.Encode (internal/compress/compression.go:88-121)
compresses with compress/zlib NewWriter (DefaultCompression = level 6, dynamic Huffman),
pierrec/lz4's NewWriter (frames, content checksum) and klauspost/zstd's NewWriter (SpeedDefault
~ level 3).  None of those Go libraries is in this image; their C counterparts at the same
settings stand in for the sizes: zlib level 6 (python zlib), liblz4 frames (tools/benchgen.c),
libzstd level 3 (tools/benchgen.c).
Workload: configs[2] keys/values (tools/bench_encode.py kv_arrays), BlockSize 4096.  The raw
blocks come from a CodecNone SST of the GPU builder; each codec's SST is then built by the GPU
builder and its data-block bytes compared with the reference-compressed raw blocks.
usage: python tools/ratio_probe.py [--kv N]   (prints one JSON object)"""
import json
import os
import sys
import zlib

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "slatedb-go_amd")]


def data_blocks(sc, ctx, sst: bytes):
    st, info, _ = sc.read_info(sst)
    st, index = ctx.decode_index(sst[info.index_offset:info.index_offset + info.index_len], info.codec)
    offs = [int(x) for x in index.block_offsets()] + [info.filter_offset]
    return [sst[a:b] for a, b in zip(offs, offs[1:])]


def main():
    import slatecodec as sc
    from tools import workload as wl
    from tools.bench_encode import kv_arrays
    n = int(sys.argv[sys.argv.index("--kv") + 1]) if "--kv" in sys.argv else 400_000
    keys, key_off, vals, val_off = kv_arrays(n)
    ctx = sc.Context(0)

    def build(codec):
        b = sc.SstBuilder(ctx, 4096, 0, 10, codec)
        b.add_batch(keys, key_off, vals, val_off)
        return b.build().encode()

    raw = [blk[:-4] for blk in data_blocks(sc, ctx, build(sc.NONE))]  # block bytes without the CRC
    raw_bytes = sum(len(r) for r in raw)
    dec = np.frombuffer(b"".join(raw), np.uint8)
    doff = np.concatenate([[0], np.cumsum([len(r) for r in raw])]).astype(np.uint64)
    ref = {
        "zlib": sum(len(zlib.compress(r, 6)) + 4 for r in raw),
    }
    for name, code in (("lz4", sc.LZ4), ("zstd", sc.ZSTD), ("snappy", sc.SNAPPY)):
        blob, off = wl.encode_blocks(code, dec, doff, threads=8)  # liblz4 frames / libzstd 3 / libsnappy, + CRC
        ref[name] = int(off[-1])
    out = {"kv": n, "blocks": len(raw), "raw_block_bytes": raw_bytes, "codecs": {}}
    for name, code in (("snappy", sc.SNAPPY), ("zlib", sc.ZLIB), ("lz4", sc.LZ4), ("zstd", sc.ZSTD)):
        mine = sum(len(b) for b in data_blocks(sc, ctx, build(code)))
        out["codecs"][name] = {"slate_bytes": mine, "reference_writer_bytes": ref[name],
                               "slate_ratio": round(mine / raw_bytes, 4),
                               "reference_ratio": round(ref[name] / raw_bytes, 4),
                               "slate_over_reference": round(mine / ref[name], 4)}
    out["reference_writers"] = {"zlib": "python zlib level 6 (Go compress/zlib DefaultCompression)",
                                "lz4": "liblz4 LZ4F frames, 4 MiB blocks, content checksum (pierrec/lz4 NewWriter)",
                                "zstd": "libzstd level 3 + checksum (klauspost/zstd SpeedDefault)",
                                "snappy": "C++ libsnappy (golang/snappy's format; our encoder is golang/snappy's)"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
