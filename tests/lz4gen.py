"""LZ4 frames for decoder tests (test infrastructure only).

A small greedy LZ4 block compressor and frame writer (LZ4 frame format v1.6.x, block
format: token = literal-length nibble | match-length nibble, 255-run length extensions,
LE16 offsets, last sequence literals only), with every frame option the decoders accept:
block max size id, independent or linked blocks, block checksums, content checksum,
content size, stored (uncompressed) blocks.  XXH32 comes from the xxhash module.  The
decoders' parity anchor is tests/golden/lz4_frames.json (frames written by liblz4).
"""
from __future__ import annotations

import random
import struct

import xxhash


def xxh32(b: bytes) -> int:
    return xxhash.xxh32(b, seed=0).intdigest()


def _lenext(n: int) -> bytes:
    out = bytearray()
    while n >= 255:
        out.append(255)
        n -= 255
    out.append(n)
    return bytes(out)


def compress_block(src: bytes, window: bytes = b"", rng: random.Random | None = None,
                   offsets_only_near: bool = False) -> bytes:
    """Greedy LZ4 block of `src`; matches may reach into `window` (the preceding output)."""
    data = window + src
    base = len(window)
    out = bytearray()
    table: dict[bytes, int] = {}
    for p in range(max(0, base - 65535), base - 3):
        table[data[p:p + 4]] = p
    i = base
    lit_start = base
    end = len(data)
    while i + 4 <= end:
        key = data[i:i + 4]
        cand = table.get(key)
        table[key] = i
        if cand is not None and 0 < i - cand <= 65535 and (not offsets_only_near or i - cand < 300):
            n = 4
            while i + n < end and data[cand + n] == data[i + n]:
                n += 1
            if rng is not None and n > 4 and rng.random() < 0.3:
                n = rng.randint(4, n)  # vary match lengths
            lits = data[lit_start:i]
            ll, ml = len(lits), n - 4
            out.append((min(ll, 15) << 4) | min(ml, 15))
            if ll >= 15:
                out += _lenext(ll - 15)
            out += lits
            out += struct.pack("<H", i - cand)
            if ml >= 15:
                out += _lenext(ml - 15)
            for p in range(i + 1, min(i + n, end - 3)):
                table[data[p:p + 4]] = p
            i += n
            lit_start = i
        else:
            i += 1
    lits = data[lit_start:]
    ll = len(lits)
    out.append(min(ll, 15) << 4)
    if ll >= 15:
        out += _lenext(ll - 15)
    out += lits
    return bytes(out)


def frame(data: bytes, bsid: int = 7, indep: bool = True, block_checksum: bool = False,
          content_checksum: bool = True, content_size: bool = False, stored_p: float = 0.0,
          rng: random.Random | None = None, block_split: int | None = None) -> bytes:
    """An LZ4 frame of `data`.  block_split (bytes per block) defaults to the max block size."""
    rng = rng or random.Random(0)
    bmax = 1 << (8 + 2 * bsid)
    split = min(block_split or bmax, bmax)
    flg = (1 << 6) | (int(indep) << 5) | (int(block_checksum) << 4) | (int(content_size) << 3) | \
          (int(content_checksum) << 2)
    desc = bytes([flg, bsid << 4]) + (struct.pack("<Q", len(data)) if content_size else b"")
    out = bytearray(struct.pack("<I", 0x184D2204) + desc + bytes([(xxh32(desc) >> 8) & 0xFF]))
    pos = 0
    while pos < len(data):
        chunk = data[pos:pos + split]
        window = b"" if indep else data[max(0, pos - 65536):pos]
        comp = compress_block(chunk, window, rng)
        if rng.random() < stored_p or len(comp) >= len(chunk):
            body, size = chunk, len(chunk) | 0x80000000
        else:
            body, size = comp, len(comp)
        out += struct.pack("<I", size) + body
        if block_checksum:
            out += struct.pack("<I", xxh32(body))
        pos += len(chunk)
    out += struct.pack("<I", 0)
    if content_checksum:
        out += struct.pack("<I", xxh32(data))
    return bytes(out)


def block(decoded: bytes, rng: random.Random, **kw) -> bytes:
    """A CodecLz4 SST block: frame(decoded) || BE32 CRC32 of the frame (block.go:54-75)."""
    import zlib
    f = frame(decoded, rng=rng, **kw)
    return f + struct.pack(">I", zlib.crc32(f))
