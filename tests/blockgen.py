"""Test-input generators built on the oracle (test infrastructure only)."""
from __future__ import annotations

import random
import struct
import zlib

import numpy as np

from oracle import binding as ob


def kv_synthetic(n: int, seed: int = 20250307, half: bool = True, tomb_every: int = 0):
    """SURVEY 8d synthetic KVs: keys b"k%015d", 84-byte values (V-half = r||r)."""
    rng = np.random.default_rng(seed)
    keys = [b"k%015d" % i for i in range(n)]
    if half:
        r = rng.integers(0, 256, (n, 42), dtype=np.uint8)
        vals = np.concatenate([r, r], axis=1)
    else:
        vals = rng.integers(0, 256, (n, 84), dtype=np.uint8)
    out = []
    for i in range(n):
        v = b"" if (tomb_every and i % tomb_every == tomb_every - 1) else vals[i].tobytes()
        out.append((keys[i], v))
    return out


def kv_mixed(n: int, seed: int = 20250307):
    """SURVEY 8d config 5 KVs: ascending keys of 8-256 bytes sharing 3 + (Zipf(s=1.2) - 1) bytes
    with the previous key (restart-scan stress; the 3-byte head absorbs carries so millions of
    keys stay sorted), 1 KiB V-half values (r||r, 512 B halves)."""
    rng = np.random.default_rng(seed)
    keys, prev = [], None
    for i in range(n):
        ln = int(rng.integers(8, 257))
        if prev is None:
            head = bytearray(b"aaaa")
        else:
            p = min(3 + int(rng.zipf(1.2)) - 1, len(prev) - 1, ln - 1)
            head = bytearray(prev[:p + 1])
            while head[p] >= 0xFE:  # carry to the left
                head = head[:p]
                p -= 1
                assert p >= 0, "kv_mixed: key space exhausted"
            head[p] += 1 + int(rng.integers(0, 2))
        tail = rng.integers(ord("a"), ord("z") + 1, max(ln - len(head), 0), dtype=np.uint8).tobytes()
        k = bytes(head) + tail
        assert prev is None or k > prev
        keys.append(k)
        prev = k
    r = rng.integers(0, 256, (n, 512), dtype=np.uint8)
    return [(keys[i], np.concatenate([r[i], r[i]]).tobytes()) for i in range(n)]


def random_kvs(rng: random.Random, n: int, klen=(1, 24), vlen=(0, 120), tomb_p=0.1, alphabet=256):
    keys = sorted({bytes(rng.randrange(alphabet) for _ in range(rng.randint(*klen))) for _ in range(n)})
    return [(k, b"" if rng.random() < tomb_p else bytes(rng.randrange(alphabet) for _ in range(rng.randint(*vlen))))
            for k in keys]


def sst_blocks(kvs, block_size=4096, codec=ob.NONE):
    """Encoded data blocks of an SST built by the oracle's sstable.Builder."""
    b = ob.SstBuilder(block_size, 1 << 30, 10, codec)
    blocks = []
    for k, v in kvs:
        assert b.add_value(k, v) == 0
        while True:
            blk = b.next_block()
            if blk is None:
                break
            blocks.append(blk)
    assert b.build() == 0
    info = b.info()
    last = b.chunks()[-1]
    # the final chunk = last block || (no filter) || index || info || BE32
    blocks.append(last[: info["filter_offset"] - sum(len(x) for x in blocks)])
    return blocks


def pack(blocks: list[bytes], misalign: int = 0):
    """Concatenate blocks into one blob + offsets (optionally not 16-byte aligned)."""
    off = np.zeros(len(blocks) + 1, np.uint64)
    pos = misalign
    parts = [b"\xee" * misalign]
    for i, b in enumerate(blocks):
        off[i] = pos
        parts.append(b)
        pos += len(b)
    off[len(blocks)] = pos
    return np.frombuffer(b"".join(parts) + b"\0" * 16, dtype=np.uint8).copy(), off


def recrc(body: bytes) -> bytes:
    return body + struct.pack(">I", zlib.crc32(body))


def mutate(rng: random.Random, blk: bytes, fix_crc: bool) -> bytes:
    body = bytearray(blk[:-4] if len(blk) >= 4 else blk)
    kind = rng.randrange(4)
    if kind == 0 and body:
        for _ in range(rng.randint(1, 4)):
            body[rng.randrange(len(body))] ^= 1 << rng.randrange(8)
    elif kind == 1 and body:
        body = body[: rng.randrange(len(body))]
    elif kind == 2 and len(body) >= 2:
        i = rng.randrange(len(body) - 1)
        body[i:i + 2] = struct.pack(">H", rng.choice([0, 1, 0xFFFF, rng.randrange(65536)]))
    else:
        body += bytes(rng.randrange(256) for _ in range(rng.randint(1, 8)))
    return recrc(bytes(body)) if fix_crc else bytes(body) + blk[-4:]


def decoded_len(blk: bytes, codec: int) -> int | None:
    if len(blk) < 6:
        return None
    body = blk[:-4]
    if codec == ob.NONE:
        return len(body)
    x = s = 0
    for i, c in enumerate(body[:10]):
        x |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return x
    return None
