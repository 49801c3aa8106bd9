"""Hand-built Snappy streams for decoder coverage (test infrastructure only).

The oracle's encoder (a golang/snappy restatement) picks its own tags, so it never
produces some tag shapes the GPU decoder handles on separate paths: copies with
offsets just past the output ring (113+), long far copies (> 16 bytes), far copies
back to back, copies that read bytes a pending far copy is still filling, and
short-period overlapping copies.  These helpers emit chosen tags (golang/snappy
block format: varint length, then literal / copy-1 / copy-2 / copy-4 tags,
snappy/format_description.txt) and build rows in the v0 layout with timestamp
flags (row.go:111-147), so the expected results come from the oracle's decoder.
"""
from __future__ import annotations

import random
import struct
import zlib


def varint(n: int) -> bytes:
    out = bytearray()
    while n >= 0x80:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def tag_literal(data: bytes) -> bytes:
    n = len(data) - 1
    if n < 60:
        return bytes([n << 2]) + data
    nb = (n.bit_length() + 7) // 8
    return bytes([(59 + nb) << 2]) + n.to_bytes(nb, "little") + data


def tag_copy(off: int, length: int, form: int | None = None) -> bytes:
    """form 1/2/4 forces the copy tag width; default: the narrowest that fits."""
    if form is None:
        form = 1 if (4 <= length <= 11 and off < 2048) else (2 if off < 65536 else 4)
    if form == 1:
        assert 4 <= length <= 11 and off < 2048
        return bytes([1 | ((length - 4) << 2) | ((off >> 8) << 5), off & 0xFF])
    assert 1 <= length <= 64
    if form == 2:
        return bytes([2 | ((length - 1) << 2)]) + struct.pack("<H", off)
    return bytes([3 | ((length - 1) << 2)]) + struct.pack("<I", off)


class Stream:
    """Builds the decoded buffer and the tag stream side by side."""

    def __init__(self):
        self.out = bytearray()
        self.tags = bytearray()

    def lit(self, data: bytes):
        for i in range(0, len(data), 3000):  # also exercises the multi-byte literal lengths
            part = data[i:i + 3000]
            self.tags += tag_literal(part)
            self.out += part

    def copy(self, off: int, length: int, form: int | None = None):
        assert 0 < off <= len(self.out)
        while length:
            n = min(length, 64)
            self.tags += tag_copy(off, n, form if (form != 1 or 4 <= n <= 11) else 2)
            for _ in range(n):
                self.out.append(self.out[-off])
            length -= n

    def emit(self, target: bytes, rng: random.Random, offsets=(1, 3, 7, 15, 16, 42, 103, 112, 113, 114, 300, 1030,
                                                                 2047, 5000)):
        """Encode `target` (appended to the output) greedily: copies at chosen offsets and at
        the offsets of earlier occurrences of the next 4 bytes (so far copies arise too)."""
        i = base = len(self.out)
        pend = bytearray()  # literal bytes not yet emitted (they join self.out in lit())
        full = bytes(self.out) + target
        seen: dict[bytes, list[int]] = {}
        for p in range(max(0, i - 4096), i - 3):
            seen.setdefault(full[p:p + 4], []).append(p)
        end = len(full)

        def note(p):
            if p + 4 <= end:
                lst = seen.setdefault(full[p:p + 4], [])
                lst.append(p)
                if len(lst) > 4:
                    del lst[0]

        while i < end:
            best = (0, 0)
            cands = set(rng.sample(offsets, k=min(len(offsets), 6)))
            cands.update(i - p for p in seen.get(full[i:i + 4], ()))
            for off in cands:
                if off > i or off <= 0:
                    continue
                n = 0
                while n < 80 and i + n < end and full[i + n - off] == full[i + n]:
                    n += 1
                if n > best[0]:
                    best = (n, off)
            if best[0] >= 4:
                if pend:
                    self.lit(bytes(pend))
                    pend.clear()
                self.copy(best[1], best[0], rng.choice([None, None, 2, 4]))
                for p in range(i, i + best[0]):
                    note(p)
                i += best[0]
            else:
                pend.append(full[i])
                note(i)
                i += 1
        if pend:
            self.lit(bytes(pend))
        assert bytes(self.out[base:]) == target

    def block(self) -> bytes:
        """A Snappy-coded block: stream || BE32 CRC32 of the stream (block.go:54-75)."""
        body = varint(len(self.out)) + bytes(self.tags)
        return body + struct.pack(">I", zlib.crc32(body))


def v0_row(prefix_len: int, suffix: bytes, value: bytes | None, seq: int = 0, expire: int | None = None,
           create: int | None = None) -> bytes:
    flags = (1 if value is None else 0) | (2 if expire is not None else 0) | (4 if create is not None else 0)
    row = struct.pack(">HH", prefix_len, len(suffix)) + suffix + struct.pack(">QB", seq, flags)
    if expire is not None:
        row += struct.pack(">q", expire)
    if create is not None:
        row += struct.pack(">q", create)
    if value is not None:
        row += struct.pack(">I", len(value)) + value
    return row


def block_bytes(rows: list[bytes]) -> bytes:
    """rows || BE16 offsets || BE16 count (block.go:54-75 before compression)."""
    offs, pos = [], 0
    for r in rows:
        offs.append(pos)
        pos += len(r)
    return b"".join(rows) + b"".join(struct.pack(">H", o) for o in offs) + struct.pack(">H", len(rows))


def rows_for(rng: random.Random, n: int, value_len=(0, 120), ts_p=0.3, tomb_p=0.1, period: bytes | None = None):
    """Rows sharing the block's first key as prefix; values repeat with period / far reuse."""
    first = b"key-%06d" % rng.randrange(10 ** 6)
    rows = [v0_row(0, first, b"v0")]
    pool = [bytes(rng.randrange(256) for _ in range(rng.randint(5, 60))) for _ in range(4)]
    for i in range(1, n):
        pl = rng.randint(0, len(first))
        suf = b"%05d" % i
        kind = rng.random()
        if kind < tomb_p:
            val = None
        elif period is not None and kind < 0.6:
            val = (period * 200)[: rng.randint(*value_len)]
        else:
            val = rng.choice(pool)[: rng.randint(0, 60)] + bytes(rng.randrange(256) for _ in range(rng.randint(0, 20)))
        exp = rng.randrange(1, 10 ** 12) if rng.random() < ts_p else None
        cre = rng.randrange(1, 10 ** 12) if rng.random() < ts_p else None
        rows.append(v0_row(pl, suf, val, seq=rng.randrange(2 ** 40), expire=exp, create=cre))
    return rows
