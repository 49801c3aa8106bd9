"""Independent pure-Python restatement of the slatedb-go SST block codec.

TEST INFRASTRUCTURE ONLY (small cases).  Written separately from the C oracle
(oracle/slate_oracle.c) directly from the Go sources, so the two double-enter the
spec: tests require them to agree byte for byte.  Citations are relative to
/root/reference.  Statuses use the same integer codes as include/slatecodec.h.
"""
from __future__ import annotations

import struct
import zlib

OK = 0
E_BLOCK_TOO_SMALL, E_BLOCK_CHECKSUM, E_BLOCK_UNCOMP_SMALL = 1, 2, 3
E_BLOCK_INDEX_OFFSET, E_BLOCK_OFFSET_BOUNDS, E_BLOCK_NO_OFFSETS, E_BLOCK_FIRSTKEY_PANIC = 4, 5, 6, 7
E_INVALID_CODEC, E_SNAPPY_CORRUPT = 10, 11
E_ROW_TOO_SHORT, E_ROW_PREFIX, E_ROW_SUFFIX, E_ROW_EXPIRE, E_ROW_CREATE = 20, 21, 22, 23, 24
E_ROW_VALUE_LEN, E_ROW_VALUE, E_ROW_PANIC, E_ROW_PEEK_SHORT = 25, 26, 27, 28
E_FILTER_TOO_SMALL, E_FILTER_CHECKSUM, E_FILTER_PANIC = 30, 31, 32
E_INDEX_TOO_SHORT, E_INDEX_CHECKSUM, E_INFO_TOO_SHORT, E_INFO_CHECKSUM = 40, 41, 42, 43

NONE, SNAPPY = 0, 1
MASK64 = (1 << 64) - 1


def crc32(b: bytes) -> int:
    """hash/crc32.ChecksumIEEE == zlib.crc32."""
    return zlib.crc32(b) & 0xFFFFFFFF


def fnv1_64(b: bytes) -> int:
    """bloom.go:141 — hash/fnv New64 (FNV-1: multiply then xor)."""
    h = 0xCBF29CE484222325
    for c in b:
        h = (h * 0x100000001B3) & MASK64
        h ^= c
    return h


def compute_prefix_len(a: bytes, b: bytes) -> int:
    """row.go:292-318; the uint16 conversion truncates."""
    n = 0
    for x, y in zip(a, b):
        if x != y:
            break
        n += 1
    return n & 0xFFFF


# ------------------------------------------------------------ snappy (golang v0.0.4)
class SnappyCorrupt(Exception):
    pass


def _uvarint(buf: bytes):
    x = s = 0
    for i, c in enumerate(buf):
        if i == 10:
            return 0, -(i + 1)
        if c < 0x80:
            if i == 9 and c > 1:
                return 0, -(i + 1)
            return x | (c << s), i + 1
        x |= (c & 0x7F) << s
        s += 7
    return 0, 0


def snappy_decode(src: bytes) -> bytes:
    v, n = _uvarint(src)
    if n <= 0 or v > 0xFFFFFFFF:
        raise SnappyCorrupt()
    dst = bytearray(v)
    s, d = n, 0
    while s < len(src):
        tag = src[s] & 3
        if tag == 0:
            x = src[s] >> 2
            if x < 60:
                s += 1
            else:
                nb = x - 59
                s += 1 + nb
                if s > len(src):
                    raise SnappyCorrupt()
                x = int.from_bytes(src[s - nb:s], "little")
            ln = x + 1
            if ln > len(dst) - d or ln > len(src) - s:
                raise SnappyCorrupt()
            dst[d:d + ln] = src[s:s + ln]
            d += ln
            s += ln
            continue
        if tag == 1:
            s += 2
            if s > len(src):
                raise SnappyCorrupt()
            ln = 4 + ((src[s - 2] >> 2) & 7)
            off = ((src[s - 2] & 0xE0) << 3) | src[s - 1]
        elif tag == 2:
            s += 3
            if s > len(src):
                raise SnappyCorrupt()
            ln = 1 + (src[s - 3] >> 2)
            off = src[s - 2] | (src[s - 1] << 8)
        else:
            s += 5
            if s > len(src):
                raise SnappyCorrupt()
            ln = 1 + (src[s - 5] >> 2)
            off = int.from_bytes(src[s - 4:s], "little")
        if off <= 0 or d < off or ln > len(dst) - d:
            raise SnappyCorrupt()
        for i in range(ln):
            dst[d + i] = dst[d - off + i]
        d += ln
    if d != len(dst):
        raise SnappyCorrupt()
    return bytes(dst)


def _emit_literal(out: bytearray, lit: bytes):
    n = len(lit) - 1
    if n < 60:
        out.append(n << 2)
    elif n < 256:
        out += bytes([60 << 2, n])
    else:
        out += bytes([61 << 2, n & 0xFF, n >> 8])
    out += lit


def _emit_copy(out: bytearray, offset: int, length: int):
    while length >= 68:
        out += bytes([63 << 2 | 2, offset & 0xFF, offset >> 8])
        length -= 64
    if length > 64:
        out += bytes([59 << 2 | 2, offset & 0xFF, offset >> 8])
        length -= 60
    if length >= 12 or offset >= 2048:
        out += bytes([(length - 1) << 2 | 2, offset & 0xFF, offset >> 8])
        return
    out += bytes([((offset >> 8) << 5) | ((length - 4) << 2) | 1, offset & 0xFF])


def _load32(b, i):
    return b[i] | (b[i + 1] << 8) | (b[i + 2] << 16) | (b[i + 3] << 24)


def _hash(u, shift):
    return ((u * 0x1E35A7BD) & 0xFFFFFFFF) >> shift


def _encode_block(out: bytearray, src: bytes):
    shift = 24
    ts = 256
    while ts < (1 << 14) and ts < len(src):
        shift -= 1
        ts *= 2
    table = [0] * (1 << 14)
    s_limit = len(src) - 15
    next_emit = 0
    s = 1
    next_hash = _hash(_load32(src, s), shift)
    while True:
        skip = 32
        next_s = s
        while True:
            s = next_s
            between = skip >> 5
            next_s = s + between
            skip += between
            if next_s > s_limit:
                if next_emit < len(src):
                    _emit_literal(out, src[next_emit:])
                return
            candidate = table[next_hash & 0x3FFF]
            table[next_hash & 0x3FFF] = s
            next_hash = _hash(_load32(src, next_s), shift)
            if _load32(src, s) == _load32(src, candidate):
                break
        _emit_literal(out, src[next_emit:s])
        while True:
            base = s
            s += 4
            i = candidate + 4
            while s < len(src) and src[i] == src[s]:
                i += 1
                s += 1
            _emit_copy(out, base - candidate, s - base)
            next_emit = s
            if s >= s_limit:
                if next_emit < len(src):
                    _emit_literal(out, src[next_emit:])
                return
            x = int.from_bytes(src[s - 1:s + 7], "little")
            table[_hash(x & 0xFFFFFFFF, shift) & 0x3FFF] = s - 1
            cur = (x >> 8) & 0xFFFFFFFF
            ch = _hash(cur, shift) & 0x3FFF
            candidate = table[ch]
            table[ch] = s
            if cur != _load32(src, candidate):
                next_hash = _hash((x >> 16) & 0xFFFFFFFF, shift)
                s += 1
                break


def snappy_encode(src: bytes) -> bytes:
    out = bytearray()
    n = len(src)
    while True:
        out.append((n & 0x7F) | (0x80 if n >= 0x80 else 0))
        if n < 0x80:
            break
        n >>= 7
    p = 0
    while p < len(src):
        chunk = src[p:p + 65536]
        p += len(chunk)
        if len(chunk) < 17:
            _emit_literal(out, chunk)
        else:
            _encode_block(out, chunk)
    return bytes(out)


def compress(buf: bytes, codec: int) -> bytes:
    if codec == NONE:
        return buf
    if codec == SNAPPY:
        return snappy_encode(buf)
    raise NotImplementedError(codec)


def decompress(buf: bytes, codec: int) -> bytes:
    if codec == NONE:
        return buf
    if codec == SNAPPY:
        return snappy_decode(buf)
    raise NotImplementedError(codec)


# ------------------------------------------------------------------ v0 rows
def v0_size(suffix_len: int, tombstone: bool, value_len: int, has_expire=False, has_create=False) -> int:
    """row.go:95-107"""
    n = 2 + 2 + suffix_len + 8 + 1 + (8 if has_expire else 0) + (8 if has_create else 0)
    return n if tombstone else n + 4 + value_len


def v0_encode(prefix_len: int, suffix: bytes, value: bytes | None, seq=0, expire_ms=None, create_ms=None) -> bytes:
    """row.go:149-189; value None = tombstone."""
    flags = (1 if value is None else 0) | (2 if expire_ms is not None else 0) | (4 if create_ms is not None else 0)
    out = struct.pack(">HH", prefix_len & 0xFFFF, len(suffix) & 0xFFFF) + suffix + struct.pack(">QB", seq, flags)
    if expire_ms is not None:
        out += struct.pack(">q", expire_ms)
    if create_ms is not None:
        out += struct.pack(">q", create_ms)
    if value is not None:
        out += struct.pack(">I", len(value)) + value
    return out


def v0_decode(data: bytes, first_key_len: int | None):
    """row.go:191-261 -> (status, fields dict)."""
    n = len(data)
    if n < 13:
        return E_ROW_TOO_SHORT, None
    pl, sl = struct.unpack_from(">HH", data)
    if pl > ((first_key_len or 0) & 0xFFFF):
        return E_ROW_PREFIX, None
    o = 4
    if n - o < sl:
        return E_ROW_SUFFIX, None
    suffix = data[o:o + sl]
    o += sl
    if n - o < 9:
        return E_ROW_PANIC, None
    seq, flags = struct.unpack_from(">QB", data, o)
    o += 9
    r = dict(prefix_len=pl, suffix=suffix, seq=seq, flags=flags, expire_ms=None, create_ms=None, value=None)
    if flags & 2:
        if n - o < 8:
            return E_ROW_EXPIRE, None
        r["expire_ms"] = struct.unpack_from(">q", data, o)[0]
        o += 8
    if flags & 4:
        if n - o < 8:
            return E_ROW_CREATE, None
        r["create_ms"] = struct.unpack_from(">q", data, o)[0]
        o += 8
    if flags & 1 == 0:
        if n - o < 4:
            return E_ROW_VALUE_LEN, None
        vl = struct.unpack_from(">I", data, o)[0]
        o += 4
        if n - o < vl:
            return E_ROW_VALUE, None
        r["value"] = data[o:o + vl]
        r["meta_len"] = o - 4 - sl
    else:
        r["meta_len"] = o - 4 - sl
    return OK, r


class BlockBuilder:
    """block.go:136-204"""

    def __init__(self, block_size: int):
        self.block_size = block_size
        self.offsets: list[int] = []
        self.data = bytearray()
        self.first_key: bytes | None = None

    def cur_size(self):
        return 2 + 2 * len(self.offsets) + len(self.data)

    def add(self, key: bytes, value: bytes | None) -> bool:
        assert key
        p = compute_prefix_len(self.first_key or b"", key)
        suffix = key[p:]
        if self.cur_size() + 2 + v0_size(len(suffix), value is None, len(value or b"")) > self.block_size \
                and self.offsets:
            return False
        self.offsets.append(len(self.data) & 0xFFFF)
        self.data += v0_encode(p, suffix, value)
        if self.first_key is None:
            self.first_key = bytes(key)
        return True

    def add_value(self, key: bytes, value: bytes) -> bool:
        return self.add(key, value if value else None)


def block_encode(data: bytes, offsets: list[int], codec: int) -> bytes:
    """block.go:54-75"""
    buf = bytes(data) + b"".join(struct.pack(">H", o) for o in offsets) + struct.pack(">H", len(offsets) & 0xFFFF)
    c = compress(buf, codec)
    return c + struct.pack(">I", crc32(c))


def block_decode(inp: bytes, codec: int):
    """block.go:78-134 + iterator row walk -> (status, detail, aux, buf, data_len, rows)"""
    if len(inp) < 6:
        return E_BLOCK_TOO_SMALL, 0, 0, b"", 0, []
    comp = inp[:-4]
    if struct.unpack(">I", inp[-4:])[0] != crc32(comp):
        return E_BLOCK_CHECKSUM, 0, 0, b"", 0, []
    try:
        buf = decompress(comp, codec)
    except SnappyCorrupt:
        return E_SNAPPY_CORRUPT, 0, 0, b"", 0, []
    if len(buf) < 2:
        return E_BLOCK_UNCOMP_SMALL, 0, 0, buf, 0, []
    cnt = struct.unpack(">H", buf[-2:])[0]
    osi = len(buf) - 2 - 2 * cnt
    if osi <= 0:
        return E_BLOCK_INDEX_OFFSET, osi, 0, buf, 0, []
    offs = list(struct.unpack_from(">%dH" % cnt, buf, osi))
    for i, off in enumerate(offs):
        if off > (osi & 0xFFFF):
            return E_BLOCK_OFFSET_BOUNDS, off, i, buf, 0, []
    if cnt == 0:
        return E_BLOCK_NO_OFFSETS, 0, 0, buf, osi, []
    off0 = offs[0]
    if osi - off0 < 2:
        return E_BLOCK_FIRSTKEY_PANIC, 0, 0, buf, osi, []
    kl = struct.unpack_from(">H", buf, off0)[0]
    lo, hi = (off0 + 2) & 0xFFFF, (off0 + 2 + kl) & 0xFFFF
    if lo > hi or hi > len(buf):
        return E_BLOCK_FIRSTKEY_PANIC, 0, 0, buf, osi, []
    data = buf[:osi]
    rows = []
    fk = None
    for i, off in enumerate(offs):
        st, r = v0_decode(data[off:], None if i == 0 else fk)
        if i == 0 and st == OK:
            fk = len(r["suffix"])
        rows.append((off, st, r))
    return OK, 0, kl, buf, osi, rows


# ------------------------------------------------------------------- bloom
def optimal_num_probes(bpk: int) -> int:
    """bloom.go:174: uint16(float32(bitsPerKey) * 0.69)"""
    return int(struct.unpack("f", struct.pack("f", struct.unpack("f", struct.pack("f", bpk))[0] *
                                              struct.unpack("f", struct.pack("f", 0.69))[0]))[0]) & 0xFFFF


def filter_bytes(nkeys: int, bpk: int) -> int:
    return (((nkeys * bpk) & 0xFFFFFFFF) + 7 & 0xFFFFFFFF) // 8


def probes_for_key(h: int, num_probes: int, filter_bits: int) -> list[int]:
    """bloom.go:147-160"""
    m = filter_bits
    hh = (h & 0xFFFFFFFF) % m
    delta = (h >> 32) % m
    out = []
    for i in range(num_probes):
        delta = (delta + i) % m
        out.append(hh)
        hh = (hh + delta) % m
    return out


def bloom_build(keys: list[bytes], bpk: int) -> tuple[int, bytes]:
    if not keys:
        return 0, b""
    k = optimal_num_probes(bpk)
    nb = filter_bytes(len(keys), bpk)
    bits = bytearray(nb)
    for key in keys:
        for p in probes_for_key(fnv1_64(key), k, nb * 8):
            bits[p // 8] |= 1 << (p % 8)
    return k, bytes(bits)


def bloom_has_key(k: int, bits: bytes, key: bytes) -> bool:
    if not bits:
        return False
    return all(bits[p // 8] & (1 << (p % 8)) for p in probes_for_key(fnv1_64(key), k, len(bits) * 8))


def bloom_encode(k: int, bits: bytes, codec: int) -> bytes:
    c = compress(struct.pack(">H", k) + bits, codec)
    return c + struct.pack(">I", crc32(c))


# ------------------------------------------------------- flatbuffers (Go builder)
class FB:
    """github.com/google/flatbuffers/go Builder, restated for the calls slatedb makes."""

    def __init__(self):
        self.buf = bytearray()  # data stored reversed-agnostic: we keep the tail (head..end)
        self.minalign = 1
        self.vtable: list[int] = []
        self.object_end = 0
        self.vtables: list[int] = []

    def offset(self):
        return len(self.buf)

    def pad(self, n):
        self.buf[0:0] = bytes(n)

    def prep(self, size, additional):
        self.minalign = max(self.minalign, size)
        align = (-(len(self.buf) + additional)) & (size - 1)
        self.pad(align)

    def prepend(self, fmt, x, size):
        self.prep(size, 0)
        self.buf[0:0] = struct.pack("<" + fmt, x)

    def prepend_uoff(self, off):
        self.prep(4, 0)
        self.buf[0:0] = struct.pack("<I", self.offset() - off + 4)

    def start_object(self, n):
        self.vtable = [0] * n
        self.object_end = self.offset()

    def slot(self, i):
        self.vtable[i] = self.offset()

    def end_object(self):
        self.prep(4, 0)
        self.buf[0:0] = b"\0\0\0\0"  # soffset placeholder
        obj = self.offset()
        vt = list(self.vtable)
        while vt and vt[-1] == 0:
            vt.pop()
        existing = 0
        for vt2off in reversed(self.vtables):
            start = len(self.buf) - vt2off
            vlen = struct.unpack_from("<H", self.buf, start)[0]
            fields = [struct.unpack_from("<H", self.buf, start + 4 + 2 * i)[0] for i in range((vlen - 4) // 2)]
            if len(fields) != len(vt):
                continue
            if all((x == 0 and a == 0) or x == obj - a for x, a in zip(fields, vt)):
                existing = vt2off
                break
        if existing == 0:
            for a in reversed(vt):
                self.prepend("H", obj - a if a else 0, 2)
            self.prepend("H", obj - self.object_end, 2)
            self.prepend("H", (len(vt) + 2) * 2, 2)
            pos = len(self.buf) - obj
            struct.pack_into("<i", self.buf, pos, self.offset() - obj)
            self.vtables.append(self.offset())
        else:
            pos = len(self.buf) - obj
            struct.pack_into("<i", self.buf, pos, existing - obj)
        return obj

    def byte_vector(self, s: bytes, nul: bool):
        self.prep(4, len(s) + (1 if nul else 0))
        if nul:
            self.buf[0:0] = b"\0"
        self.buf[0:0] = s
        self.buf[0:0] = struct.pack("<I", len(s))
        return self.offset()

    def start_vector(self, elem, n, align):
        self.prep(4, elem * n)
        self.prep(align, elem * n)

    def end_vector(self, n):
        self.buf[0:0] = struct.pack("<I", n)
        return self.offset()

    def finish(self, root):
        self.prep(self.minalign, 4)
        self.prepend_uoff(root)
        return bytes(self.buf)


def encode_info(first_key: bytes | None, index_offset, index_len, filter_offset, filter_len, codec) -> bytes:
    """flatbuf.go:62-81"""
    b = FB()
    fk = b.byte_vector(first_key or b"", nul=False)
    b.start_object(6)
    b.prepend_uoff(fk)
    b.slot(0)
    for slot, v in ((1, index_offset), (2, index_len), (3, filter_offset), (4, filter_len)):
        if v:
            b.prepend("Q", v, 8)
            b.slot(slot)
    if codec:
        b.prepend("b", codec, 1)
        b.slot(5)
    out = b.finish(b.end_object())
    return out + struct.pack(">I", crc32(out))


def encode_index(metas: list[tuple[int, bytes]], codec: int) -> bytes:
    """flatbuf.go:126-139 + manifest_generated.go:457-469, 586-606"""
    b = FB()
    offs = []
    for off, key in metas:
        fk = b.byte_vector(key, nul=True)
        b.start_object(2)
        if off:
            b.prepend("Q", off, 8)
            b.slot(0)
        b.prepend_uoff(fk)
        b.slot(1)
        offs.append(b.end_object())
    b.start_vector(4, len(metas), 4)
    for o in reversed(offs):
        b.prepend_uoff(o)
    vec = b.end_vector(len(metas))
    b.start_object(1)
    b.prepend_uoff(vec)
    b.slot(0)
    out = compress(b.finish(b.end_object()), codec)
    return out + struct.pack(">I", crc32(out))


class SstBuilder:
    """builder.go:92-268"""

    def __init__(self, block_size=4096, min_filter_keys=0, bits_per_key=10, codec=NONE):
        self.cfg = (block_size, min_filter_keys, bits_per_key, codec)
        self.bb = BlockBuilder(block_size)
        self.keys: list[bytes] = []
        self.metas: list[tuple[int, bytes]] = []
        self.first_key = None
        self.blocks: list[bytes] = []
        self.current_len = 0

    def _finish_block(self):
        if not self.bb.offsets:
            return b""
        bb = self.bb
        self.bb = BlockBuilder(self.cfg[0])
        buf = block_encode(bytes(bb.data), bb.offsets, self.cfg[3])
        self.metas.append((self.current_len, bb.first_key))
        return buf

    def add(self, key: bytes, value: bytes | None):
        if not self.bb.add(key, value):
            buf = self._finish_block()
            self.current_len += len(buf)
            self.blocks.append(buf)
            assert self.bb.add(key, value)
        if self.first_key is None:
            self.first_key = key
        self.keys.append(key)

    def add_value(self, key: bytes, value: bytes):
        self.add(key, value if value else None)

    def next_block(self):
        return self.blocks.pop(0) if self.blocks else None

    def build(self) -> bytes:
        """returns the last deque element; self.blocks holds the table chunks"""
        buf = self._finish_block()
        bs, mfk, bpk, codec = self.cfg
        filter_off = self.current_len + len(buf)
        filter_len = 0
        self.bloom = None
        if len(self.keys) >= mfk:
            k, bits = bloom_build(self.keys, bpk)
            enc = bloom_encode(k, bits, codec)
            filter_len = len(enc)
            buf += enc
            self.bloom = (k, bits)
        idx = encode_index(self.metas, codec)
        index_off = self.current_len + len(buf)
        buf += idx
        meta_off = self.current_len + len(buf)
        self.info = dict(first_key=self.first_key, index_offset=index_off, index_len=len(idx),
                         filter_offset=filter_off, filter_len=filter_len, codec=codec)
        buf += encode_info(self.first_key, index_off, len(idx), filter_off, filter_len, codec)
        buf += struct.pack(">I", meta_off & 0xFFFFFFFF)
        self.blocks.append(buf)
        return buf

    def encode_table(self) -> bytes:
        return b"".join(self.blocks)
