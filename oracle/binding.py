"""ctypes binding of the C oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  The product never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")

NONE, SNAPPY, ZLIB, LZ4, ZSTD = 0, 1, 2, 3, 4

u8p = C.POINTER(C.c_uint8)
u16p = C.POINTER(C.c_uint16)
u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)
szp = C.POINTER(C.c_size_t)


class BlockMeta(C.Structure):
    _fields_ = [("status", C.c_int16), ("flags", C.c_uint16), ("detail", C.c_int32),
                ("data_len", C.c_uint32), ("n_rows", C.c_uint16), ("aux", C.c_uint16)]


class Row(C.Structure):
    _fields_ = [("row_off", C.c_uint32), ("key_prefix_len", C.c_uint16), ("key_suffix_len", C.c_uint16),
                ("value_len", C.c_uint32), ("flags", C.c_uint8), ("meta_len", C.c_uint8),
                ("status", C.c_int16)]


class SstInfo(C.Structure):
    _fields_ = [("index_offset", C.c_uint64), ("index_len", C.c_uint64), ("filter_offset", C.c_uint64),
                ("filter_len", C.c_uint64), ("codec", C.c_int32), ("first_key_len", C.c_uint32)]


class RowValue(C.Structure):
    _fields_ = [("key_prefix_len", C.c_uint16), ("key_suffix", u8p), ("key_suffix_len", C.c_size_t),
                ("seq", C.c_uint64), ("tombstone", C.c_int), ("has_expire", C.c_int),
                ("expire_ms", C.c_int64), ("has_create", C.c_int), ("create_ms", C.c_int64),
                ("value", u8p), ("value_len", C.c_size_t)]


META_DTYPE = np.dtype([("status", "<i2"), ("flags", "<u2"), ("detail", "<i4"), ("data_len", "<u4"),
                       ("n_rows", "<u2"), ("aux", "<u2")])
ROW_DTYPE = np.dtype([("row_off", "<u4"), ("key_prefix_len", "<u2"), ("key_suffix_len", "<u2"),
                      ("value_len", "<u4"), ("flags", "u1"), ("meta_len", "u1"), ("status", "<i2")])
assert META_DTYPE.itemsize == 16 and ROW_DTYPE.itemsize == 16


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        sig = {
            "or_status_string": (C.c_char_p, [C.c_int]),
            "or_crc32": (C.c_uint32, [u8p, C.c_size_t]),
            "or_fnv1_64": (C.c_uint64, [u8p, C.c_size_t]),
            "or_compute_prefix_len": (C.c_uint16, [u8p, C.c_size_t, u8p, C.c_size_t]),
            "or_snappy_max_encoded_len": (C.c_size_t, [C.c_size_t]),
            "or_snappy_encode": (C.c_size_t, [u8p, C.c_size_t, u8p]),
            "or_snappy_decoded_len": (C.c_int, [u8p, C.c_size_t, u64p, C.POINTER(C.c_int)]),
            "or_snappy_decode": (C.c_int, [u8p, C.c_size_t, u8p, C.c_size_t]),
            "or_xxh32": (C.c_uint32, [u8p, C.c_size_t, C.c_uint32]),
            "or_lz4_frame_len": (C.c_int, [u8p, C.c_size_t, u64p]),
            "or_lz4_decode": (C.c_int, [u8p, C.c_size_t, u8p, C.c_size_t, szp]),
            "or_zlib_decode": (C.c_int, [u8p, C.c_size_t, u8p, C.c_size_t, szp]),
            "or_xxh64": (C.c_uint64, [u8p, C.c_size_t, C.c_uint64]),
            "or_zstd_plan": (C.c_int, [u8p, C.c_size_t, u64p]),
            "or_zstd_decode": (C.c_int, [u8p, C.c_size_t, u8p, C.c_size_t, szp]),
            "or_decompress_len": (C.c_int, [C.c_int, u8p, C.c_size_t, u64p]),
            "or_v0_size": (C.c_size_t, [C.POINTER(RowValue)]),
            "or_v0_encode": (C.c_size_t, [C.POINTER(RowValue), u8p]),
            "or_v0_decode": (C.c_int, [u8p, C.c_size_t, C.c_long, C.POINTER(RowValue)]),
            "or_v0_peek": (C.c_int, [u8p, C.c_size_t, C.c_long, u16p, u16p]),
            "or_block_seek": (C.c_int, [u8p, C.c_uint32, u16p, C.c_uint32, u8p, C.c_size_t,
                                        C.POINTER(C.c_uint32), C.POINTER(C.c_int32), C.POINTER(C.c_uint32),
                                        C.POINTER(C.c_uint32)]),
            "or_block_seek_w": (C.c_int, [u8p, C.c_uint32, u16p, C.c_uint32, u8p, C.c_size_t,
                                          C.POINTER(C.c_uint32), C.POINTER(C.c_int32), C.POINTER(C.c_uint32),
                                          C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_uint32]),
            "or_index_seek": (C.c_uint64, [u8p, u64p, C.c_uint64, u8p, C.c_size_t]),
            "or_v0_estimate_block_size": (C.c_uint64, [u8p, u64p, u8p, u64p, C.c_size_t]),
            "or_block_builder_new": (C.c_void_p, [C.c_uint64]),
            "or_block_builder_free": (None, [C.c_void_p]),
            "or_block_builder_add": (C.c_int, [C.c_void_p, u8p, C.c_size_t, C.c_int, u8p, C.c_size_t]),
            "or_block_builder_add_value": (C.c_int, [C.c_void_p, u8p, C.c_size_t, u8p, C.c_size_t]),
            "or_block_builder_is_empty": (C.c_int, [C.c_void_p]),
            "or_block_builder_data": (C.c_size_t, [C.c_void_p, C.POINTER(u8p)]),
            "or_block_builder_offsets": (C.c_size_t, [C.c_void_p, C.POINTER(u16p)]),
            "or_block_builder_first_key": (C.c_size_t, [C.c_void_p, C.POINTER(u8p)]),
            "or_block_encode_bound": (C.c_size_t, [C.c_size_t, C.c_size_t]),
            "or_block_encode": (C.c_int, [u8p, C.c_size_t, u16p, C.c_size_t, C.c_int, u8p, C.c_size_t, szp]),
            "or_block_decode": (C.c_int, [u8p, C.c_size_t, C.c_int, u8p, C.c_size_t, szp,
                                          C.POINTER(BlockMeta), C.POINTER(Row), C.c_size_t]),
            "or_block_decode_batch": (C.c_int, [C.c_int, u8p, u64p, C.c_uint32, u8p, C.c_uint64, u64p,
                                                C.c_void_p, C.c_void_p, C.c_uint64, u64p, C.c_int]),
            "or_row_capacity": (C.c_uint64, [C.c_uint64]),
            "or_bloom_optimal_num_probes": (C.c_uint16, [C.c_uint32]),
            "or_bloom_filter_bytes": (C.c_uint64, [C.c_uint32, C.c_uint32]),
            "or_bloom_probes": (None, [C.c_uint64, C.c_uint16, C.c_uint32, u32p]),
            "or_bloom_build": (C.c_int, [u8p, u64p, C.c_uint64, C.c_uint32, u8p, C.c_size_t, szp, u16p]),
            "or_bloom_has_key": (C.c_int, [C.c_uint16, u8p, C.c_size_t, u8p, C.c_size_t]),
            "or_bloom_encode": (C.c_int, [C.c_uint16, u8p, C.c_size_t, C.c_int, u8p, C.c_size_t, szp]),
            "or_bloom_decode": (C.c_int, [u8p, C.c_size_t, C.c_int, u16p, u8p, C.c_size_t, szp]),
            "or_encode_info": (C.c_int, [C.POINTER(SstInfo), u8p, u8p, C.c_size_t, szp]),
            "or_decode_info": (C.c_int, [u8p, C.c_size_t, C.POINTER(SstInfo), u8p, C.c_size_t]),
            "or_encode_index": (C.c_int, [u64p, u8p, u64p, C.c_size_t, C.c_int, u8p, C.c_size_t, szp]),
            "or_decode_index": (C.c_int, [u8p, C.c_size_t, C.c_int, u64p, u8p, u64p, C.c_size_t,
                                          C.c_size_t, szp]),
            "or_sst_builder_new": (C.c_void_p, [C.c_uint64, C.c_uint32, C.c_uint32, C.c_int]),
            "or_sst_builder_free": (None, [C.c_void_p]),
            "or_sst_builder_add": (C.c_int, [C.c_void_p, u8p, C.c_size_t, u8p, C.c_size_t, C.c_int]),
            "or_sst_builder_add_value": (C.c_int, [C.c_void_p, u8p, C.c_size_t, u8p, C.c_size_t]),
            "or_sst_builder_add_batch": (C.c_int, [C.c_void_p, u8p, u64p, u8p, u64p, C.c_uint64]),
            "or_sst_builder_next_block": (C.c_int, [C.c_void_p, C.POINTER(u8p), szp]),
            "or_sst_builder_build": (C.c_int, [C.c_void_p]),
            "or_sst_table_num_chunks": (C.c_size_t, [C.c_void_p]),
            "or_sst_table_chunk": (C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(u8p), szp]),
            "or_sst_table_encoded_len": (C.c_size_t, [C.c_void_p]),
            "or_sst_table_encode": (C.c_int, [C.c_void_p, u8p, C.c_size_t]),
            "or_sst_table_info": (C.c_int, [C.c_void_p, C.POINTER(SstInfo), u8p, C.c_size_t]),
            "or_sst_table_bloom": (C.c_int, [C.c_void_p, C.POINTER(C.c_int), u16p, u8p, C.c_size_t, szp]),
            "or_sst_read_info": (C.c_int, [u8p, C.c_size_t, C.POINTER(SstInfo), u8p, C.c_size_t]),
            "or_merge_sort": (C.c_int, [C.c_uint32, u8p, u64p, u64p, u32p, u64p]),
            "or_compact": (C.c_int, [u8p, u64p, C.c_uint32, u32p, C.c_uint32, C.c_uint64, C.c_int, C.c_uint64,
                                     C.c_int, u8p, C.c_uint64, u64p, C.c_uint32, u32p]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _buf(b: bytes | bytearray | np.ndarray | None):
    """Pointer to bytes (kept alive by the returned holder)."""
    if b is None:
        return None, None
    if isinstance(b, np.ndarray):
        a = np.ascontiguousarray(b)
        return a, a.ctypes.data_as(u8p)
    a = np.frombuffer(bytes(b), dtype=np.uint8) if len(b) else np.zeros(1, np.uint8)
    return a, a.ctypes.data_as(u8p)


def status_string(code: int) -> str:
    return lib().or_status_string(code).decode()


def crc32(b: bytes) -> int:
    h, p = _buf(b)
    return lib().or_crc32(p, len(b))


def fnv1_64(b: bytes) -> int:
    h, p = _buf(b)
    return lib().or_fnv1_64(p, len(b))


def compute_prefix_len(a: bytes, b: bytes) -> int:
    ha, pa = _buf(a)
    hb, pb = _buf(b)
    return lib().or_compute_prefix_len(pa, len(a), pb, len(b))


def snappy_encode(src: bytes) -> bytes:
    cap = lib().or_snappy_max_encoded_len(len(src))
    out = np.zeros(cap, np.uint8)
    h, p = _buf(src)
    n = lib().or_snappy_encode(p, len(src), out.ctypes.data_as(u8p))
    return out[:n].tobytes()


def snappy_decode(src: bytes) -> tuple[int, bytes]:
    h, p = _buf(src)
    dl = C.c_uint64()
    hdr = C.c_int()
    st = lib().or_snappy_decoded_len(p, len(src), C.byref(dl), C.byref(hdr))
    if st:
        return st, b""
    if dl.value > 22 * len(src):
        return 11, b""
    out = np.zeros(max(dl.value, 1), np.uint8)
    st = lib().or_snappy_decode(p, len(src), out.ctypes.data_as(u8p), dl.value)
    return st, (out[:dl.value].tobytes() if st == 0 else b"")


def xxh32(src: bytes, seed: int = 0) -> int:
    h, p = _buf(src)
    return lib().or_xxh32(p, len(src), seed)


def lz4_decode(src: bytes) -> tuple[int, bytes]:
    """compress.Decode(CodecLz4): (status, decoded bytes) - the frame decoded in order."""
    h, p = _buf(src)
    dl = C.c_uint64()
    lib().or_lz4_frame_len(p, len(src), C.byref(dl))
    out = np.zeros(max(dl.value, 1), np.uint8)
    n = C.c_size_t()
    st = lib().or_lz4_decode(p, len(src), out.ctypes.data_as(u8p), dl.value, C.byref(n))
    return st, (out[:n.value].tobytes() if st == 0 else b"")


def zlib_decode(src: bytes) -> tuple[int, bytes]:
    """compress.Decode(CodecZlib): (status, decoded bytes) - the stream decoded in order."""
    h, p = _buf(src)
    dl = C.c_uint64()
    lib().or_decompress_len(ZLIB, p, len(src), C.byref(dl))
    out = np.zeros(max(dl.value, 1), np.uint8)
    n = C.c_size_t()
    st = lib().or_zlib_decode(p, len(src), out.ctypes.data_as(u8p), dl.value, C.byref(n))
    return st, (out[:n.value].tobytes() if st == 0 else b"")


def zstd_plan(src: bytes) -> int:
    h, p = _buf(src)
    dl = C.c_uint64()
    lib().or_zstd_plan(p, len(src), C.byref(dl))
    return dl.value


def zstd_decode(src: bytes) -> tuple[int, bytes]:
    """compress.Decode(CodecZstd): (status, decoded bytes) - frames decoded in order into the plan size."""
    h, p = _buf(src)
    cap = zstd_plan(src)
    out = np.zeros(max(cap, 1), np.uint8)
    n = C.c_size_t()
    st = lib().or_zstd_decode(p, len(src), out.ctypes.data_as(u8p), cap, C.byref(n))
    return st, (out[:n.value].tobytes() if st == 0 else b"")


def xxh64(b: bytes, seed: int = 0) -> int:
    h, p = _buf(b)
    return lib().or_xxh64(p, len(b), seed)


@dataclass
class DecodedRow:
    status: int
    key_prefix_len: int = 0
    key_suffix: bytes = b""
    seq: int = 0
    tombstone: bool = False
    expire_ms: int | None = None
    create_ms: int | None = None
    value: bytes = b""


def v0_encode(prefix_len: int, suffix: bytes, value: bytes | None, seq: int = 0,
              expire_ms: int | None = None, create_ms: int | None = None) -> bytes:
    hs, ps = _buf(suffix)
    hv, pv = _buf(value or b"")
    r = RowValue(prefix_len, ps, len(suffix), seq, int(value is None), int(expire_ms is not None),
                 expire_ms or 0, int(create_ms is not None), create_ms or 0, pv, len(value or b""))
    n = lib().or_v0_size(C.byref(r))
    out = np.zeros(max(n, 1), np.uint8)
    m = lib().or_v0_encode(C.byref(r), out.ctypes.data_as(u8p))
    assert m == n
    return out[:n].tobytes()


def v0_decode(data: bytes, first_key_len: int | None) -> DecodedRow:
    h, p = _buf(data)
    r = RowValue()
    st = lib().or_v0_decode(p, len(data), -1 if first_key_len is None else first_key_len, C.byref(r))
    if st:
        return DecodedRow(st)
    return DecodedRow(0, r.key_prefix_len, C.string_at(r.key_suffix, r.key_suffix_len) if r.key_suffix_len else b"",
                      r.seq, bool(r.tombstone), r.expire_ms if r.has_expire else None,
                      r.create_ms if r.has_create else None,
                      C.string_at(r.value, r.value_len) if r.value_len else b"")


def v0_peek(data: bytes, first_key_len: int | None) -> tuple[int, int, int]:
    h, p = _buf(data)
    pl, sl = C.c_uint16(), C.c_uint16()
    st = lib().or_v0_peek(p, len(data), -1 if first_key_len is None else first_key_len, C.byref(pl), C.byref(sl))
    return st, pl.value, sl.value


def block_seek(data: bytes, offsets: list[int], key: bytes) -> tuple[int, int, int, int, int]:
    """block.NewIteratorAtKey over a decoded block -> (status, start, first_idx, first_len, n_warn)."""
    hd, pd = _buf(data)
    offs = np.array(offsets or [0], dtype=np.uint16)
    hk, pk = _buf(key)
    st_, fi, fl, nw = C.c_uint32(), C.c_int32(), C.c_uint32(), C.c_uint32()
    st = lib().or_block_seek(pd, len(data), offs.ctypes.data_as(u16p), len(offsets), pk, len(key), C.byref(st_),
                             C.byref(fi), C.byref(fl), C.byref(nw))
    return st, st_.value, fi.value, fl.value, nw.value


def block_seek_warnings(data: bytes, offsets: list[int], key: bytes, cap: int = 64):
    """block_seek plus the warnings NewIteratorAtKey adds, in order: [(kind, err, a, b), ...]
    (the first `cap` of them; n_warn in the result counts all)."""
    hd, pd = _buf(data)
    offs = np.array(offsets or [0], dtype=np.uint16)
    hk, pk = _buf(key)
    st_, fi, fl, nw = C.c_uint32(), C.c_int32(), C.c_uint32(), C.c_uint32()
    w = np.zeros(4 * max(cap, 1), np.uint32)
    st = lib().or_block_seek_w(pd, len(data), offs.ctypes.data_as(u16p), len(offsets), pk, len(key), C.byref(st_),
                               C.byref(fi), C.byref(fl), C.byref(nw), w.ctypes.data_as(C.POINTER(C.c_uint32)), cap)
    warns = [(int(w[4 * k]), int(np.int32(w[4 * k + 1])), int(w[4 * k + 2]), int(w[4 * k + 3]))
             for k in range(min(nw.value, cap))]
    return (st, st_.value, fi.value, fl.value, nw.value), warns


def index_seek(first_keys: list[bytes], key: bytes) -> int:
    """sstable.Iterator.firstBlockIncludingOrAfterKey over the index's first keys."""
    kd, ko = _arena(first_keys)
    hk, pk = _buf(key)
    return int(lib().or_index_seek(kd.ctypes.data_as(u8p), ko.ctypes.data_as(u64p), len(first_keys), pk, len(key)))


def _arena(items: list[bytes]):
    off = np.zeros(len(items) + 1, np.uint64)
    off[1:] = np.cumsum([len(x) for x in items], dtype=np.uint64) if items else []
    data = np.frombuffer(b"".join(items) or b"\0", dtype=np.uint8).copy()
    return data, off


def v0_estimate_block_size(kvs: list[tuple[bytes, bytes]]) -> int:
    kd, ko = _arena([k for k, _ in kvs])
    vd, vo = _arena([v for _, v in kvs])
    return lib().or_v0_estimate_block_size(kd.ctypes.data_as(u8p), ko.ctypes.data_as(u64p),
                                           vd.ctypes.data_as(u8p), vo.ctypes.data_as(u64p), len(kvs))


class BlockBuilder:
    """block.Builder (block.go:136-204)."""

    def __init__(self, block_size: int):
        self._h = lib().or_block_builder_new(block_size)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().or_block_builder_free(self._h)

    def add(self, key: bytes, value: bytes | None) -> bool:
        hk, pk = _buf(key)
        hv, pv = _buf(value or b"")
        return bool(lib().or_block_builder_add(self._h, pk, len(key), int(value is None), pv, len(value or b"")))

    def add_value(self, key: bytes, value: bytes) -> bool:
        hk, pk = _buf(key)
        hv, pv = _buf(value)
        return bool(lib().or_block_builder_add_value(self._h, pk, len(key), pv, len(value)))

    def is_empty(self) -> bool:
        return bool(lib().or_block_builder_is_empty(self._h))

    def build(self) -> tuple[bytes, list[int], bytes]:
        """(Data, Offsets, FirstKey)"""
        d = u8p()
        n = lib().or_block_builder_data(self._h, C.byref(d))
        o = u16p()
        m = lib().or_block_builder_offsets(self._h, C.byref(o))
        k = u8p()
        kl = lib().or_block_builder_first_key(self._h, C.byref(k))
        return (C.string_at(d, n) if n else b"", [o[i] for i in range(m)], C.string_at(k, kl) if kl else b"")


def block_encode(data: bytes, offsets: list[int], codec: int) -> tuple[int, bytes]:
    cap = lib().or_block_encode_bound(len(data), len(offsets))
    out = np.zeros(cap, np.uint8)
    hd, pd = _buf(data)
    offs = np.array(offsets or [0], dtype=np.uint16)
    ol = C.c_size_t()
    st = lib().or_block_encode(pd, len(data), offs.ctypes.data_as(u16p), len(offsets), codec,
                               out.ctypes.data_as(u8p), cap, C.byref(ol))
    return st, out[:ol.value].tobytes()


def block_decode(encoded: bytes, codec: int, cap: int | None = None):
    """block.Decode -> (meta dict, decoded buffer, rows ndarray)."""
    if cap is None:
        cap = max(len(encoded) * 24, 64)
    out = np.zeros(cap, np.uint8)
    rows_cap = lib().or_row_capacity(cap)
    rows = (Row * max(rows_cap, 1))()
    meta = BlockMeta()
    ol = C.c_size_t()
    h, p = _buf(encoded)
    lib().or_block_decode(p, len(encoded), codec, out.ctypes.data_as(u8p), cap, C.byref(ol), C.byref(meta),
                          rows, rows_cap)
    m = {f: getattr(meta, f) for f, _ in BlockMeta._fields_}
    nr = min(meta.n_rows, rows_cap) if meta.status == 0 else 0
    rarr = np.frombuffer(bytes(rows)[: 16 * nr], dtype=ROW_DTYPE).copy()
    return m, out[:ol.value].tobytes(), rarr


def block_decode_batch(codec: int, blob: np.ndarray, in_off: np.ndarray, nthreads: int = 1):
    n = len(in_off) - 1
    # plan pass (mirrors slate_block_decode_plan_device)
    out_off = np.zeros(n + 1, np.uint64)
    row_base = np.zeros(n + 1, np.uint64)
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    if blob.size == 0:  # an empty blob has no data pointer; the offsets say every block is empty
        blob = np.zeros(1, np.uint8)
    in_off = np.ascontiguousarray(in_off, dtype=np.uint64)
    # first call with zero capacity just computes the plan
    L = lib()
    st = L.or_block_decode_batch(codec, blob.ctypes.data_as(u8p), in_off.ctypes.data_as(u64p), n,
                                 None, 0, out_off.ctypes.data_as(u64p), None, None, 0,
                                 row_base.ctypes.data_as(u64p), nthreads)
    out = np.zeros(max(int(out_off[n]), 1), np.uint8)
    meta = np.zeros(max(n, 1), META_DTYPE)
    rows = np.zeros(max(int(row_base[n]), 1), ROW_DTYPE)
    st = L.or_block_decode_batch(codec, blob.ctypes.data_as(u8p), in_off.ctypes.data_as(u64p), n,
                                 out.ctypes.data_as(u8p), out.size, out_off.ctypes.data_as(u64p),
                                 meta.ctypes.data, rows.ctypes.data, rows.size,
                                 row_base.ctypes.data_as(u64p), nthreads)
    assert st == 0, st
    return out, out_off, meta[:n], rows, row_base


def row_capacity(decoded_len: int) -> int:
    return lib().or_row_capacity(decoded_len)


# ------------------------------------------------------------------ bloom
def bloom_optimal_num_probes(bpk: int) -> int:
    return lib().or_bloom_optimal_num_probes(bpk)


def bloom_filter_bytes(n: int, bpk: int) -> int:
    return lib().or_bloom_filter_bytes(n, bpk)


def bloom_probes(h: int, num_probes: int, filter_bits: int) -> list[int]:
    out = (C.c_uint32 * max(num_probes, 1))()
    lib().or_bloom_probes(h, num_probes, filter_bits, out)
    return list(out[:num_probes])


def bloom_build(keys: list[bytes], bits_per_key: int) -> tuple[int, bytes]:
    kd, ko = _arena(keys)
    cap = max(bloom_filter_bytes(len(keys), bits_per_key), 1)
    out = np.zeros(cap, np.uint8)
    bl = C.c_size_t()
    np_ = C.c_uint16()
    st = lib().or_bloom_build(kd.ctypes.data_as(u8p), ko.ctypes.data_as(u64p), len(keys), bits_per_key,
                              out.ctypes.data_as(u8p), cap, C.byref(bl), C.byref(np_))
    assert st == 0, st
    return np_.value, out[:bl.value].tobytes()


def bloom_has_key(num_probes: int, bits: bytes, key: bytes) -> bool:
    hb, pb = _buf(bits)
    hk, pk = _buf(key)
    return bool(lib().or_bloom_has_key(num_probes, pb, len(bits), pk, len(key)))


def bloom_encode(num_probes: int, bits: bytes, codec: int) -> bytes:
    cap = lib().or_snappy_max_encoded_len(len(bits) + 2) + 8
    out = np.zeros(cap, np.uint8)
    hb, pb = _buf(bits)
    ol = C.c_size_t()
    st = lib().or_bloom_encode(num_probes, pb, len(bits), codec, out.ctypes.data_as(u8p), cap, C.byref(ol))
    assert st == 0, st
    return out[:ol.value].tobytes()


def bloom_decode(buf: bytes, codec: int, cap: int | None = None) -> tuple[int, int, bytes]:
    cap = cap or max(len(buf) * 24, 16)
    out = np.zeros(cap, np.uint8)
    h, p = _buf(buf)
    np_ = C.c_uint16()
    bl = C.c_size_t()
    st = lib().or_bloom_decode(p, len(buf), codec, C.byref(np_), out.ctypes.data_as(u8p), cap, C.byref(bl))
    return st, np_.value, (out[:bl.value].tobytes() if st == 0 else b"")


# --------------------------------------------------------------- flatbuffers
def encode_info(first_key: bytes | None, index_offset: int, index_len: int, filter_offset: int,
                filter_len: int, codec: int) -> bytes:
    info = SstInfo(index_offset, index_len, filter_offset, filter_len, codec,
                   len(first_key) if first_key is not None else 0)
    h, p = _buf(first_key if first_key is not None else None)
    out = np.zeros(256 + len(first_key or b""), np.uint8)
    ol = C.c_size_t()
    st = lib().or_encode_info(C.byref(info), p, out.ctypes.data_as(u8p), out.size, C.byref(ol))
    assert st == 0, st
    return out[:ol.value].tobytes()


def decode_info(buf: bytes) -> tuple[int, dict]:
    h, p = _buf(buf)
    info = SstInfo()
    fk = np.zeros(max(len(buf), 1), np.uint8)
    st = lib().or_decode_info(p, len(buf), C.byref(info), fk.ctypes.data_as(u8p), fk.size)
    d = {f: getattr(info, f) for f, _ in SstInfo._fields_}
    d["first_key"] = fk[: info.first_key_len].tobytes()
    return st, d


def encode_index(metas: list[tuple[int, bytes]], codec: int) -> bytes:
    offs = np.array([m[0] for m in metas] or [0], dtype=np.uint64)
    kd, ko = _arena([m[1] for m in metas])
    cap = lib().or_snappy_max_encoded_len(64 + 40 * len(metas) + int(ko[-1])) + 8
    out = np.zeros(cap, np.uint8)
    ol = C.c_size_t()
    st = lib().or_encode_index(offs.ctypes.data_as(u64p), kd.ctypes.data_as(u8p), ko.ctypes.data_as(u64p),
                               len(metas), codec, out.ctypes.data_as(u8p), cap, C.byref(ol))
    assert st == 0, st
    return out[:ol.value].tobytes()


def decode_index(buf: bytes, codec: int, cap: int | None = None) -> tuple[int, list[tuple[int, bytes]]]:
    h, p = _buf(buf)
    cap = cap or max(len(buf) * 24, 64)
    offs = np.zeros(cap, np.uint64)
    keys = np.zeros(cap, np.uint8)
    ko = np.zeros(cap + 1, np.uint64)
    n = C.c_size_t()
    st = lib().or_decode_index(p, len(buf), codec, offs.ctypes.data_as(u64p), keys.ctypes.data_as(u8p),
                               ko.ctypes.data_as(u64p), cap, cap, C.byref(n))
    if st:
        return st, []
    return 0, [(int(offs[i]), keys[int(ko[i]):int(ko[i + 1])].tobytes()) for i in range(n.value)]


# ------------------------------------------------------------- SST builder
class SstBuilder:
    """sstable.Builder (builder.go:92-268) restated in C."""

    def __init__(self, block_size=4096, min_filter_keys=0, filter_bits_per_key=10, codec=NONE):
        self._h = lib().or_sst_builder_new(block_size, min_filter_keys, filter_bits_per_key, codec)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().or_sst_builder_free(self._h)

    def add_value(self, key: bytes, value: bytes) -> int:
        hk, pk = _buf(key)
        hv, pv = _buf(value)
        return lib().or_sst_builder_add_value(self._h, pk, len(key), pv, len(value))

    def add(self, key: bytes, value: bytes | None) -> int:
        hk, pk = _buf(key)
        hv, pv = _buf(value or b"")
        return lib().or_sst_builder_add(self._h, pk, len(key), pv, len(value or b""), int(value is None))

    def add_batch(self, keys: np.ndarray, key_off: np.ndarray, vals: np.ndarray, val_off: np.ndarray) -> int:
        return lib().or_sst_builder_add_batch(self._h, keys.ctypes.data_as(u8p), key_off.ctypes.data_as(u64p),
                                              vals.ctypes.data_as(u8p), val_off.ctypes.data_as(u64p),
                                              len(key_off) - 1)

    def next_block(self) -> bytes | None:
        d = u8p()
        n = C.c_size_t()
        if not lib().or_sst_builder_next_block(self._h, C.byref(d), C.byref(n)):
            return None
        return C.string_at(d, n.value)

    def build(self) -> int:
        return lib().or_sst_builder_build(self._h)

    def chunks(self) -> list[bytes]:
        out = []
        for i in range(lib().or_sst_table_num_chunks(self._h)):
            d = u8p()
            n = C.c_size_t()
            lib().or_sst_table_chunk(self._h, i, C.byref(d), C.byref(n))
            out.append(C.string_at(d, n.value))
        return out

    def encode_table(self) -> bytes:
        n = lib().or_sst_table_encoded_len(self._h)
        out = np.zeros(max(n, 1), np.uint8)
        assert lib().or_sst_table_encode(self._h, out.ctypes.data_as(u8p), out.size) == 0
        return out[:n].tobytes()

    def info(self) -> dict:
        info = SstInfo()
        fk = np.zeros(1 << 16, np.uint8)
        assert lib().or_sst_table_info(self._h, C.byref(info), fk.ctypes.data_as(u8p), fk.size) == 0
        d = {f: getattr(info, f) for f, _ in SstInfo._fields_}
        d["first_key"] = fk[: info.first_key_len].tobytes()
        return d

    def bloom(self):
        present = C.c_int()
        np_ = C.c_uint16()
        bl = C.c_size_t()
        cap = 1 << 26
        out = np.zeros(cap, np.uint8)
        assert lib().or_sst_table_bloom(self._h, C.byref(present), C.byref(np_), out.ctypes.data_as(u8p), cap,
                                        C.byref(bl)) == 0
        if not present.value:
            return None
        return np_.value, out[:bl.value].tobytes()


def sst_read_info(sst: bytes) -> tuple[int, dict]:
    h, p = _buf(sst)
    info = SstInfo()
    fk = np.zeros(max(len(sst), 1), np.uint8)
    st = lib().or_sst_read_info(p, len(sst), C.byref(info), fk.ctypes.data_as(u8p), fk.size)
    d = {f: getattr(info, f) for f, _ in SstInfo._fields_}
    d["first_key"] = fk[: info.first_key_len].tobytes()
    return st, d


def merge_arrays(keys: np.ndarray, key_off: np.ndarray, src_start: np.ndarray) -> np.ndarray:
    """iter.MergeSort (merge.go:12-111) over k concatenated sorted iterators: element indices
    of the entries Next() returns, in order (u32)."""
    keys = np.ascontiguousarray(keys, np.uint8) if len(keys) else np.zeros(1, np.uint8)
    key_off = np.ascontiguousarray(key_off, np.uint64)
    src_start = np.ascontiguousarray(src_start, np.uint64)
    k = len(src_start) - 1
    out = np.zeros(max(int(src_start[-1]), 1), np.uint32)
    n = C.c_uint64(0)
    st = lib().or_merge_sort(k, keys.ctypes.data_as(u8p), key_off.ctypes.data_as(u64p),
                             src_start.ctypes.data_as(u64p), out.ctypes.data_as(u32p), C.byref(n))
    assert st == 0, st
    return out[: n.value]


def merge_sort(sources: list[list[bytes]]) -> np.ndarray:
    """merge_arrays over a list of per-iterator key lists."""
    flat = [k for s in sources for k in s]
    kd, ko = _arena(flat)
    ss = np.zeros(len(sources) + 1, np.uint64)
    ss[1:] = np.cumsum([len(s) for s in sources])
    return merge_arrays(kd, ko, ss)


def compact_arrays(blob: np.ndarray, sst_off: np.ndarray, src_sst: np.ndarray, max_sst_size: int, codec: int = NONE,
                   nthreads: int = 1, block_size: int = 4096) -> tuple[int, np.ndarray, np.ndarray]:
    """executeCompaction over SSTs packed in one array (compact_oracle.c or_compact): -> (status,
    outputs packed, out_off)."""
    blob = np.ascontiguousarray(blob, np.uint8)
    sst_off = np.ascontiguousarray(sst_off, np.uint64)
    src_sst = np.ascontiguousarray(src_sst, np.uint32)
    cap = int(blob.size) * 2 + (1 << 20)
    out = np.empty(cap, np.uint8)
    oo_cap = int(blob.size) // 64 + 64
    out_off = np.zeros(oo_cap, np.uint64)
    n_out = C.c_uint32(0)
    st = lib().or_compact(blob.ctypes.data_as(u8p), sst_off.ctypes.data_as(u64p), len(sst_off) - 1,
                          src_sst.ctypes.data_as(u32p), len(src_sst) - 1, block_size, codec, max_sst_size, nthreads,
                          out.ctypes.data_as(u8p), cap, out_off.ctypes.data_as(u64p), oo_cap, C.byref(n_out))
    n = n_out.value
    return st, out[: int(out_off[n]) if n else 0], out_off[: n + 1]


def compact(sources: list[list[bytes]], max_sst_size: int, codec: int = NONE, nthreads: int = 1,
            block_size: int = 4096) -> list[bytes]:
    """compact_arrays over sources of SSTs (lists of bytes): the output SSTs' bytes."""
    ssts = [s for run in sources for s in run]
    blob = np.frombuffer(b"".join(ssts) or b"\0", np.uint8)
    sst_off = np.zeros(len(ssts) + 1, np.uint64)
    sst_off[1:] = np.cumsum([len(s) for s in ssts])
    src_sst = np.zeros(len(sources) + 1, np.uint32)
    src_sst[1:] = np.cumsum([len(r) for r in sources])
    st, out, off = compact_arrays(blob, sst_off, src_sst, max_sst_size, codec, nthreads, block_size)
    assert st == 0, status_string(st)
    return [out[int(off[i]):int(off[i + 1])].tobytes() for i in range(len(off) - 1)]
