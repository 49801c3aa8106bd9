"""Python binding of libslatecodec.so (the MI355X SST block codec C-ABI).

Thin ctypes plumbing for tests and bench.py.  The product is the C-ABI library
declared in include/slatecodec.h; this module only marshals buffers.  It never
falls back to a CPU implementation: if the HIP library or a GPU is missing,
calls raise SlateError.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)  # slatedb-go_amd/
LIB_PATH = os.path.join(ROOT, "lib", os.environ.get("SLATE_LIB_VARIANT", "libslatecodec.so"))  # variant: profiling only
HEADER = os.path.join(os.path.dirname(ROOT), "include", "slatecodec.h")

NONE, SNAPPY, ZLIB, LZ4, ZSTD = 0, 1, 2, 3, 4
OK = 0
E_NO_DEVICE = 100
E_CAPACITY = 103
E_INVALID_ARG = 102
E_MERGE_UNSORTED = 105
E_LIMIT = 106
E_WARNINGS = 107
E_READER_NEED_DATA, E_READER_END = 108, 109

u8p = C.POINTER(C.c_uint8)
u16p = C.POINTER(C.c_uint16)
u64p = C.POINTER(C.c_uint64)
szp = C.POINTER(C.c_size_t)
vp = C.c_void_p

SEEK_WARN_DTYPE = np.dtype([("kind", "<u2"), ("err", "<i2"), ("a", "<u4"), ("b", "<u4"), ("reserved", "<u4")])
SEEK_DTYPE = np.dtype([("start", "<u4"), ("first_idx", "<i4"), ("n_warn", "<u4"), ("status", "<i2"),
                       ("first_len", "<u2")])
META_DTYPE = np.dtype([("status", "<i2"), ("flags", "<u2"), ("detail", "<i4"), ("data_len", "<u4"),
                       ("n_rows", "<u2"), ("aux", "<u2")])
ROW_DTYPE = np.dtype([("row_off", "<u4"), ("key_prefix_len", "<u2"), ("key_suffix_len", "<u2"),
                      ("value_len", "<u4"), ("flags", "u1"), ("meta_len", "u1"), ("status", "<i2")])


class SstConfig(C.Structure):
    _fields_ = [("block_size", C.c_uint64), ("min_filter_keys", C.c_uint32),
                ("filter_bits_per_key", C.c_uint32), ("codec", C.c_int32)]


class SstInfo(C.Structure):
    _fields_ = [("index_offset", C.c_uint64), ("index_len", C.c_uint64), ("filter_offset", C.c_uint64),
                ("filter_len", C.c_uint64), ("codec", C.c_int32), ("first_key_len", C.c_uint32)]


class BlockView(C.Structure):
    _fields_ = [("block", C.c_uint64), ("meta", C.c_uint8 * 16), ("data", C.c_void_p), ("rows", C.c_void_p)]


class SlateError(RuntimeError):
    def __init__(self, status: int, where: str = ""):
        self.status = status
        super().__init__(f"{where}: {status_string(status)} (status {status})")


def build(verbose: bool = False) -> str:
    """Compile the HIP library for gfx950 (hipcc cross-compiles without a GPU)."""
    jobs = str(min(16, os.cpu_count() or 4))
    subprocess.run(["make", "-s", "-j", jobs, "-C", ROOT], check=True,
                   stdout=None if verbose else subprocess.DEVNULL)
    return LIB_PATH


_SIGS = {
    "slate_abi_version": (C.c_int, []),
    "slate_status_string": (C.c_char_p, [C.c_int]),
    "slate_ctx_create": (vp, [C.c_int, C.POINTER(C.c_int)]),
    "slate_ctx_destroy": (None, [vp]),
    "slate_ctx_set_stream": (C.c_int, [vp, vp]),
    "slate_ctx_set_copy_threads": (C.c_int, [vp, C.c_uint32]),
    "slate_ctx_set_timing": (C.c_int, [vp, C.c_int]),
    "slate_ctx_gpu_time": (C.c_int, [vp, C.POINTER(C.c_double), C.c_int]),
    "slate_ctx_handbacks": (C.c_int, [vp, C.POINTER(C.c_uint64), C.c_int]),
    "slate_ctx_gpu_busy": (C.c_int, [vp, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int]),
    "slate_ctx_synchronize": (C.c_int, [vp]),
    "slate_decode_scratch_bytes": (C.c_size_t, [C.c_uint32]),
    "slate_decode_scratch_bytes_codec": (C.c_size_t, [C.c_uint32, C.c_int]),
    "slate_block_decode_plan_device": (C.c_int, [vp, C.c_int, vp, vp, C.c_uint32, vp, vp, vp]),
    "slate_block_decode_device": (C.c_int, [vp, C.c_int, vp, vp, C.c_uint32, vp, vp, vp, vp, vp]),
    "slate_block_decode_batch": (C.c_int, [vp, C.c_int, vp, vp, C.c_uint32, vp, C.c_uint64, vp, vp, vp,
                                           C.c_uint64, vp]),
    "slate_block_decode": (C.c_int, [vp, C.c_int, vp, C.c_size_t, vp, C.c_size_t, szp, vp, vp, C.c_size_t]),
    "slate_shard_blocks": (C.c_uint32, [C.c_uint32, C.c_uint32, C.c_uint32]),
    "slate_block_seek_device": (C.c_int, [vp, vp, vp, vp, vp, vp, vp, C.c_uint64, vp]),
    "slate_block_seek": (C.c_int, [vp, vp, vp, vp, C.c_uint32, vp, vp, vp, C.c_uint64, vp]),
    "slate_index_seek": (C.c_int, [vp, vp, vp, vp, C.c_uint64, vp]),
    "slate_devbuf_alloc": (vp, [vp, C.c_uint64, C.POINTER(C.c_int)]),
    "slate_devbuf_free": (None, [vp]),
    "slate_devbuf_ptr": (vp, [vp]),
    "slate_devbuf_size": (C.c_uint64, [vp]),
    "slate_devbuf_upload": (C.c_int, [vp, vp, C.c_uint64, vp, C.c_uint64]),
    "slate_devbuf_download": (C.c_int, [vp, vp, vp, C.c_uint64, C.c_uint64]),
    "slate_devbuf_copy": (C.c_int, [vp, vp, C.c_uint64, vp, C.c_uint64, C.c_uint64]),
    "slate_devbuf_memset": (C.c_int, [vp, vp, C.c_uint64, C.c_int, C.c_uint64]),
    "slate_hostbuf_alloc": (vp, [vp, C.c_uint64, C.POINTER(C.c_int)]),
    "slate_hostbuf_free": (None, [vp]),
    "slate_hostbuf_ptr": (vp, [vp]),
    "slate_hostbuf_size": (C.c_uint64, [vp]),
    "slate_devbuf_upload_async": (C.c_int, [vp, vp, C.c_uint64, vp, C.c_uint64, C.c_uint64]),
    "slate_devbuf_download_async": (C.c_int, [vp, vp, C.c_uint64, vp, C.c_uint64, C.c_uint64]),
    "slate_compact": (C.c_int, [vp, vp, vp, C.c_uint32, vp, C.c_uint32, C.POINTER(SstConfig), C.c_uint64, vp,
                                C.c_uint32, C.POINTER(C.c_uint32)]),
    "slate_crc32_device": (C.c_int, [vp, vp, C.c_size_t, C.POINTER(C.c_uint32)]),
    "slate_compact_ex": (C.c_int, [vp, vp, vp, C.c_uint32, vp, C.c_uint32, C.POINTER(SstConfig), C.c_uint64, vp,
                                   C.c_uint32, C.POINTER(C.c_uint32), vp, C.c_uint32, C.POINTER(C.c_uint32)]),
    "slate_block_seek_warn_device": (C.c_int, [vp, vp, vp, vp, vp, vp, vp, C.c_uint64, vp, vp, C.c_uint32]),
    "slate_block_seek_warn": (C.c_int, [vp, vp, vp, vp, C.c_uint32, vp, vp, vp, C.c_uint64, vp, vp, C.c_uint32]),
    "slate_shard_pack": (C.c_int, [vp, vp, C.c_uint32, C.c_uint32, C.c_uint32, vp, C.c_uint64, vp]),
    "slate_block_decode_sharded": (C.c_int, [vp, C.c_uint32, C.c_int, vp, vp, C.c_uint32, vp, C.c_uint64, vp, vp,
                                             vp, C.c_uint64, vp]),
    "slate_block_encode": (C.c_int, [vp, C.c_int, vp, C.c_size_t, vp, C.c_size_t, vp, C.c_size_t, szp]),
    "slate_sst_builder_new": (vp, [vp, C.POINTER(SstConfig), C.POINTER(C.c_int)]),
    "slate_sst_builder_free": (None, [vp]),
    "slate_sst_builder_add": (C.c_int, [vp, vp, C.c_size_t, vp, C.c_size_t, C.c_int]),
    "slate_sst_builder_add_value": (C.c_int, [vp, vp, C.c_size_t, vp, C.c_size_t]),
    "slate_sst_builder_add_batch": (C.c_int, [vp, vp, vp, vp, vp, vp, C.c_uint64]),
    "slate_sst_builder_add_batch_device": (C.c_int, [vp, vp, vp, vp, vp, vp, C.c_uint64]),
    "slate_sst_builder_next_block": (C.c_int, [vp, vp, C.c_size_t, szp, C.POINTER(C.c_int)]),
    "slate_sst_builder_build": (C.c_int, [vp, C.POINTER(vp)]),
    "slate_sst_table_free": (None, [vp]),
    "slate_sst_table_info": (C.c_int, [vp, C.POINTER(SstInfo), vp, C.c_size_t]),
    "slate_sst_table_num_chunks": (C.c_size_t, [vp]),
    "slate_sst_table_chunk": (C.c_int, [vp, C.c_size_t, C.POINTER(vp), szp]),
    "slate_sst_table_encoded_len": (C.c_size_t, [vp]),
    "slate_sst_table_encode": (C.c_int, [vp, vp, C.c_size_t]),
    "slate_sst_table_bloom": (C.c_int, [vp, C.POINTER(C.c_int), u16p, vp, C.c_size_t, szp]),
    "slate_sst_read_info": (C.c_int, [vp, C.c_size_t, C.POINTER(SstInfo), vp, C.c_size_t]),
    "slate_decode_info": (C.c_int, [vp, C.c_size_t, C.POINTER(SstInfo), vp, C.c_size_t]),
    "slate_encode_info": (C.c_int, [C.POINTER(SstInfo), vp, vp, C.c_size_t, szp]),
    "slate_decode_index": (C.c_int, [vp, vp, C.c_size_t, C.c_int, C.POINTER(vp)]),
    "slate_index_free": (None, [vp]),
    "slate_index_num_blocks": (C.c_size_t, [vp]),
    "slate_index_block_meta": (C.c_int, [vp, C.c_size_t, u64p, C.POINTER(vp), szp]),
    "slate_read_blocks_range": (C.c_int, [C.POINTER(SstInfo), vp, C.c_uint64, C.c_uint64, u64p, u64p]),
    "slate_read_blocks": (C.c_int, [vp, C.POINTER(SstInfo), vp, C.c_uint64, C.c_uint64, vp, C.c_size_t, vp,
                                    C.c_uint64, vp, vp, vp, C.c_uint64, vp, u64p]),
    "slate_block_reader_create": (C.c_int, [vp, C.POINTER(SstInfo), vp, C.c_uint64, C.c_uint32, C.POINTER(vp)]),
    "slate_block_reader_free": (None, [vp]),
    "slate_block_reader_next": (C.c_int, [vp, C.POINTER(BlockView)]),
    "slate_block_reader_want": (C.c_int, [vp, u64p, u64p]),
    "slate_block_reader_feed": (C.c_int, [vp, vp, C.c_size_t]),
    "slate_bloom_build": (C.c_int, [vp, vp, vp, C.c_uint64, C.c_uint32, vp, C.c_size_t, szp, u16p]),
    "slate_bloom_encode": (C.c_int, [vp, C.c_uint16, vp, C.c_size_t, C.c_int, vp, C.c_size_t, szp]),
    "slate_bloom_decode": (C.c_int, [vp, vp, C.c_size_t, C.c_int, u16p, vp, C.c_size_t, szp]),
    "slate_bloom_has_keys": (C.c_int, [vp, C.c_uint16, vp, C.c_size_t, vp, vp, C.c_uint64, vp]),
    "slate_merge_sorted": (C.c_int, [vp, C.c_uint32, vp, vp, vp, vp, u64p]),
    "slate_merge_scratch_bytes": (C.c_size_t, [C.c_uint64, C.c_uint32]),
    "slate_merge_sorted_device": (C.c_int, [vp, C.c_uint32, vp, vp, vp, vp, vp, vp, vp]),
    "slate_kv_scratch_bytes": (C.c_size_t, [C.c_uint64]),
    "slate_index_block_offsets": (C.c_int, [vp, vp, C.c_size_t]),
    "slate_rows_kv_lengths_device": (C.c_int, [vp, C.c_uint32, vp, vp, vp, C.c_uint64, vp, vp, vp, vp, vp, vp]),
    "slate_rows_kv_copy_device": (C.c_int, [vp, C.c_uint32, vp, vp, vp, vp, C.c_uint64, vp, vp, vp, vp, vp, vp]),
    "slate_kv_gather_lengths_device": (C.c_int, [vp, vp, C.c_uint64, vp, vp, vp, vp, vp, vp, vp]),
    "slate_kv_gather_copy_device": (C.c_int, [vp, vp, C.c_uint64, vp, vp, vp, vp, vp, vp, vp, vp]),
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise SlateError(E_NO_DEVICE, f"{LIB_PATH} missing (run __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        variant = bool(os.environ.get("SLATE_LIB_VARIANT"))
        for name, (res, args) in _SIGS.items():
            if variant and not hasattr(L, name):  # an older library in an A/B run: entry points it predates
                continue
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def status_string(code: int) -> str:
    try:
        return lib().slate_status_string(code).decode()
    except Exception:  # library missing
        return f"status {code}"


def _ptr(a: np.ndarray):
    return C.c_void_p(a.ctypes.data) if a is not None and a.size else None


def _check(st: int, where: str):
    if st != OK:
        raise SlateError(st, where)


class Context:
    """slate_ctx: one device + one HIP stream."""

    def __init__(self, device: int = 0):
        st = C.c_int()
        self._h = lib().slate_ctx_create(device, C.byref(st))
        if not self._h:
            raise SlateError(st.value, "slate_ctx_create")
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            lib().slate_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except (TypeError, AttributeError):  # interpreter shutdown: module globals already gone
            pass

    @property
    def handle(self):
        return self._h

    def set_stream(self, stream_handle: int | None):
        _check(lib().slate_ctx_set_stream(self._h, C.c_void_p(stream_handle) if stream_handle else None),
               "slate_ctx_set_stream")

    def set_copy_threads(self, threads: int):
        """Host copy threads of this context (slate_ctx_set_copy_threads)."""
        _check(lib().slate_ctx_set_copy_threads(self._h, int(threads)), "slate_ctx_set_copy_threads")


    def set_timing(self, on: bool) -> None:
        """Sum the SST builder's GPU pass times on this context (slate_ctx_set_timing)."""
        _check(lib().slate_ctx_set_timing(self._h, 1 if on else 0), "slate_ctx_set_timing")

    def handbacks(self, reset: bool = False) -> int:
        """slate_ctx_handbacks: blocks the fast paths handed to the exact decoder since the last reset."""
        v = C.c_uint64()
        _check(lib().slate_ctx_handbacks(self._h, C.byref(v), 1 if reset else 0), "slate_ctx_handbacks")
        return v.value

    def gpu_time_ms(self, reset: bool = False) -> float:
        v = C.c_double()
        _check(lib().slate_ctx_gpu_time(self._h, C.byref(v), 1 if reset else 0), "slate_ctx_gpu_time")
        return v.value

    def gpu_busy_ms(self, reset: bool = False) -> tuple:
        """(union, sum) of the timed spans in ms (slate_ctx_gpu_busy)."""
        u, t = C.c_double(), C.c_double()
        _check(lib().slate_ctx_gpu_busy(self._h, C.byref(u), C.byref(t), 1 if reset else 0), "slate_ctx_gpu_busy")
        return u.value, t.value
    def synchronize(self):
        _check(lib().slate_ctx_synchronize(self._h), "slate_ctx_synchronize")

    # ------------------------------------------------------------ decode
    def decode_batch(self, codec: int, blob: np.ndarray, in_off: np.ndarray):
        """block.Decode over a batch of host blocks -> (out, out_off, meta, rows, row_base)."""
        blob = np.ascontiguousarray(blob, dtype=np.uint8)
        in_off = np.ascontiguousarray(in_off, dtype=np.uint64)
        n = len(in_off) - 1
        out_off = np.zeros(n + 1, np.uint64)
        row_base = np.zeros(n + 1, np.uint64)
        meta = np.zeros(max(n, 1), META_DTYPE)
        L = lib()
        st = L.slate_block_decode_batch(self._h, codec, _ptr(blob), _ptr(in_off), n, None, 0, _ptr(out_off),
                                        _ptr(meta), None, 0, _ptr(row_base))
        if st not in (OK, E_CAPACITY):
            raise SlateError(st, "slate_block_decode_batch")
        out = np.zeros(max(int(out_off[n]), 1), np.uint8)
        rows = np.zeros(max(int(row_base[n]), 1), ROW_DTYPE)
        st = L.slate_block_decode_batch(self._h, codec, _ptr(blob), _ptr(in_off), n, _ptr(out), out.size,
                                        _ptr(out_off), _ptr(meta), _ptr(rows), rows.size, _ptr(row_base))
        _check(st, "slate_block_decode_batch")
        return out, out_off, meta[:n], rows, row_base

    def decode_batch_into(self, codec: int, blob: np.ndarray, in_off: np.ndarray, out: np.ndarray,
                          rows: np.ndarray, meta: np.ndarray, out_off: np.ndarray, row_base: np.ndarray) -> int:
        """slate_block_decode_batch into caller-sized buffers (one pass; a caller that knows
        capacity bounds, as an object-store reader does).  Returns the status."""
        n = len(in_off) - 1
        return lib().slate_block_decode_batch(self._h, codec, _ptr(blob), _ptr(in_off), n, _ptr(out), out.size,
                                              _ptr(out_off), _ptr(meta), _ptr(rows), rows.size, _ptr(row_base))

    def block_seek(self, out: np.ndarray, out_off: np.ndarray, meta: np.ndarray, qblock: list[int],
                   keys: list[bytes]) -> np.ndarray:
        """block.NewIteratorAtKey for (block, key) queries over a decode_batch result -> SEEK_DTYPE."""
        kd, ko = _arena(keys)
        qb = np.ascontiguousarray(qblock, np.uint32)
        res = np.zeros(max(len(keys), 1), SEEK_DTYPE)
        out = np.ascontiguousarray(out, np.uint8)
        _check(lib().slate_block_seek(self._h, _ptr(out), _ptr(np.ascontiguousarray(out_off, np.uint64)),
                                      _ptr(np.ascontiguousarray(meta)), len(out_off) - 1, _ptr(qb), _ptr(kd), _ptr(ko),
                                      len(keys), _ptr(res)), "slate_block_seek")
        return res[: len(keys)]

    def block_seek_warn(self, out: np.ndarray, out_off: np.ndarray, meta: np.ndarray, qblock: list[int],
                        keys: list[bytes], warn_cap: int = 16):
        """block_seek plus each query's warnings: (SEEK_DTYPE[n], SEEK_WARN_DTYPE[n, warn_cap])."""
        kd, ko = _arena(keys)
        qb = np.ascontiguousarray(qblock, np.uint32)
        res = np.zeros(max(len(keys), 1), SEEK_DTYPE)
        warn = np.zeros((max(len(keys), 1), max(warn_cap, 1)), SEEK_WARN_DTYPE)
        out = np.ascontiguousarray(out, np.uint8)
        _check(lib().slate_block_seek_warn(self._h, _ptr(out), _ptr(np.ascontiguousarray(out_off, np.uint64)),
                                           _ptr(np.ascontiguousarray(meta)), len(out_off) - 1, _ptr(qb), _ptr(kd),
                                           _ptr(ko), len(keys), _ptr(res), _ptr(warn), warn_cap),
               "slate_block_seek_warn")
        return res[: len(keys)], warn[: len(keys), :warn_cap]

    def block_seek_device(self, d_data: int, d_out_off: int, d_meta: int, d_qblock: int, d_keys: int, d_key_off: int,
                          n: int, d_res: int) -> None:
        _check(lib().slate_block_seek_device(self._h, d_data, d_out_off, d_meta, d_qblock, d_keys, d_key_off, n, d_res),
               "slate_block_seek_device")

    def index_seek(self, index: "Index", keys: list[bytes]) -> np.ndarray:
        """sstable.Iterator.firstBlockIncludingOrAfterKey for each key (u64 block indexes)."""
        kd, ko = _arena(keys)
        out = np.zeros(max(len(keys), 1), np.uint64)
        _check(lib().slate_index_seek(self._h, index.handle, _ptr(kd), _ptr(ko), len(keys), _ptr(out)),
               "slate_index_seek")
        return out[: len(keys)]

    def block_decode(self, encoded: bytes, codec: int):
        """block.Decode(&b, input, codec) -> (status, meta, Data, Offsets)."""
        a = np.frombuffer(bytes(encoded) or b"\0", dtype=np.uint8)
        cap = max(len(encoded) * 24, 64)
        out = np.empty(cap, np.uint8)
        offs = np.empty(cap // 2 + 1, np.uint16)
        meta = np.zeros(1, META_DTYPE)
        ol = C.c_size_t()
        st = lib().slate_block_decode(self._h, codec, _ptr(a), len(encoded), _ptr(out), cap, C.byref(ol),
                                      _ptr(meta), _ptr(offs), offs.size)
        m = meta[0]
        if st != OK:
            return st, m, b"", []
        return st, m, out[: m["data_len"]].tobytes(), offs[: m["n_rows"]].tolist()

    def decode_plan_device(self, codec: int, d_in: int, d_in_off: int, n: int, d_out_off: int, d_row_base: int,
                           d_scratch: int):
        _check(lib().slate_block_decode_plan_device(self._h, codec, d_in, d_in_off, n, d_out_off, d_row_base,
                                                    d_scratch), "slate_block_decode_plan_device")

    def decode_device(self, codec: int, d_in: int, d_in_off: int, n: int, d_out: int, d_out_off: int, d_meta: int,
                      d_rows: int, d_row_base: int):
        _check(lib().slate_block_decode_device(self._h, codec, d_in, d_in_off, n, d_out, d_out_off, d_meta, d_rows,
                                               d_row_base), "slate_block_decode_device")


    # ------------------------------------------------------------ encode / SST
    def block_encode(self, data: bytes, offsets: list[int], codec: int) -> tuple[int, bytes]:
        d = np.frombuffer(bytes(data) or b"\0", dtype=np.uint8)
        o = np.array(offsets or [0], dtype=np.uint16)
        cap = len(data) * 2 + 2 * len(offsets) + 64
        out = np.zeros(cap, np.uint8)
        ol = C.c_size_t()
        st = lib().slate_block_encode(self._h, codec, _ptr(d), len(data), _ptr(o), len(offsets), _ptr(out), cap,
                                      C.byref(ol))
        return st, (out[: ol.value].tobytes() if st == OK else b"")

    def bloom_build(self, keys: list[bytes], bits_per_key: int) -> tuple[int, bytes]:
        kd, ko = _arena(keys)
        cap = max(((len(keys) * bits_per_key) & 0xFFFFFFFF) // 8 + 8, 8)
        out = np.zeros(cap, np.uint8)
        bl = C.c_size_t()
        npr = C.c_uint16()
        _check(lib().slate_bloom_build(self._h, _ptr(kd), _ptr(ko), len(keys), bits_per_key, _ptr(out), cap,
                                       C.byref(bl), C.byref(npr)), "slate_bloom_build")
        return npr.value, out[: bl.value].tobytes()

    def merge_arrays(self, keys: np.ndarray, key_off: np.ndarray, src_start: np.ndarray) -> np.ndarray:
        """iter.MergeSort (merge.go:12-111) over k concatenated sorted iterators: the element
        indices of the entries Next() returns, in order (u32).  Raises SlateError
        (E_MERGE_UNSORTED) for an unsorted iterator."""
        keys = np.ascontiguousarray(keys, np.uint8) if len(keys) else np.zeros(1, np.uint8)
        key_off = np.ascontiguousarray(key_off, np.uint64)
        src_start = np.ascontiguousarray(src_start, np.uint64)
        out = np.zeros(max(int(src_start[-1]), 1), np.uint32)
        n = C.c_uint64()
        _check(lib().slate_merge_sorted(self._h, len(src_start) - 1, _ptr(keys), _ptr(key_off), _ptr(src_start),
                                        _ptr(out), C.byref(n)), "slate_merge_sorted")
        return out[: n.value]

    def merge_sort(self, sources: list[list[bytes]]) -> np.ndarray:
        """merge_arrays over per-iterator key lists."""
        kd, ko = _arena([k for s in sources for k in s])
        ss = np.zeros(len(sources) + 1, np.uint64)
        ss[1:] = np.cumsum([len(s) for s in sources])
        return self.merge_arrays(kd, ko, ss)

    def merge_device(self, d_keys: int, d_key_off: int, src_start: np.ndarray, d_out_idx: int, d_n_out: int,
                     d_flags: int, d_scratch: int) -> None:
        src_start = np.ascontiguousarray(src_start, np.uint64)
        _check(lib().slate_merge_sorted_device(self._h, len(src_start) - 1, d_keys, d_key_off, _ptr(src_start),
                                               d_out_idx, d_n_out, d_flags, d_scratch), "slate_merge_sorted_device")

    def bloom_has_keys(self, num_probes: int, bits: bytes, keys: list[bytes]) -> list[bool]:
        kd, ko = _arena(keys)
        b = np.frombuffer(bytes(bits) or b"\0", dtype=np.uint8)
        out = np.zeros(max(len(keys), 1), np.uint8)
        _check(lib().slate_bloom_has_keys(self._h, num_probes, _ptr(b), len(bits), _ptr(kd), _ptr(ko), len(keys),
                                          _ptr(out)), "slate_bloom_has_keys")
        return [bool(x) for x in out[: len(keys)]]

    def bloom_encode(self, num_probes: int, bits: bytes, codec: int) -> tuple[int, bytes]:
        b = np.frombuffer(bytes(bits) or b"\0", dtype=np.uint8)
        cap = len(bits) + 64
        out = np.zeros(cap, np.uint8)
        ol = C.c_size_t()
        st = lib().slate_bloom_encode(self._h, num_probes, _ptr(b), len(bits), codec, _ptr(out), cap, C.byref(ol))
        return st, (out[: ol.value].tobytes() if st == OK else b"")

    def bloom_decode(self, buf: bytes, codec: int) -> tuple[int, int, bytes]:
        b = np.frombuffer(bytes(buf) or b"\0", dtype=np.uint8)
        cap = len(buf) + 64
        if codec == SNAPPY:  # the decoded length is the payload's varint header
            x, sh = 0, 0
            for byte in bytes(buf[:10]):
                x |= (byte & 0x7F) << sh
                sh += 7
                if byte < 0x80:
                    break
            cap = max(cap, min(x, 1 << 32) + 64)
        elif codec != NONE:  # no size header: room for 4x, so a typical filter decodes in one call
            cap = 4 * len(buf) + 65536
        out = np.zeros(cap, np.uint8)
        npr = C.c_uint16()
        bl = C.c_size_t()
        st = lib().slate_bloom_decode(self._h, _ptr(b), len(buf), codec, C.byref(npr), _ptr(out), cap, C.byref(bl))
        if st == E_CAPACITY:  # compressed filter: bits_len holds the decoded size
            cap = bl.value + 16
            out = np.zeros(cap, np.uint8)
            st = lib().slate_bloom_decode(self._h, _ptr(b), len(buf), codec, C.byref(npr), _ptr(out), cap, C.byref(bl))
        return st, npr.value, (out[: bl.value].tobytes() if st == OK else b"")

    def decode_index(self, buf: bytes, codec: int):
        b = np.frombuffer(bytes(buf) or b"\0", dtype=np.uint8)
        h = C.c_void_p()
        st = lib().slate_decode_index(self._h, _ptr(b), len(buf), codec, C.byref(h))
        if st != OK:
            return st, None
        return st, Index(h)

    def iter_blocks(self, info: "SstInfo", index: "Index", sst: bytes, first: int = 0, read_ahead: int = 64):
        """sstable.Iterator's block walk through slate_block_reader (read-ahead batches): a list of
        (block, status, meta, data bytes incl. offsets, rows) in order; a failing block comes last."""
        return reader_walk(self, info, index, sst, first, read_ahead)[0]

    def read_blocks(self, info: "SstInfo", index: "Index", start: int, end: int, sst: bytes):
        """ReadBlocks over the object bytes: returns (status, failed_block, decode outputs)."""
        rs, re_ = C.c_uint64(), C.c_uint64()
        st = lib().slate_read_blocks_range(C.byref(info), index.handle, start, end, C.byref(rs), C.byref(re_))
        if st != OK:
            return st, None, None
        data = np.frombuffer(sst[rs.value:re_.value] or b"\0", dtype=np.uint8)
        n = end - start
        out_cap = (re_.value - rs.value) * 24 + 64
        out = np.zeros(out_cap, np.uint8)
        out_off = np.zeros(n + 1, np.uint64)
        row_base = np.zeros(n + 1, np.uint64)
        meta = np.zeros(n, META_DTYPE)
        rows = np.zeros(out_cap // 15 + 8, ROW_DTYPE)
        failed = C.c_uint64()
        st = lib().slate_read_blocks(self._h, C.byref(info), index.handle, start, end, _ptr(data),
                                     re_.value - rs.value, _ptr(out), out_cap, _ptr(out_off), _ptr(meta), _ptr(rows),
                                     rows.size, _ptr(row_base), C.byref(failed))
        return st, failed.value, (out, out_off, meta, rows, row_base)


class DevBuf:
    """slate_devbuf: HBM owned by the library (the device-resident entry points take .ptr)."""

    def __init__(self, ctx: "Context", nbytes: int):
        st = C.c_int()
        self._h = lib().slate_devbuf_alloc(ctx.handle, int(nbytes), C.byref(st))
        if not self._h:
            raise SlateError(st.value, "slate_devbuf_alloc")
        self.ctx = ctx
        self.size = int(nbytes)
        self.ptr = int(lib().slate_devbuf_ptr(self._h))

    @property
    def handle(self):
        return self._h

    def at(self, off: int) -> int:
        """Device address of byte `off` (what a cgo caller computes from slate_devbuf_ptr)."""
        assert 0 <= off <= self.size
        return self.ptr + off

    def upload(self, a, off: int = 0) -> "DevBuf":
        a = np.ascontiguousarray(a)
        _check(lib().slate_devbuf_upload(self.ctx.handle, self._h, off, _ptr(a), a.nbytes), "slate_devbuf_upload")
        return self

    def download(self, nbytes: int | None = None, off: int = 0, dtype=np.uint8) -> np.ndarray:
        n = self.size - off if nbytes is None else int(nbytes)
        out = np.zeros(max(n, 1), np.uint8)
        _check(lib().slate_devbuf_download(self.ctx.handle, _ptr(out), self._h, off, n), "slate_devbuf_download")
        return out[:n].view(dtype)

    def u64(self, index: int) -> int:
        return int(self.download(8, 8 * index, np.uint64)[0])

    def memset(self, value: int = 0, off: int = 0, nbytes: int | None = None) -> "DevBuf":
        n = self.size - off if nbytes is None else int(nbytes)
        _check(lib().slate_devbuf_memset(self.ctx.handle, self._h, off, value, n), "slate_devbuf_memset")
        return self

    def free(self):
        if getattr(self, "_h", None):
            lib().slate_devbuf_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except (TypeError, AttributeError):
            pass


def devbuf_from(ctx: "Context", a) -> DevBuf:
    """A DevBuf holding a copy of host array a."""
    a = np.ascontiguousarray(a)
    return DevBuf(ctx, a.nbytes).upload(a)


class HostBuf:
    """slate_hostbuf: page-locked host memory owned by the library (async copy endpoint)."""

    def __init__(self, ctx: "Context", nbytes: int):
        st = C.c_int()
        self._h = lib().slate_hostbuf_alloc(ctx.handle, int(nbytes), C.byref(st))
        if not self._h:
            raise SlateError(st.value, "slate_hostbuf_alloc")
        self.size = int(nbytes)
        self.view = np.ctypeslib.as_array(C.cast(lib().slate_hostbuf_ptr(self._h), u8p), shape=(max(self.size, 1),))

    @property
    def handle(self):
        return self._h

    def free(self):
        if getattr(self, "_h", None):
            self.view = None
            lib().slate_hostbuf_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except (TypeError, AttributeError):
            pass


# slate_compact_warning (include/slatecodec.h): one types.ErrWarn entry of a compaction
COMPACT_WARN_DTYPE = np.dtype([("src", "<u4"), ("sst", "<u4"), ("block", "<u4"), ("row", "<i4"), ("status", "<i4"),
                               ("block_len", "<u4")])


def compact_ex(ctx: "Context", sources: list[list[bytes]], max_sst_size: int, block_size: int = 4096,
               min_filter_keys: int = 0, filter_bits_per_key: int = 10, codec: int = NONE):
    """slate_compact_ex -> (encoded output SSTs, warning records in ErrWarn order): corrupt input
    blocks / rows end their SST / block iterators as Go's do and the compaction goes on."""
    flat = [s for run in sources for s in run]
    blob = np.frombuffer(b"".join(flat) or b"\0", np.uint8)
    off = np.concatenate([[0], np.cumsum([len(s) for s in flat])]).astype(np.uint64)
    src = np.concatenate([[0], np.cumsum([len(r) for r in sources])]).astype(np.uint32)
    cfg = SstConfig(block_size, min_filter_keys, filter_bits_per_key, codec)
    cap, wcap = 16, 16
    while True:
        tabs = (C.c_void_p * cap)()
        warns = np.zeros(wcap, COMPACT_WARN_DTYPE)
        n, nw = C.c_uint32(), C.c_uint32()
        st = lib().slate_compact_ex(ctx.handle, _ptr(blob), _ptr(off), len(flat), _ptr(src), len(sources),
                                    C.byref(cfg), max_sst_size, tabs, cap, C.byref(n), _ptr(warns), wcap, C.byref(nw))
        if st == E_CAPACITY and n.value > cap:
            cap = n.value
            continue
        if st not in (0, E_WARNINGS):
            _check(st, "slate_compact_ex")
        out = [SstTable(tabs[k]).encode() for k in range(n.value)]
        if nw.value > wcap:  # more warnings than records: run again with room for all of them
            wcap = nw.value
            continue
        return out, warns[:nw.value]


def compact(ctx: "Context", sources: list[list[bytes]], max_sst_size: int, block_size: int = 4096,
            min_filter_keys: int = 0, filter_bits_per_key: int = 10, codec: int = NONE) -> list[bytes]:
    """slate_compact: executeCompaction's codec path in one C-ABI call -> encoded output SSTs."""
    flat = [s for run in sources for s in run]
    blob = np.frombuffer(b"".join(flat) or b"\0", np.uint8)
    off = np.concatenate([[0], np.cumsum([len(s) for s in flat])]).astype(np.uint64)
    src = np.concatenate([[0], np.cumsum([len(r) for r in sources])]).astype(np.uint32)
    return [a.tobytes() for a in compact_arrays(ctx, blob, off, src, max_sst_size, block_size, min_filter_keys,
                                                filter_bits_per_key, codec)]


def compact_arrays(ctx: "Context", blob: np.ndarray, off: np.ndarray, src: np.ndarray, max_sst_size: int,
                   block_size: int = 4096, min_filter_keys: int = 0, filter_bits_per_key: int = 10, codec: int = NONE,
                   sink: np.ndarray | None = None) -> list[np.ndarray]:
    """slate_compact over SSTs packed in one array (sst i = blob[off[i]:off[i+1]], source j = SSTs
    src[j]..src[j+1]) as a cgo caller passes them: the output SSTs encoded back to back into `sink`
    (reused when large enough) -> views of it, one per output."""
    blob = np.ascontiguousarray(blob, np.uint8)
    off = np.ascontiguousarray(off, np.uint64)
    src = np.ascontiguousarray(src, np.uint32)
    flat = range(len(off) - 1)
    sources = range(len(src) - 1)
    cfg = SstConfig(block_size, min_filter_keys, filter_bits_per_key, codec)
    cap = 16
    while True:
        tabs = (C.c_void_p * cap)()
        n = C.c_uint32()
        st = lib().slate_compact(ctx.handle, _ptr(blob), _ptr(off), len(flat), _ptr(src), len(sources), C.byref(cfg),
                                 max_sst_size, tabs, cap, C.byref(n))
        if st == E_CAPACITY and n.value > cap:
            cap = n.value
            continue
        _check(st, "slate_compact")
        tables = [SstTable(tabs[k]) for k in range(n.value)]
        sizes = [int(lib().slate_sst_table_encoded_len(t._h)) for t in tables]
        if sink is None or sink.size < sum(sizes) + 1:
            sink = np.empty(sum(sizes) + 1, np.uint8)
        out, at = [], 0
        for t, z in zip(tables, sizes):
            out.append(t.encode_array(sink[at:at + z + 1])[:z])
            at += z
        return out


def shard_blocks(n_blocks: int, n_shards: int, shard: int) -> int:
    """Blocks of shard `shard` when block i goes to shard i mod n_shards."""
    return int(lib().slate_shard_blocks(n_blocks, n_shards, shard))


def shard_pack(blob: np.ndarray, in_off: np.ndarray, n_shards: int, shard: int):
    """slate_shard_pack: shard `shard`'s blocks back to back -> (bytes, offsets)."""
    blob = np.ascontiguousarray(blob, np.uint8)
    in_off = np.ascontiguousarray(in_off, np.uint64)
    n = len(in_off) - 1
    m = shard_blocks(n, n_shards, shard)
    idx = np.arange(shard, n, n_shards, dtype=np.int64)
    nbytes = int((in_off[idx + 1] - in_off[idx]).sum()) if m else 0
    out = np.zeros(max(nbytes, 1), np.uint8)
    off = np.zeros(m + 1, np.uint64)
    _check(lib().slate_shard_pack(_ptr(blob), _ptr(in_off), n, n_shards, shard, _ptr(out), nbytes, _ptr(off)),
           "slate_shard_pack")
    return out[:nbytes], off


def decode_sharded(ctxs: list["Context"], codec: int, blob: np.ndarray, in_off: np.ndarray):
    """slate_block_decode_sharded: block i decoded by ctxs[i % len(ctxs)], results in block order
    -> (out, out_off, meta, rows, row_base) as Context.decode_batch."""
    blob = np.ascontiguousarray(blob, np.uint8)
    in_off = np.ascontiguousarray(in_off, np.uint64)
    n = len(in_off) - 1
    hs = (C.c_void_p * len(ctxs))(*[c.handle for c in ctxs])
    out_off = np.zeros(n + 1, np.uint64)
    row_base = np.zeros(n + 1, np.uint64)
    meta = np.zeros(max(n, 1), META_DTYPE)
    L = lib()
    st = L.slate_block_decode_sharded(hs, len(ctxs), codec, _ptr(blob), _ptr(in_off), n, None, 0, _ptr(out_off),
                                      _ptr(meta), None, 0, _ptr(row_base))
    if st not in (OK, E_CAPACITY):
        raise SlateError(st, "slate_block_decode_sharded")
    out = np.zeros(max(int(out_off[n]), 1), np.uint8)
    rows = np.zeros(max(int(row_base[n]), 1), ROW_DTYPE)
    st = L.slate_block_decode_sharded(hs, len(ctxs), codec, _ptr(blob), _ptr(in_off), n, _ptr(out), out.size,
                                      _ptr(out_off), _ptr(meta), _ptr(rows), rows.size, _ptr(row_base))
    _check(st, "slate_block_decode_sharded")
    return out, out_off, meta[:n], rows, row_base


def decode_sharded_into(ctxs: list["Context"], codec: int, blob: np.ndarray, in_off: np.ndarray, out: np.ndarray,
                        rows: np.ndarray, meta: np.ndarray, out_off: np.ndarray, row_base: np.ndarray) -> int:
    """slate_block_decode_sharded into caller-sized buffers (one pass). Returns the status."""
    hs = (C.c_void_p * len(ctxs))(*[c.handle for c in ctxs])
    return lib().slate_block_decode_sharded(hs, len(ctxs), codec, _ptr(blob), _ptr(in_off), len(in_off) - 1,
                                            _ptr(out), out.size, _ptr(out_off), _ptr(meta), _ptr(rows), rows.size,
                                            _ptr(row_base))


class Index:
    def __init__(self, h):
        self._h = h

    @property
    def handle(self):
        return self._h

    def __del__(self):
        if getattr(self, "_h", None):
            try:
                lib().slate_index_free(self._h)
            except TypeError:  # interpreter shutdown: the module's globals are already gone
                pass
            self._h = None

    def block_offsets(self) -> np.ndarray:
        n = lib().slate_index_num_blocks(self._h)
        out = np.zeros(max(n, 1), np.uint64)
        _check(lib().slate_index_block_offsets(self._h, _ptr(out), out.size), "slate_index_block_offsets")
        return out[:n]

    def block_metas(self) -> list[tuple[int, bytes]]:
        out = []
        for i in range(lib().slate_index_num_blocks(self._h)):
            off = C.c_uint64()
            p = C.c_void_p()
            ln = C.c_size_t()
            _check(lib().slate_index_block_meta(self._h, i, C.byref(off), C.byref(p), C.byref(ln)), "block_meta")
            out.append((off.value, C.string_at(p.value, ln.value) if ln.value else b""))
        return out


class SstBuilder:
    """sstable.Builder (builder.go:92-268) on the GPU through the C-ABI."""

    def __init__(self, ctx: Context, block_size=4096, min_filter_keys=0, filter_bits_per_key=10, codec=NONE):
        cfg = SstConfig(block_size, min_filter_keys, filter_bits_per_key, codec)
        st = C.c_int()
        self._ctx = ctx
        self._h = lib().slate_sst_builder_new(ctx.handle, C.byref(cfg), C.byref(st))
        if not self._h:
            raise SlateError(st.value, "slate_sst_builder_new")

    def __del__(self):
        if getattr(self, "_h", None):
            lib().slate_sst_builder_free(self._h)
            self._h = None

    def add_value(self, key: bytes, value: bytes) -> int:
        return lib().slate_sst_builder_add_value(self._h, C.c_char_p(key), len(key), C.c_char_p(value), len(value))

    def add(self, key: bytes, value: bytes | None) -> int:
        return lib().slate_sst_builder_add(self._h, C.c_char_p(key), len(key), C.c_char_p(value or b""),
                                           len(value or b""), 1 if value is None else 0)

    def add_batch(self, keys: np.ndarray, key_off: np.ndarray, vals: np.ndarray, val_off: np.ndarray,
                  is_tomb: np.ndarray | None = None) -> int:
        return lib().slate_sst_builder_add_batch(self._h, _ptr(keys), _ptr(key_off), _ptr(vals), _ptr(val_off),
                                                 _ptr(is_tomb) if is_tomb is not None else None, len(key_off) - 1)

    def add_batch_device(self, d_keys: int, d_key_off: int, d_vals: int, d_val_off: int, n: int,
                         d_is_tomb: int | None = None) -> int:
        """slate_sst_builder_add_batch_device: device pointers (e.g. tensor.data_ptr())."""
        return lib().slate_sst_builder_add_batch_device(self._h, C.c_void_p(d_keys), C.c_void_p(d_key_off),
                                                        C.c_void_p(d_vals), C.c_void_p(d_val_off),
                                                        C.c_void_p(d_is_tomb) if d_is_tomb else None, n)

    def next_block(self) -> bytes | None:
        cap = 1 << 16
        while True:
            out = np.zeros(cap, np.uint8)
            ln = C.c_size_t()
            present = C.c_int()
            st = lib().slate_sst_builder_next_block(self._h, _ptr(out), cap, C.byref(ln), C.byref(present))
            if st == E_CAPACITY:
                cap = ln.value + 64
                continue
            _check(st, "slate_sst_builder_next_block")
            return out[: ln.value].tobytes() if present.value else None

    def build(self) -> "SstTable":
        t = C.c_void_p()
        _check(lib().slate_sst_builder_build(self._h, C.byref(t)), "slate_sst_builder_build")
        return SstTable(t)


class SstTable:
    def __init__(self, h):
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            lib().slate_sst_table_free(self._h)
            self._h = None

    def chunks(self) -> list[bytes]:
        out = []
        for i in range(lib().slate_sst_table_num_chunks(self._h)):
            p = C.c_void_p()
            ln = C.c_size_t()
            _check(lib().slate_sst_table_chunk(self._h, i, C.byref(p), C.byref(ln)), "chunk")
            out.append(C.string_at(p.value, ln.value) if ln.value else b"")
        return out

    def encode(self) -> bytes:
        return self.encode_array().tobytes()

    def encode_array(self, out: np.ndarray | None = None) -> np.ndarray:
        """The SST bytes (Table.Blocks concatenated) into `out` (reused when large enough) or a
        fresh uint8 array; returns the filled prefix."""
        n = lib().slate_sst_table_encoded_len(self._h)
        if out is None or out.size < max(n, 1):
            out = np.empty(max(n, 1), np.uint8)
        _check(lib().slate_sst_table_encode(self._h, _ptr(out), out.size), "encode")
        return out[:n]

    def info(self) -> dict:
        info = SstInfo()
        fk = np.zeros(1 << 16, np.uint8)
        _check(lib().slate_sst_table_info(self._h, C.byref(info), _ptr(fk), fk.size), "info")
        d = {f: getattr(info, f) for f, _ in SstInfo._fields_}
        d["first_key"] = fk[: info.first_key_len].tobytes()
        return d

    def bloom(self):
        present = C.c_int()
        npr = C.c_uint16()
        bl = C.c_size_t()
        lib().slate_sst_table_bloom(self._h, C.byref(present), C.byref(npr), None, 0, C.byref(bl))
        if not present.value:
            return None
        out = np.zeros(max(bl.value, 1), np.uint8)
        _check(lib().slate_sst_table_bloom(self._h, C.byref(present), C.byref(npr), _ptr(out), out.size,
                                           C.byref(bl)), "bloom")
        return npr.value, out[: bl.value].tobytes()


def _arena(items: list[bytes]):
    off = np.zeros(len(items) + 1, np.uint64)
    if items:
        off[1:] = np.cumsum([len(x) for x in items], dtype=np.uint64)
    data = np.frombuffer(b"".join(items) or b"\0", dtype=np.uint8).copy()
    return data, off


def reader_walk(ctx: "Context", info: "SstInfo", index: "Index", sst: bytes, first: int = 0, read_ahead: int = 64):
    """Drives slate_block_reader as a Go shim would: -> ([(block, status, meta, data, rows)], [(rs, re)
    ranges fetched])."""
    h = C.c_void_p()
    _check(lib().slate_block_reader_create(ctx._h, C.byref(info), index.handle, first, read_ahead, C.byref(h)),
           "slate_block_reader_create")
    out, fetches = [], []
    buf = None
    try:
        v = BlockView()
        while True:
            st = lib().slate_block_reader_next(h, C.byref(v))
            if st == E_READER_END:
                break
            if st == E_READER_NEED_DATA:
                rs, re_ = C.c_uint64(), C.c_uint64()
                _check(lib().slate_block_reader_want(h, C.byref(rs), C.byref(re_)), "slate_block_reader_want")
                fetches.append((rs.value, re_.value))
                buf = np.frombuffer(bytes(sst[rs.value:re_.value]) or b"\0", dtype=np.uint8)
                _check(lib().slate_block_reader_feed(h, _ptr(buf), re_.value - rs.value), "slate_block_reader_feed")
                continue
            meta = np.frombuffer(bytes(v.meta), META_DTYPE)[0]
            n = int(meta["n_rows"])
            dl = int(meta["data_len"]) + 2 * n
            data = C.string_at(v.data, dl) if st == OK else b""
            rows = np.frombuffer(C.string_at(v.rows, 16 * n), ROW_DTYPE).copy() if st == OK and n else \
                np.zeros(0, ROW_DTYPE)
            out.append((int(v.block), st, meta, data, rows))
            if st != OK:
                break
    finally:
        lib().slate_block_reader_free(h)
    return out, fetches


def read_info(sst: bytes) -> tuple[int, "SstInfo", bytes]:
    b = np.frombuffer(bytes(sst) or b"\0", dtype=np.uint8)
    info = SstInfo()
    fk = np.zeros(max(len(sst), 16), np.uint8)
    st = lib().slate_sst_read_info(_ptr(b), len(sst), C.byref(info), _ptr(fk), fk.size)
    return st, info, fk[: info.first_key_len].tobytes()


def decode_scratch_bytes(n: int, codec: int = None) -> int:
    if codec is None:
        return lib().slate_decode_scratch_bytes(n)
    return lib().slate_decode_scratch_bytes_codec(n, codec)


def header_symbols() -> list[str]:
    """Every function declared in include/slatecodec.h."""
    import re
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(slate_[a-z0-9_]+)\s*\(", src)) - {"slate_ctx", "slate_row"})
