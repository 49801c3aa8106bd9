"""Synthetic SST-block workloads for bench.py, built with
tools/benchgen.c: keys b"k%015d", 84-byte values (V-half r||r from
numpy.random.default_rng(20250307), or V-rand), BlockSize 4096, then Snappy
(C++ libsnappy from /opt/conda), LZ4 frames (liblz4) or None, plus the block CRC32 trailer."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libbenchgen.so")
LIBSNAPPY = "/opt/conda/lib/libsnappy.so.1"
LIBLZ4 = "/opt/conda/lib/liblz4.so.1"
LIBZSTD = "/opt/conda/lib/libzstd.so.1"

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        L = C.CDLL(LIB)
        L.bg_init.argtypes = [C.c_char_p]
        L.bg_build_blocks.restype = C.c_uint64
        L.bg_build_blocks.argtypes = [C.c_uint64, C.c_uint64, C.c_void_p, C.c_uint32, C.c_int, C.c_uint64,
                                      C.c_void_p, C.c_void_p, C.c_uint64]
        L.bg_encode_blocks.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                       C.c_void_p, C.c_int]
        L.bg_compact.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]
        rc = L.bg_init(LIBSNAPPY.encode())
        if rc != 0:
            raise RuntimeError(f"benchgen: cannot load {LIBSNAPPY} ({rc})")
        L.bg_init_lz4.argtypes = [C.c_char_p]
        L.bg_init_lz4(LIBLZ4.encode())  # codec 3 (LZ4 frames) only: optional
        L.bg_init_zstd.argtypes = [C.c_char_p]
        L.bg_init_zstd(LIBZSTD.encode())  # codec 4 (Zstd level 3 + checksum) only: optional
        L.bg_build_set.restype = C.c_int
        L.bg_build_set.argtypes = [C.c_uint64, C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int,
                                   C.c_void_p, C.c_uint64, C.c_void_p, C.c_int]
        L.bg_verify_set.restype = C.c_int64
        L.bg_verify_set.argtypes = [C.c_uint64, C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p,
                                    C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.bg_compare_blocks.restype = C.c_int64
        L.bg_compare_blocks.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
        L.bg_build_mixed.restype = C.c_uint64
        L.bg_build_mixed.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint64]
        _lib = L
    return _lib


def decoded_blocks(n_blocks: int, seed: int = 20250307, half: bool = True, block_size: int = 4096,
                   kv_begin: int = 0):
    """-> (decoded blob uint8, offsets uint64[n+1]) for exactly n_blocks blocks."""
    kv_per_block = 40  # >= rows per 4 KiB block for 100-byte KVs (38 typical)
    n_kv = n_blocks * kv_per_block + 64
    rng = np.random.default_rng(seed)
    rv = rng.integers(0, 256, (n_kv, 42 if half else 84), dtype=np.uint8)
    out = np.empty(n_blocks * (block_size + 256), np.uint8)
    off = np.zeros(n_blocks + 1, np.uint64)
    nb = lib().bg_build_blocks(kv_begin, n_kv, rv.ctypes.data, rv.shape[1], int(half), block_size,
                               out.ctypes.data, off.ctypes.data, n_blocks)
    assert nb == n_blocks, (nb, n_blocks)
    return out[: int(off[nb])], off


def mixed_blocks(n_blocks: int, seed: int = 20250307, block_size: int = 4096):
    """BASELINE configs[4] decoded blocks (1 KiB V-half values, Zipf-prefixed 8-256 B keys)."""
    out = np.empty(n_blocks * (block_size + 256), np.uint8)
    off = np.zeros(n_blocks + 1, np.uint64)
    kvs = n_blocks * max(8, block_size // 512) + 64  # (1 KiB values: enough KVs for every block)
    nb = lib().bg_build_mixed(seed, kvs, block_size, out.ctypes.data, off.ctypes.data, n_blocks)
    assert nb == n_blocks, (nb, n_blocks)
    return out[: int(off[nb])], off


def encode_blocks(codec: int, dec: np.ndarray, dec_off: np.ndarray, threads: int = 16):
    n = len(dec_off) - 1
    lens = np.diff(dec_off.astype(np.int64))
    stride = int(lens.max()) + int(lens.max()) // 6 + 64
    slots = np.empty(n * stride, np.uint8)
    elen = np.zeros(n, np.uint64)
    rc = lib().bg_encode_blocks(codec, dec.ctypes.data, dec_off.ctypes.data, n, slots.ctypes.data, stride,
                                elen.ctypes.data, threads)
    assert rc == 0, rc
    blob = np.empty(int(elen.sum()) + 16, np.uint8)
    off = np.zeros(n + 1, np.uint64)
    lib().bg_compact(slots.ctypes.data, stride, elen.ctypes.data, n, blob.ctypes.data, off.ctypes.data)
    return blob, off


def snappy_vhalf(n_blocks: int, codec: int = 1, seed: int = 20250307, half: bool = True, threads: int = 16,
                 kv_begin: int = 0):
    dec, doff = decoded_blocks(n_blocks, seed=seed, half=half, kv_begin=kv_begin)
    blob, off = encode_blocks(codec, dec, doff, threads)
    return blob, off, int(doff[-1])


def block_set(codec: int, i_begin: int, stride: int, count: int, seed: int = 20250307, half: bool = True,
              block_size: int = 4096, threads: int = 16, chunk: int = 262144):
    """Encoded blocks i_begin + k * stride (k < count) of the per-block synthetic set (tools/benchgen.c
    bg_build_set): one rank's round-robin shard of a set that no rank holds whole -> (blob, in_off)."""
    stride_e = block_size + block_size // 6 + 64
    off = np.zeros(count + 1, np.uint64)
    blob = None
    pos = 0
    for k0 in range(0, count, chunk):
        m = min(chunk, count - k0)
        slots = np.empty(m * stride_e, np.uint8)
        elen = np.zeros(m, np.uint64)
        rc = lib().bg_build_set(seed, int(half), block_size, i_begin + k0 * stride, stride, m, codec,
                                slots.ctypes.data, stride_e, elen.ctypes.data, threads)
        assert rc == 0, rc
        part = np.empty(int(elen.sum()) + 16, np.uint8)
        poff = np.zeros(m + 1, np.uint64)
        lib().bg_compact(slots.ctypes.data, stride_e, elen.ctypes.data, m, part.ctypes.data, poff.ctypes.data)
        del slots
        nb = int(poff[m])
        if blob is None:  # size the whole shard from the first chunk's average, grow if needed
            blob = np.empty(int(nb / m * count * 1.02) + 4096, np.uint8)
        if pos + nb + 16 > blob.size:
            blob = np.resize(blob, int((pos + nb) * 1.1) + 4096)
        blob[pos:pos + nb] = part[:nb]
        off[k0:k0 + m + 1] = poff + np.uint64(pos)
        pos += nb
    if blob is None:
        blob = np.zeros(16, np.uint8)
    return blob[:pos + 16], off


def verify_set(i_begin: int, stride: int, count: int, out: np.ndarray, out_off: np.ndarray, rows: np.ndarray,
               row_base: np.ndarray, meta: np.ndarray, seed: int = 20250307, half: bool = True,
               block_size: int = 4096, threads: int = 16) -> int:
    """Blocks k < count decoded by the GPU (bytes at out[out_off[k]:], row descriptors from
    rows[row_base[k]], 16-byte meta) against the generator: number of mismatching blocks."""
    return int(lib().bg_verify_set(seed, int(half), block_size, i_begin, stride, count, out.ctypes.data,
                                   out_off.ctypes.data, rows.ctypes.data, row_base.ctypes.data, meta.ctypes.data,
                                   threads))


def compare_blocks(out: np.ndarray, out_off: np.ndarray, dec: np.ndarray, dec_off: np.ndarray) -> int:
    """Blocks whose decoded bytes (at out[out_off[i]:]) differ from dec's block i."""
    out_off = np.ascontiguousarray(out_off, np.uint64)
    dec_off = np.ascontiguousarray(dec_off, np.uint64)
    return int(lib().bg_compare_blocks(out.ctypes.data, out_off.ctypes.data, dec.ctypes.data, dec_off.ctypes.data,
                                       len(dec_off) - 1))
