"""Zstandard frames for decoder tests (test infrastructure only), written by libzstd 1.4.9
through ctypes (/opt/conda/lib/libzstd.so.1, present in this image here and on the GPU box).
libzstd is an independent producer: klauspost/compress (the reference's encoder) is absent,
so its exact frames are parity unpinned; decoded bytes are pinned by the format."""
import ctypes as C
import os

_PATHS = ["/opt/conda/lib/libzstd.so.1", "libzstd.so.1"]
_L = None
C_LEVEL, C_WINDOWLOG, C_STRATEGY = 100, 101, 107
C_CONTENTSIZE, C_CHECKSUM = 200, 201


def available() -> bool:
    try:
        lib()
        return True
    except OSError:
        return False


def lib():
    global _L
    if _L is None:
        err = None
        for p in _PATHS:
            try:
                _L = C.CDLL(p)
                break
            except OSError as e:
                err = e
        if _L is None:
            raise err
        _L.ZSTD_createCCtx.restype = C.c_void_p
        _L.ZSTD_freeCCtx.argtypes = [C.c_void_p]
        _L.ZSTD_CCtx_setParameter.argtypes = [C.c_void_p, C.c_int, C.c_int]
        _L.ZSTD_CCtx_setParameter.restype = C.c_size_t
        _L.ZSTD_compress2.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        _L.ZSTD_compress2.restype = C.c_size_t
        _L.ZSTD_compressBound.argtypes = [C.c_size_t]
        _L.ZSTD_compressBound.restype = C.c_size_t
        _L.ZSTD_isError.argtypes = [C.c_size_t]
        _L.ZSTD_isError.restype = C.c_uint
        _L.ZSTD_getErrorName.argtypes = [C.c_size_t]
        _L.ZSTD_getErrorName.restype = C.c_char_p
        _L.ZSTD_decompress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        _L.ZSTD_decompress.restype = C.c_size_t
    return _L


def frame(data: bytes, level: int = 3, checksum: bool = True, content_size: bool = True, window_log: int = 0,
          strategy: int = 0) -> bytes:
    L = lib()
    cc = L.ZSTD_createCCtx()
    try:
        for k, v in ((C_LEVEL, level), (C_CHECKSUM, int(checksum)), (C_CONTENTSIZE, int(content_size)),
                     (C_WINDOWLOG, window_log), (C_STRATEGY, strategy)):
            r = L.ZSTD_CCtx_setParameter(cc, k, v)
            assert not L.ZSTD_isError(r), L.ZSTD_getErrorName(r)
        cap = L.ZSTD_compressBound(len(data))
        out = C.create_string_buffer(cap)
        src = C.create_string_buffer(bytes(data), len(data) or 1)
        n = L.ZSTD_compress2(cc, out, cap, src, len(data))
        assert not L.ZSTD_isError(n), L.ZSTD_getErrorName(n)
        return out.raw[:n]
    finally:
        L.ZSTD_freeCCtx(cc)
