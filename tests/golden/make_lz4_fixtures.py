"""Writes tests/golden/lz4_frames.json: LZ4 frames produced by liblz4 1.9.3 (LZ4F_compressFrame,
/opt/conda/lib/liblz4.so.1 in the build container) with the options pierrec/lz4/v4's writer
and other producers use, with the decoded length and SHA-256.  They pin the oracle's LZ4 frame decoder
(and through it the GPU decoder) to an independent implementation of the format.
Run once here; the JSON is committed (the GPU box never runs this)."""
import ctypes
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


class Prefs(ctypes.Structure):
    # LZ4F_preferences_t (lz4frame.h 1.9.3): frameInfo, compressionLevel, autoFlush,
    # favorDecSpeed, reserved[3]
    _fields_ = [("blockSizeID", ctypes.c_int), ("blockMode", ctypes.c_int), ("contentChecksumFlag", ctypes.c_int),
                ("frameType", ctypes.c_int), ("contentSize", ctypes.c_ulonglong), ("dictID", ctypes.c_uint),
                ("blockChecksumFlag", ctypes.c_int), ("compressionLevel", ctypes.c_int),
                ("autoFlush", ctypes.c_uint), ("favorDecSpeed", ctypes.c_uint), ("reserved", ctypes.c_uint * 3)]


def main():
    lib = ctypes.CDLL("/opt/conda/lib/liblz4.so.1")
    lib.LZ4F_compressFrameBound.restype = ctypes.c_size_t
    lib.LZ4F_compressFrame.restype = ctypes.c_size_t
    lib.LZ4F_isError.restype = ctypes.c_uint
    sys.path.insert(0, HERE)
    from lz4_payloads import payloads
    cases = []
    options = [(7, 1, 1, 0, 0, 1),   # pierrec/lz4 v4 writer defaults: 4 MiB blocks, independent, content checksum
               (4, 1, 0, 0, 0, 1),   # 64 KiB blocks, no checksums
               (4, 0, 1, 1, 1, 1),   # linked blocks, block + content checksums, content size
               (5, 1, 1, 1, 0, 9)]   # 256 KiB blocks, block checksums, HC level
    for pi, data in enumerate(payloads()):
        for bsid, indep, ccheck, bcheck, csize, level in options:
            p = Prefs()
            p.blockSizeID, p.blockMode, p.contentChecksumFlag = bsid, 0 if indep else 1, ccheck
            p.blockChecksumFlag, p.contentSize, p.compressionLevel = bcheck, len(data) if csize else 0, level
            cap = lib.LZ4F_compressFrameBound(ctypes.c_size_t(len(data)), ctypes.byref(p))
            dst = ctypes.create_string_buffer(cap)
            n = lib.LZ4F_compressFrame(dst, ctypes.c_size_t(cap), data, ctypes.c_size_t(len(data)), ctypes.byref(p))
            assert not lib.LZ4F_isError(ctypes.c_size_t(n)), n
            cases.append({"payload": pi, "bsid": bsid, "independent": indep, "content_checksum": ccheck,
                          "block_checksum": bcheck, "content_size": csize, "level": level,
                          "frame": dst.raw[:n].hex(), "decoded_len": len(data),
                          "decoded_sha256": hashlib.sha256(data).hexdigest()})
    json.dump({"generator": "liblz4 %d LZ4F_compressFrame" % lib.LZ4_versionNumber(), "cases": cases},
              open(os.path.join(HERE, "lz4_frames.json"), "w"))
    print(len(cases), "frames")


if __name__ == "__main__":
    main()
