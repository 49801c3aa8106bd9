"""The oracle's LZ4 frame decoder (compress.Decode CodecLz4, compression.go:143-144) pinned
to frames written by liblz4 (tests/golden/lz4_frames.json), plus XXH32 against the xxhash
module, round trips of tests/lz4gen.py frames over every frame option, and the error
codes for damaged frames.  CPU only."""
import hashlib
import json
import os
import random
import struct
import sys

import pytest

from oracle import binding as ob
from tests import lz4gen

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLDEN)
from lz4_payloads import payloads  # noqa: E402

E_MAGIC, E_HDR, E_BLOCK, E_FRAME, E_CORRUPT = 14, 15, 16, 17, 18


def test_golden_liblz4_frames():
    data = json.load(open(os.path.join(GOLDEN, "lz4_frames.json")))
    pl = payloads()
    assert len(data["cases"]) == 32
    for c in data["cases"]:
        st, out = ob.lz4_decode(bytes.fromhex(c["frame"]))
        assert st == 0, c
        assert len(out) == c["decoded_len"] and hashlib.sha256(out).hexdigest() == c["decoded_sha256"]
        assert out == pl[c["payload"]]


def test_xxh32_matches_reference():
    rng = random.Random(1)
    for n in list(range(0, 40)) + [100, 1000, 4097]:
        b = bytes(rng.randrange(256) for _ in range(n))
        assert ob.xxh32(b) == lz4gen.xxh32(b)


@pytest.mark.parametrize("seed", range(8))
def test_generated_frames_round_trip(seed):
    rng = random.Random(seed)
    for _ in range(20):
        n = rng.choice([0, 1, 5, 15, 16, 300, 4000, 70000])
        alphabet = rng.choice([2, 16, 256])
        data = bytes(rng.randrange(alphabet) for _ in range(n))
        if rng.random() < 0.5:
            data = data[: n // 2] * 2
        f = lz4gen.frame(data, bsid=rng.choice([4, 5, 7]), indep=rng.random() < 0.5,
                         block_checksum=rng.random() < 0.5, content_checksum=rng.random() < 0.7,
                         content_size=rng.random() < 0.3, stored_p=rng.choice([0, 0.3]), rng=rng,
                         block_split=rng.choice([None, 1000, 4096]))
        st, out = ob.lz4_decode(f)
        assert st == 0 and out == data


def test_damaged_frames():
    data = b"".join(b"row-%05d:" % i for i in range(300))
    f = bytearray(lz4gen.frame(data, bsid=4, block_checksum=True, content_checksum=True))
    assert ob.lz4_decode(bytes(f)) == (0, data)
    bad = bytearray(f); bad[0] ^= 1
    assert ob.lz4_decode(bytes(bad))[0] == E_MAGIC
    bad = bytearray(f); bad[6] ^= 0xFF  # the header checksum byte
    assert ob.lz4_decode(bytes(bad))[0] == E_HDR
    bad = bytearray(f); bad[20] ^= 0x40  # inside the first block
    assert ob.lz4_decode(bytes(bad))[0] == E_BLOCK
    bad = bytearray(f); bad[-1] ^= 1  # content checksum
    assert ob.lz4_decode(bytes(bad))[0] == E_FRAME
    assert ob.lz4_decode(bytes(f) + b"\0")[0] == E_CORRUPT  # trailing data
    assert ob.lz4_decode(bytes(f[:-5]))[0] == E_CORRUPT  # truncated
    g = bytearray(lz4gen.frame(data, bsid=4, content_checksum=False))
    g[4] |= 2  # reserved flag bit
    assert ob.lz4_decode(bytes(g))[0] in (E_HDR, E_CORRUPT)
    # offset 0 inside a block (no checksums to catch it first)
    body = bytes([0x10 | 0x00]) + b"a" + struct.pack("<H", 0) + bytes([0x10]) + b"b"
    desc = bytes([0x60, 0x40])
    h = struct.pack("<I", 0x184D2204) + desc + bytes([(lz4gen.xxh32(desc) >> 8) & 0xFF])
    fr = h + struct.pack("<I", len(body)) + body + struct.pack("<I", 0)
    assert ob.lz4_decode(fr)[0] == E_CORRUPT
