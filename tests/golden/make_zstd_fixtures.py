"""Writes tests/golden/zstd_frames.json: Zstandard frames written by libzstd 1.4.9 (ctypes,
/opt/conda/lib/libzstd.so.1) and by pyarrow's zstd codec, with their decoded bytes and the low
32 bits of XXH64 (the frame content checksum).  Test fixtures for the oracle's CodecZstd
decoder (klauspost/compress is absent, so libzstd is the independent producer).
Run: python tests/golden/make_zstd_fixtures.py"""
import json
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from tests import zstdgen  # noqa: E402

# XXH64 low 32 bits from libzstd's own frames: the checksum field of a frame written with
# checksumFlag=1 is exactly that value, so it is read back from the frame.


def main():
    rng = random.Random(20250307)
    cases = []

    def add(name, data, frame):
        ck = int.from_bytes(zstdgen.frame(data, 1, True, True)[-4:], "little")
        cases.append({"name": name, "data": data.hex(), "frame": frame.hex(), "xxh64_lo": ck})

    words = [bytes(rng.randrange(97, 123) for _ in range(rng.randint(2, 8))) for _ in range(30)]
    texts = [b" ".join(rng.choice(words) for _ in range(n)) for n in (3, 40, 300, 900)]
    rand = [bytes(rng.randrange(256) for _ in range(n)) for n in (1, 17, 700, 1500)]
    rle = [bytes([7]) * 1000, b"ab" * 700]
    datas = texts + rand + rle + [b""]
    for i, d in enumerate(datas):
        for lvl in (-3, 1, 3, 19):
            if lvl in (1, 19) and i % 2:
                continue
            add(f"libzstd-l{lvl}-d{i}", d, zstdgen.frame(d, lvl, lvl != 1, lvl != 19))
    try:
        import pyarrow as pa
        c = pa.Codec("zstd", compression_level=3)
        for i, d in enumerate(texts + rand[:2]):
            add(f"pyarrow-d{i}", d, c.compress(d).to_pybytes())
    except Exception as e:  # pyarrow optional
        print("pyarrow zstd skipped:", e)
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "zstd_frames.json")
    json.dump({"producer": "libzstd 1.4.9 (ctypes) + pyarrow zstd; Go reference not executed", "cases": cases},
              open(out, "w"), indent=0)
    print(len(cases), "cases ->", out, os.path.getsize(out), "bytes")


if __name__ == "__main__":
    main()
