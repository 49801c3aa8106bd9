"""CodecZstd index / filter payloads written the way the reference writes them -- klauspost/compress's
streaming writer (compression.go:105-118): one frame of up to 128 KiB blocks that share entropy
state (repeat offsets across blocks, treeless literals, repeat FSE tables) -- decoded by the
block-parallel decoder (api_sst.cpp zstd_payload_par_run, csrc/zstd_par.hip), against the oracle's
restatement of the reference reader (compression.go:146-153 under bloom.Decode bloom.go:70-91 and
DecodeIndex flatbuf.go:83-100).  klauspost is absent here; libzstd 1.4.9 writes the same frame shape
(tests/zstdgen.py) and is what the tests use (klauspost's exact frames are parity unpinned).
Damaged frames fail a check of the parallel passes and reach the exact decoder, which reports them."""
import os
import random
import subprocess
import sys
import time

import numpy as np
import pytest

from oracle import binding as ob
from tests import sstgen, zstdgen

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not zstdgen.available(), reason="libzstd not in this image")]

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def sc():
    import slatecodec
    return slatecodec


@pytest.fixture(scope="module")
def ctx(sc):
    return sc.Context(0)


@pytest.fixture(scope="module")
def sst_parts(sc, ctx):
    """Index and filter bytes of a 2 M-KV CodecNone SST (built by the library)."""
    from tools.bench_encode import kv_arrays
    keys, key_off, vals, val_off = kv_arrays(2_000_000)
    b = sc.SstBuilder(ctx, 4096, 0, 10, ob.NONE)
    assert b.add_batch(keys, key_off, vals, val_off) == 0
    sst = b.build().encode()
    st, info, _ = sc.read_info(sst)
    ib = sst[info.index_offset:info.index_offset + info.index_len][:-4]
    fb = sst[info.filter_offset:info.filter_offset + info.filter_len][:-4]
    return ib, fb


def _check(ctx, frame: bytes):
    g = ctx.bloom_decode(frame, ob.ZSTD)
    o = ob.bloom_decode(frame, ob.ZSTD, cap=1 << 26)
    assert g[0] == o[0] and g[1:] == o[1:], (g[0], o[0])
    return g[0]


def _blocks(frame: bytes):
    """(block count, literal section types of the compressed blocks) of a single frame."""
    fhd = frame[4]
    ss = (fhd >> 5) & 1
    p = 5 + (0 if ss else 1) + [0, 1, 2, 4][fhd & 3] + [ss, 2, 4, 8][fhd >> 6]
    n, lts = 0, set()
    while True:
        bh = int.from_bytes(frame[p:p + 3], "little")
        p += 3
        bt, bs = (bh >> 1) & 3, bh >> 3
        n += 1
        if bt == 2:
            lts.add(frame[p] & 3)
        p += 1 if bt == 1 else bs
        if bh & 1:
            return n, lts


def test_zstd_multiblock_sst_payloads(ctx, sst_parts):
    """The index and filter compressed at libzstd level 3 (the klauspost default's band), streaming
    shape (no content size, with checksum): many blocks, treeless literals among them; decoded like
    the oracle, in far less time than the exact one-wave path (~1.3 s / ~6 s at this size)."""
    ib, fb = sst_parts
    iz = sstgen.crc(zstdgen.frame(ib, level=3, content_size=False))
    fz = sstgen.crc(zstdgen.frame(fb, level=3, content_size=False))
    n, lts = _blocks(iz[:-4])
    assert n > 8, n
    _check(ctx, fz)  # warm-up
    t0 = time.perf_counter()
    assert _check(ctx, fz) == 0
    dt_f = time.perf_counter() - t0
    t0 = time.perf_counter()
    st, index = ctx.decode_index(iz, ob.ZSTD)
    dt_i = time.perf_counter() - t0
    ost, ometas = ob.decode_index(iz, ob.ZSTD, cap=1 << 26)
    assert st == ost == 0 and index.block_metas() == ometas
    print(f"\n2 M KV zstd-3: filter {len(fb)} B ({len(fz)} compressed) in {dt_f * 1e3:.1f} ms, "
          f"index {len(ib)} B ({len(iz)} compressed, {n} blocks) in {dt_i * 1e3:.1f} ms")
    assert dt_f < 0.5 and dt_i < 0.5, (dt_f, dt_i)


def test_zstd_par_taken(sst_parts, tmp_path):
    """The block-parallel path is the one that decodes them (SLATE_HOST_TRACE: no hand-off to the
    exact decoder), in a child process (the trace switch is read once)."""
    ib, fb = sst_parts
    p = tmp_path / "payloads.bin"
    iz = sstgen.crc(zstdgen.frame(ib, level=3, content_size=False))
    fz = sstgen.crc(zstdgen.frame(fb, level=9, content_size=True))
    p.write_bytes(len(iz).to_bytes(8, "little") + iz + fz)
    code = r"""
import sys
sys.path[:0] = [%r, %r]
import torch; torch.cuda.init()
import slatecodec as sc
from oracle import binding as ob
d = open(%r, "rb").read()
n = int.from_bytes(d[:8], "little")
iz, fz = d[8:8 + n], d[8 + n:]
ctx = sc.Context(0)
st, index = ctx.decode_index(iz, ob.ZSTD)
assert st == 0
g = ctx.bloom_decode(fz, ob.ZSTD)
assert g[0] == 0
print("ok")
""" % (REPO, os.path.join(REPO, "slatedb-go_amd"), str(p))
    env = dict(os.environ, SLATE_HOST_TRACE="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-2000:] + r.stderr[-2000:]
    print("\n" + "\n".join(ln for ln in r.stderr.splitlines() if ln.startswith("[slate zstd-par]")))
    ends = [ln for ln in r.stderr.splitlines() if ln.startswith("[slate zstd-par] bytes")]
    assert len(ends) == 2 and all(ln.endswith("fail 0") for ln in ends), r.stderr[-3000:]


def test_zstd_treeless_and_repeat_tables(ctx):
    """Key-like bytes at level 3: blocks whose literals reuse the previous block's Huffman tree
    (treeless) among many blocks, with repeat offsets across block boundaries."""
    raw = b"".join(b"\x0c\x00\x00\x00key%012d" % (i * 37) for i in range(300000))
    for level in (1, 3, 9):
        f = zstdgen.frame(raw, level=level, content_size=level != 3)
        n, lts = _blocks(f)
        if level == 3:
            assert n > 8 and 3 in lts, (n, lts)
        assert _check(ctx, sstgen.crc(f)) == 0


@pytest.mark.parametrize("level", [-1, 1, 3, 9, 19])
def test_zstd_levels(ctx, sst_parts, level):
    """Every level band, with and without content size and checksum."""
    ib, fb = sst_parts
    rng = random.Random(level)
    for raw in (ib[:900_000], fb[:600_000]):
        f = zstdgen.frame(raw, level=level, checksum=rng.random() < 0.7, content_size=rng.random() < 0.5)
        assert _check(ctx, sstgen.crc(f)) == 0


@pytest.mark.parametrize("kind", ["zeros", "random", "pattern", "text"])
def test_zstd_shapes(ctx, kind):
    """Frame shapes: RLE blocks, raw (incompressible) blocks, repeat offsets with short matches
    reaching across blocks, text with Huffman literals."""
    rng = np.random.default_rng(6)
    if kind == "zeros":
        raw = bytes(2_000_000)
    elif kind == "random":
        raw = rng.integers(0, 256, 1_000_000, dtype=np.uint8).tobytes()
    elif kind == "pattern":
        unit = rng.integers(0, 256, 900, dtype=np.uint8)
        parts = []
        for i in range(3000):
            u = unit.copy()
            u[rng.integers(0, 900, 9)] = rng.integers(0, 256, 9, dtype=np.uint8)
            parts.append(u[: 200 + (i * 53) % 700].tobytes())
        raw = b"".join(parts)
    else:
        words = [bytes(rng.integers(97, 123, int(rng.integers(2, 9)), dtype=np.uint8)) for _ in range(3000)]
        raw = b" ".join(words[int(i)] for i in rng.integers(0, 3000, 300_000))
    for level in (1, 3):
        assert _check(ctx, sstgen.crc(zstdgen.frame(raw, level=level, content_size=False))) == 0


def test_zstd_damaged(ctx, sst_parts):
    """Flipped bits under a valid CRC, a wrong checksum, a wrong content size and truncation: the
    statuses (and bytes where a frame still decodes) are the oracle's."""
    rng = random.Random(8)
    ib, fb = sst_parts
    base = [zstdgen.frame(ib[:500_000], level=3, content_size=True),
            zstdgen.frame(fb[:300_000], level=3, content_size=False)]
    for trial in range(24):
        body = bytearray(base[trial % 2])
        kind = trial % 6
        if kind == 0:
            body[-1] ^= 0x10  # XXH64
        elif kind == 1:
            body = body[: len(body) - rng.randrange(5, 300)]
        else:
            for _ in range(rng.randint(1, 3)):
                body[rng.randrange(12, len(body) - 4)] ^= 1 << rng.randrange(8)
        _check(ctx, sstgen.crc(bytes(body)))
