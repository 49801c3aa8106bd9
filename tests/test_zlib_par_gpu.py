"""CodecZlib index / filter payloads written the way the reference writes them -- compress/zlib at
the default level (compression.go:96-103), one deflate stream without flush points -- decoded by the
speculative block-parallel inflate (api_sst.cpp zlib_payload_par_run, csrc/zlib_par.hip), against
the oracle's restatement of the reference reader (compression.go:134-140 under bloom.Decode
bloom.go:70-91 and DecodeIndex flatbuf.go:83-100): decoded bytes and statuses.  Go's compress/flate
is absent here; zlib's deflate (levels 1-9 and its strategies) writes the same stream shape --
dynamic, fixed and stored blocks, matches reaching into earlier blocks -- and is what the tests use
(parity for Go's own block choices is unpinned).  Damaged streams fail a check of the parallel
passes and reach the exact decoder, which reports them."""
import os
import random
import subprocess
import sys
import time
import zlib

import numpy as np
import pytest

from oracle import binding as ob
from tests import sstgen

pytestmark = pytest.mark.gpu

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


def _zlib(raw: bytes, level: int = 6, strategy: int = zlib.Z_DEFAULT_STRATEGY, wbits: int = 15) -> bytes:
    c = zlib.compressobj(level, zlib.DEFLATED, wbits, 8, strategy)
    return sstgen.crc(c.compress(raw) + c.flush())


def _check_filter(ctx, frame: bytes):
    g = ctx.bloom_decode(frame, ob.ZLIB)
    o = ob.bloom_decode(frame, ob.ZLIB, cap=1 << 26)
    assert g[0] == o[0] and g[1:] == o[1:], (g[0], o[0])
    return g[0]


def test_zlib_default_level_sst_payloads(ctx, sst_parts):
    """The index and filter compressed as compress/zlib's default writer would (level 6, no flush
    points) open like the oracle, in far less time than the exact one-wave path (~0.8 s for this
    index and ~3 s for this filter)."""
    ib, fb = sst_parts
    iz, fz = _zlib(ib), _zlib(fb)
    _check_filter(ctx, fz)  # warm-up (tables, buffers)
    t0 = time.perf_counter()
    assert _check_filter(ctx, fz) == 0
    dt_f = time.perf_counter() - t0
    t0 = time.perf_counter()
    st, index = ctx.decode_index(iz, ob.ZLIB)
    dt_i = time.perf_counter() - t0
    ost, ometas = ob.decode_index(iz, ob.ZLIB, cap=1 << 26)
    assert st == ost == 0 and index.block_metas() == ometas
    print(f"\n2 M KV zlib-6: filter {len(fb)} B ({len(fz)} compressed) in {dt_f * 1e3:.1f} ms, "
          f"index {len(ib)} B ({len(iz)} compressed) in {dt_i * 1e3:.1f} ms")
    assert dt_f < 0.5 and dt_i < 0.5, (dt_f, dt_i)


def test_zlib_par_taken(sst_parts, tmp_path):
    """The parallel path is the one that decodes these streams (SLATE_HOST_TRACE reports its chain:
    no hand-off to the exact decoder), in a child process (the trace switch is read once)."""
    ib, fb = sst_parts
    _par_chains(tmp_path, _zlib(ib, 6), _zlib(fb, 9))


def test_go_shaped_streams(ctx, sst_parts, tmp_path):
    """Streams closed the way Go's compress/zlib closes them (data blocks, then an empty final
    stored block: sstgen.go_zlib): decoded like the oracle, and by the parallel path (no hand-off)."""
    ib, fb = sst_parts
    iz, fz = sstgen.crc(sstgen.go_zlib(ib, 6)), sstgen.crc(sstgen.go_zlib(fb, 9))
    assert iz[-12:-8] == fz[-12:-8] == b"\x00\x00\xff\xff"  # LEN / NLEN of the empty stored block
    assert _check_filter(ctx, fz) == 0
    st, index = ctx.decode_index(iz, ob.ZLIB)
    ost, ometas = ob.decode_index(iz, ob.ZLIB, cap=1 << 26)
    assert st == ost == 0 and index.block_metas() == ometas
    _par_chains(tmp_path, iz, fz)


def _par_chains(tmp_path, iz: bytes, fz: bytes):
    p = tmp_path / "payloads.bin"
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
st, index = ctx.decode_index(iz, ob.ZLIB)
assert st == 0
g = ctx.bloom_decode(fz, ob.ZLIB)
assert g[0] == 0
print("ok")
""" % (REPO, os.path.join(REPO, "slatedb-go_amd"), str(p))
    env = dict(os.environ, SLATE_HOST_TRACE="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout[-2000:] + r.stderr[-2000:]
    print("\n" + "\n".join(ln for ln in r.stderr.splitlines() if ln.startswith("[slate zlib-par]")))
    chains = [ln for ln in r.stderr.splitlines() if ln.startswith("[slate zlib-par]") and "candidates" in ln]
    # the index and the filter (and the filter again if the binding's first capacity was short)
    assert len(chains) >= 2 and all("fail 0" in ln for ln in chains), r.stderr[-3000:]


@pytest.mark.parametrize("level,strategy", [(1, zlib.Z_DEFAULT_STRATEGY), (9, zlib.Z_DEFAULT_STRATEGY),
                                            (6, zlib.Z_FILTERED), (6, zlib.Z_HUFFMAN_ONLY), (6, zlib.Z_RLE),
                                            (6, zlib.Z_FIXED), (0, zlib.Z_DEFAULT_STRATEGY)])
def test_zlib_levels_and_strategies(ctx, sst_parts, level, strategy):
    """Every zlib level band and strategy: fixed-Huffman blocks (decoded by the walk), stored blocks
    (level 0, incompressible filter bits), Huffman-only and RLE streams."""
    ib, fb = sst_parts
    for raw in (ib[:700_000], fb[:400_000]):
        assert _check_filter(ctx, _zlib(raw, level, strategy)) == 0


@pytest.mark.parametrize("kind", ["zeros", "random", "pattern", "text"])
def test_zlib_shapes(ctx, kind):
    """Stream shapes: very long runs (blocks of 16 k maximal matches), incompressible data (stored
    blocks), short matches with mixed distances reaching across block boundaries, text."""
    rng = np.random.default_rng(5)
    if kind == "zeros":
        raw = bytes(3_000_000)
    elif kind == "random":
        raw = rng.integers(0, 256, 1_500_000, dtype=np.uint8).tobytes()
    elif kind == "pattern":
        unit = rng.integers(0, 256, 900, dtype=np.uint8)
        parts = []
        for i in range(4000):
            u = unit.copy()
            u[rng.integers(0, 900, 9)] = rng.integers(0, 256, 9, dtype=np.uint8)
            parts.append(u[: 200 + (i * 53) % 700].tobytes())
        raw = b"".join(parts)
    else:
        words = [bytes(rng.integers(97, 123, int(rng.integers(2, 9)), dtype=np.uint8)) for _ in range(3000)]
        raw = b" ".join(words[int(i)] for i in rng.integers(0, 3000, 400_000))
    for level in (1, 6):
        assert _check_filter(ctx, _zlib(raw, level)) == 0


def test_zlib_small_window_and_headers(ctx, sst_parts):
    """Smaller windows (CINFO < 7) and the FDICT header (the exact path reports it)."""
    ib, _ = sst_parts
    for wbits in (9, 12, 15):
        assert _check_filter(ctx, _zlib(ib[:300_000], 6, wbits=wbits)) == 0
    z = bytearray(_zlib(ib[:300_000])[:-4])
    z[1] |= 0x20
    z[1] = (z[1] & 0xE0) | (31 - ((z[0] << 8) | (z[1] & 0xE0)) % 31) % 31
    assert _check_filter(ctx, sstgen.crc(bytes(z))) != 0


def test_zlib_damaged(ctx, sst_parts):
    """Flipped bits under a valid CRC, a wrong Adler-32, a truncated stream and bytes after the
    trailer: the statuses (and, where a stream still decodes, the bytes) are the oracle's."""
    rng = random.Random(7)
    ib, fb = sst_parts
    base = [_zlib(ib[:400_000])[:-4], _zlib(fb[:200_000])[:-4]]
    for trial in range(24):
        body = bytearray(base[trial % 2])
        kind = trial % 6
        if kind == 0:
            body[-1] ^= 0x01  # Adler-32
        elif kind == 1:
            body = body[: len(body) - rng.randrange(5, 400)]  # truncated
        elif kind == 2:
            body += bytes(rng.randrange(1, 9))  # bytes after the trailer (not read by the reader)
        else:
            for _ in range(rng.randint(1, 3)):
                body[rng.randrange(2, len(body) - 4)] ^= 1 << rng.randrange(8)
        _check_filter(ctx, sstgen.crc(bytes(body)))
