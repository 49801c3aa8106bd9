"""GPU executeCompaction for the SST codec path (slatecodec.compaction.compact: device decode of
every input block -> full-key rows -> MergeSort -> gather -> SST builder, cut at MaxSSTSize) against
the oracle's restatement of the same loop (tests/compactgen.py): output SST bytes bit-exact.
Cases: L0 SSTs with overlapping keys and tombstones, sorted runs of several SSTs, Snappy inputs
and outputs, an output split into many SSTs, keys with skewed shared prefixes."""
import random

import pytest

from oracle import binding as ob
from tests import compactgen as cg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import slatecodec as sc
    return sc.Context(0)


@pytest.fixture(params=["c_abi", "steps"])
def compact_fn(request):
    """slate_compact (one C-ABI call) and the same chain step by step on slate_devbufs."""
    from slatecodec import compaction
    return compaction.compact if request.param == "c_abi" else compaction.compact_steps


@pytest.mark.parametrize("seed,n_src,n_keys,space,codec,run_ssts,max_size,out_codec", [
    (1, 3, 400, 900, ob.NONE, 1, 1 << 30, ob.NONE),
    (2, 4, 1500, 3000, ob.SNAPPY, 1, 1 << 30, ob.SNAPPY),
    (3, 2, 3000, 5000, ob.NONE, 3, 40_000, ob.NONE),
    (4, 5, 800, 1200, ob.SNAPPY, 2, 9_000, ob.NONE),
    (5, 1, 2000, 2000, ob.NONE, 4, 1 << 30, ob.SNAPPY),
])
def test_compaction_bit_exact(ctx, compact_fn, seed, n_src, n_keys, space, codec, run_ssts, max_size, out_codec):
    rng = random.Random(seed)
    srcs = cg.random_sources(rng, n_src, n_keys, space, codec=codec, run_ssts=run_ssts)
    got = compact_fn(ctx, srcs, max_size, codec=out_codec)
    want = cg.oracle_compact(srcs, max_size, codec=out_codec)
    assert len(got) == len(want)
    for i, (g, w) in enumerate(zip(got, want)):
        assert g == w, f"output SST {i}"


def test_compaction_skewed_prefixes(ctx):
    from slatecodec import compaction
    rng = random.Random(9)
    # shared-prefix lengths from a few bytes to ~70 (past the merge's 16-byte key head)
    def key(i):
        return b"t" + b"/" * (i % 7) * (i % 11) + b"%08d" % i
    srcs = cg.random_sources(rng, 3, 600, 1500, key_fmt=key)
    got = compaction.compact(ctx, srcs, 20_000)
    assert got == cg.oracle_compact(srcs, 20_000)


def test_compaction_many_snappy_ssts(ctx):
    """More input SSTs than index-decode workers (8), all with Snappy indexes: each worker owns
    its context for a contiguous slice of the SST list."""
    from slatecodec import compaction
    rng = random.Random(21)
    srcs = cg.random_sources(rng, 4, 1200, 2500, codec=ob.SNAPPY, run_ssts=5)
    assert sum(len(r) for r in srcs) > 8
    got = compaction.compact(ctx, srcs, 30_000, codec=ob.SNAPPY)
    assert got == cg.oracle_compact(srcs, 30_000, codec=ob.SNAPPY)


def test_compaction_mixed_codecs(ctx, compact_fn):
    """Each SST carries its own codec (sstable.Info.CompressionCodec): a DB whose compression
    option changed has L0 SSTs and sorted runs in different codecs."""
    rng = random.Random(22)
    srcs = []
    for j, codec in enumerate((ob.NONE, ob.SNAPPY, ob.NONE, ob.SNAPPY)):
        srcs += cg.random_sources(rng, 1, 700, 1600, codec=codec, run_ssts=1 + j % 3)
    got = compact_fn(ctx, srcs, 1 << 30, codec=ob.SNAPPY)
    assert got == cg.oracle_compact(srcs, 1 << 30, codec=ob.SNAPPY)


def _corrupt_first_block(sst: bytes, body: bytes) -> bytes:
    """Replace the SST's first data block by `body` (padded to the block's length) + a valid CRC."""
    import struct
    import zlib
    st, info = ob.sst_read_info(sst)
    st, metas = ob.decode_index(sst[info["index_offset"]:info["index_offset"] + info["index_len"]], info["codec"])
    a = metas[0][0]
    b = metas[1][0] if len(metas) > 1 else info["filter_offset"]
    body = (body + b"\0" * (b - a))[: b - a - 4]
    return sst[:a] + body + struct.pack(">I", zlib.crc32(body)) + sst[b:]


@pytest.mark.parametrize("body,status", [
    (b"\x00", 11),       # Snappy header says 0 bytes, more input follows: snappy: corrupt input
    (b"\x01\x00a", 11),  # decoded length 1 (no row slot) with trailing input
    (None, 2),           # CRC mismatch
])
def test_compaction_bad_block_fails(ctx, compact_fn, body, status):
    """A block that fails block.Decode stops the compaction (sstable.Iterator returns the error,
    executeCompaction returns it: iterator.go:62-68, executor.go:107-150), also when the block
    fails before it owns a row slot."""
    from slatecodec import SlateError
    rng = random.Random(23)
    srcs = cg.random_sources(rng, 2, 600, 1200, codec=ob.SNAPPY)
    if body is None:
        s = bytearray(srcs[1][0])
        s[20] ^= 0x40
        srcs[1][0] = bytes(s)
    else:
        srcs[1][0] = _corrupt_first_block(srcs[1][0], body)
    with pytest.raises(SlateError) as e:
        compact_fn(ctx, srcs, 1 << 30)
    assert e.value.status == status


def test_compaction_empty_and_capacity(ctx):
    """No input entries: no output SST; out_cap smaller than the outputs: SLATE_E_CAPACITY with the
    count needed (the binding then retries with enough room)."""
    from slatecodec import compaction
    assert compaction.compact(ctx, [[]], 1 << 30) == []
    rng = random.Random(31)
    srcs = cg.random_sources(rng, 2, 2000, 3000)
    got = compaction.compact(ctx, srcs, 2_000)  # > 16 outputs: the first call reports the count
    want = cg.oracle_compact(srcs, 2_000)
    assert len(want) > 16 and got == want


def _corrupt_row(sst: bytes, block: int, row: int, field: int = 0) -> bytes:
    """CodecNone SST: row `row` of data block `block` gets a key prefix longer than the block's first
    key (field 0, row.go:203-206) or a key suffix longer than the block (field 2, :208-211): a corrupt
    v0 row; the block's CRC32 re-sealed."""
    import struct
    import zlib
    st, info = ob.sst_read_info(sst)
    assert info["codec"] == ob.NONE
    st, metas = ob.decode_index(sst[info["index_offset"]:info["index_offset"] + info["index_len"]], info["codec"])
    offs = [o for o, _ in metas] + [info["filter_offset"]]
    a, b = offs[block], offs[block + 1]
    m, data, rows = ob.block_decode(sst[a:b], ob.NONE)
    body = bytearray(sst[a:b - 4])
    o = int(rows[row]["row_off"])
    body[o + field:o + field + 2] = b"\xff\xff"
    return sst[:a] + bytes(body) + struct.pack(">I", zlib.crc32(bytes(body))) + sst[b:]


@pytest.mark.parametrize("case", ["block", "row", "both", "first_row", "run", "dup"])
def test_compaction_corrupt_inputs_warn(ctx, case):
    """Corrupt inputs end iterators as Go's do and the compaction goes on (sstable.Iterator,
    block.Iterator, iter.MergeSort, executeCompaction returning warn.If()): the output SSTs are
    built from the rows Go still returns, and slate_compact_ex reports one warning record per
    ErrWarn entry, in Go's order -- against the oracle restated with the same iterator rules."""
    import slatecodec as sc
    rng = random.Random(41)
    srcs = cg.random_sources(rng, 3, 900, 2000, run_ssts=2 if case == "run" else 1)
    if case in ("block", "both"):
        srcs[1][0] = _corrupt_first_block(srcs[1][0], b"\x00")  # CodecNone: 1 byte "block": too small
    if case in ("row", "both"):
        srcs[2][0] = _corrupt_row(srcs[2][0], 1, 5)
    if case == "first_row":  # before source 0's first row (merged when the merge starts), then source 1's
        srcs[0][0] = _corrupt_row(srcs[0][0], 0, 0, field=2)
        srcs[1][0] = _corrupt_row(srcs[1][0], 2, 7)
    if case == "dup":  # the same row index and status in two sources: Go's ErrWarn keeps one text
        srcs[1][0] = _corrupt_row(srcs[1][0], 1, 5)
        srcs[2][0] = _corrupt_row(srcs[2][0], 2, 5)
    if case == "run":  # the second SST of source 0's run: its first block, then a row of source 2
        srcs[0][1] = _corrupt_first_block(srcs[0][1], b"\x00")
        srcs[2][1] = _corrupt_row(srcs[2][1], 2, 3)
    got, warns = sc.compact_ex(ctx, srcs, 30_000)
    want, want_w = cg.oracle_compact_go(srcs, 30_000)
    assert len(want_w) >= 1
    if case == "dup":
        assert len(want_w) == 1
    assert [tuple(int(x) for x in w) for w in warns] == [tuple(w) for w in want_w]
    assert len(got) == len(want) and all(g == w for g, w in zip(got, want))
    # slate_compact: the first warning's status, no outputs (startCompaction drops the sorted run)
    from slatecodec import SlateError
    with pytest.raises(SlateError) as e:
        sc.compact(ctx, srcs, 30_000)
    assert e.value.status == want_w[0][4]


@pytest.mark.parametrize("n_keys", [300, 4000])
def test_compaction_zlib_sources(ctx, compact_fn, n_keys):
    """Input SSTs in CodecZlib (built by this library's sstable.Builder; the oracle's reader decodes
    them): the compaction's decode takes the staged Zlib plan (phase Z once) when an input batch has
    >= 64 blocks; outputs bit-exact against the oracle's executeCompaction, in both output codecs."""
    import slatecodec as sc
    rng = random.Random(60 + n_keys)

    def gpu_sst(kvs):
        b = sc.SstBuilder(ctx, 4096, 0, 10, ob.ZLIB)
        for k, v in kvs:
            assert b.add(k, v) == 0
        return b.build().encode()

    srcs = []
    for kvs in cg.random_kv_runs(rng, 3, n_keys, 3 * n_keys, run_ssts=2):
        srcs.append([gpu_sst(part) for part in kvs])
    for out_codec in (ob.NONE, ob.SNAPPY):
        got = compact_fn(ctx, srcs, 1 << 30, codec=out_codec)
        assert got == cg.oracle_compact(srcs, 1 << 30, codec=out_codec)
