"""Oracle pinning for the block/SST seek path: block.NewIteratorAtKey
(internal/sstable/block/iterator.go:31-82, firstFullKey :117-132) and
sstable.Iterator.firstBlockIncludingOrAfterKey (internal/sstable/iterator.go:123-153), against
the reference's own cases (block_test.go:112-245 seeks, :416-527 corrupted keys)."""
import random

from oracle import binding as ob


def _block(kvs, block_size=4096):
    bb = ob.BlockBuilder(block_size)
    for k, v in kvs:
        assert bb.add_value(k.encode(), (v or "").encode())
    data, offs, _ = bb.build()
    return bytearray(data), list(offs)


def iterate_from(data: bytes, offs: list[int], start: int, first_idx: int, first_len: int):
    """block.Iterator.Next from offsetIndex `start` with firstKey = row first_idx's suffix
    (iterator.go:84-107): (key, value) pairs until the first row that fails to decode."""
    fo = offs[first_idx] + 4
    fk = bytes(data[fo:fo + first_len])
    out = []
    for i in range(start, len(offs)):
        r = ob.v0_decode(bytes(data[offs[i]:]), len(fk))
        if r.status:
            break
        out.append((fk[:r.key_prefix_len] + r.key_suffix, None if r.tombstone else r.value))
    return out


def test_iterator_seek_vectors(ref_vectors):
    v = ref_vectors["iterator_seek"]
    data, offs = _block(v["kvs"], 1024)
    for c in v["cases"]:
        st, start, fi, fl, nw = ob.block_seek(bytes(data), offs, c["key"].encode())
        assert (st, start, nw) == (0, c["start"], 0), c
        got = iterate_from(data, offs, start, fi, fl)
        assert [k.decode() for k, _ in got] == [k for k, _ in v["kvs"]][c["start"]:]


def test_iterator_seek_corrupted_keys(ref_vectors):
    for c in ref_vectors["iterator_seek_corrupt"]:
        data, offs = _block(c["kvs"])
        for r in c["corrupt"]:
            data[0 if r == "data0" else offs[r]] = 0xFF
        st, start, fi, fl, nw = ob.block_seek(bytes(data), offs, c["key"].encode())
        if "error" in c:
            assert st == 63 and ob.status_string(st) == c["error"], c["name"]
            continue
        assert st == 0, c["name"]
        assert (nw > 0) == c["warnings"], c["name"]
        got = iterate_from(data, offs, start, fi, fl)
        assert [(k.decode(), v.decode()) for k, v in got] == [tuple(x) for x in c["next"]], c["name"]


def test_seek_no_offsets():
    st, *_ = ob.block_seek(b"\0\0\0\0", [], b"k")
    assert st == 62 and ob.status_string(st) == "number of block.Offsets must be greater than zero"


def test_index_seek_cases():
    keys = [b"b", b"d", b"f"]
    # before the first block's key -> 0; equal -> that block; between -> the block before; after -> last
    for k, want in ((b"a", 0), (b"b", 0), (b"c", 0), (b"d", 1), (b"e", 1), (b"f", 2), (b"z", 2), (b"", 0)):
        assert ob.index_seek(keys, k) == want, k
    assert ob.index_seek([], b"x") == 0


def test_index_seek_matches_bisect():
    """On sorted first keys the Go loop equals 'last block whose first key <= key' (0 if none)."""
    import bisect
    rng = random.Random(5)
    for _ in range(200):
        keys = sorted({rng.randbytes(rng.randint(1, 6)) for _ in range(rng.randint(1, 40))})
        k = rng.randbytes(rng.randint(0, 6))
        assert ob.index_seek(keys, k) == max(0, bisect.bisect_right(keys, k) - 1)


WARN_FORMATS = {1: "while peeking at key at offset {a}: {err}", 2: "unable to locate uncorrupted first key in block; "
                "block is corrupt", 3: "block.Offset[{a}] = {b} is out of bounds", 4: "while peeking at block.Offset[{a}]: {err}"}


def render_warnings(warns) -> str:
    """types.ErrWarn.Error() (internal/types/errors.go:13-15) rebuilt from the warning records the
    C-ABI returns (slate_seek_warn), as the cgo shim in INTEGRATION.md does."""
    return "\n".join(WARN_FORMATS[k].format(a=a, b=b, err=ob.status_string(e)) for k, e, a, b in warns)


def test_iterator_seek_warning_text(ref_vectors):
    """The warning records reproduce the reference's ErrWarn text: the 'unable to locate' error of
    the all-corrupt cases (block_test.go:416-466) and the first-key recovery warnings (:468-527)."""
    for c in ref_vectors["iterator_seek_corrupt"]:
        data, offs = _block(c["kvs"])
        for r in c["corrupt"]:
            data[0 if r == "data0" else offs[r]] = 0xFF
        (st, start, fi, fl, nw), warns = ob.block_seek_warnings(bytes(data), offs, c["key"].encode())
        assert len(warns) == nw, c["name"]
        text = render_warnings(warns)
        if "error" in c:
            assert c["error"] in text and warns[-1][0] == 2, c["name"]
        elif c["warnings"]:
            assert nw > 0 and all(": corrupt v0 row: " in line for line in text.split("\n")), (c["name"], text)
            if 0 in c["corrupt"] or "data0" in c["corrupt"]:
                # firstFullKey skipped the corrupted first row: its 0xFF prefix-length byte
                assert warns[0][0] == 1 and warns[0][2] == offs[0], c["name"]
                assert text.startswith(f"while peeking at key at offset {offs[0]}: corrupt v0 row: "), text
            else:  # sort.Search peeked at a corrupted row
                assert warns[0][0] == 4, c["name"]
        else:
            assert nw == 0 and text == "", c["name"]
