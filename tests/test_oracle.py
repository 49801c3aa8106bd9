"""Pins the CPU oracle (oracle/slate_oracle.c) before it is trusted as the checker.

1. Every known-answer vector from the reference's own tests
   (tests/golden/reference_vectors.json, file:line cited there).
2. Double entry: the C restatement vs the independent Python restatement
   (oracle/pyoracle.py) on seeded random inputs.
3. Non-authoritative cross-checks of the restated golang/snappy against the C++
   libsnappy 1.1.8 shipped in /opt/conda (decode must accept its output; encoded
   bytes are compared for information only where the algorithms coincide).
"""
import ctypes
import os
import random
import struct
import zlib

import numpy as np
import pytest

from oracle import pyoracle as py

H = "0123456789abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ" * 4
PREFIX200 = H[:200]


def test_status_strings_match(oracle):
    """The oracle's status enum and strings are the same as the product header's."""
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "slatecodec.h")).read()
    import re
    codes = dict((m.group(1), int(m.group(2))) for m in re.finditer(r"SLATE_(E_\w+|OK) = (\d+)", hdr))
    assert codes["OK"] == 0 and codes["E_SNAPPY_CORRUPT"] == 11 and codes["E_ROW_VALUE"] == 26
    for name, val in codes.items():
        if val < 100:  # >= 100 are C-ABI runtime conditions with no Go counterpart
            assert oracle.status_string(val) != "unknown status", name


# ------------------------------------------------------------ reference vectors
def test_compute_probes(oracle, ref_vectors):
    v = ref_vectors["compute_probes"]
    assert oracle.bloom_probes(int(v["hash"], 16), v["num_probes"], v["filter_bits"]) == v["expected"]
    assert py.probes_for_key(int(v["hash"], 16), v["num_probes"], v["filter_bits"]) == v["expected"]


def test_filter_has_key(oracle, ref_vectors):
    v = ref_vectors["filter_has_key"]
    k, bits = oracle.bloom_build([s.encode() for s in v["add"]], v["bits_per_key"])
    assert k == 6  # uint16(float32(10)*0.69)
    for s in v["present"]:
        assert oracle.bloom_has_key(k, bits, s.encode())
    for s in v["absent"]:
        assert not oracle.bloom_has_key(k, bits, s.encode())
    assert (k, bits) == py.bloom_build([s.encode() for s in v["add"]], v["bits_per_key"])


def test_num_probes_and_filter_bytes(oracle):
    assert oracle.bloom_optimal_num_probes(10) == 6 == py.optimal_num_probes(10)
    assert oracle.bloom_optimal_num_probes(20) == 13 == py.optimal_num_probes(20)
    for bpk in range(0, 40):
        assert oracle.bloom_optimal_num_probes(bpk) == py.optimal_num_probes(bpk)
    assert oracle.bloom_filter_bytes(8, 10) == 10
    assert oracle.bloom_filter_bytes(10_000_000, 10) == 12_500_000


def test_set_bit_cases(oracle, ref_vectors):
    # setBit semantics (LSB-first within a byte) through HasKey on a crafted filter
    for c in ref_vectors["set_bit"]:
        buf = bytearray(c["buf"])
        buf[c["bit"] // 8] |= 1 << (c["bit"] % 8)
        assert list(buf) == c["expected"]


def test_filter_effective(oracle, ref_vectors):
    v = ref_vectors["filter_effective"]
    keys = [struct.pack(">I", i) for i in range(v["n"])]
    k, bits = oracle.bloom_build(keys, v["bits_per_key"])
    assert all(oracle.bloom_has_key(k, bits, x) for x in keys[:2000])
    fp = sum(oracle.bloom_has_key(k, bits, struct.pack(">I", i)) for i in range(v["n"], 2 * v["n"]))
    assert fp / v["n"] < v["max_fp_rate"]


def test_filter_encoded_len(oracle, ref_vectors):
    for c in ref_vectors["filter_encoded_len"]:
        b = oracle.SstBuilder(4096, 0, c["bits_per_key"], oracle.NONE)
        for key in c["keys"]:
            assert b.add_value(key.encode(), c["value"].encode()) == 0
        assert b.build() == 0
        k, bits = b.bloom()
        assert len(oracle.bloom_encode(k, bits, oracle.NONE)) == c["expected_len"]
        assert b.info()["filter_len"] == c["expected_len"]


def test_estimate_block_size(oracle, ref_vectors):
    v = ref_vectors["estimate_block_size"]
    bb = oracle.BlockBuilder(4096)
    assert bb.is_empty()
    assert bb.add_value(v["key"].encode(), v["value"].encode())
    data, offs, fk = bb.build()
    st, enc = oracle.block_encode(data, offs, oracle.NONE)
    assert st == 0
    assert len(enc) == v["expected_len"] == oracle.v0_estimate_block_size([(b"k", b"v")])
    assert enc.hex() == v["derived_block_hex"]


def test_row_decode_errors(oracle, ref_vectors):
    for c in ref_vectors["row_decode_errors"]:
        r = oracle.v0_decode(bytes(c["input"]), None)
        assert c["error"] in oracle.status_string(r.status), c["name"]
        assert py.v0_decode(bytes(c["input"]), None)[0] == r.status


def test_row_peek_errors(oracle, ref_vectors):
    for c in ref_vectors["row_peek_errors"]:
        st, _, _ = oracle.v0_peek(bytes(c["input"]), None)
        assert c["error"] in oracle.status_string(st), c["name"]


def test_row_roundtrip(oracle, ref_vectors):
    for c in ref_vectors["row_roundtrip"]:
        val = c["value"].encode() if c["value"] is not None else None
        enc = oracle.v0_encode(c["prefix_len"], c["suffix"].encode(), val, c["seq"], c["expire_ms"], c["create_ms"])
        assert enc == py.v0_encode(c["prefix_len"], c["suffix"].encode(), val, c["seq"], c["expire_ms"],
                                   c["create_ms"])
        r = oracle.v0_decode(enc, len(c["first_key"].encode()))
        assert r.status == 0, c["name"]
        assert (r.key_prefix_len, r.key_suffix, r.seq) == (c["prefix_len"], c["suffix"].encode(), c["seq"])
        assert r.tombstone == (val is None)
        assert (r.expire_ms, r.create_ms) == (c["expire_ms"], c["create_ms"])
        if val is not None:
            assert r.value == val


def test_compute_prefix(oracle, ref_vectors):
    for c in ref_vectors["compute_prefix"]:
        if "lhs_str" in c:
            def mk(s):
                if s.startswith("P*"):
                    return (PREFIX200 * int(s[2])).encode() + s[3:].encode()
                return s.encode()
            a, b = mk(c["lhs_str"]), mk(c["rhs_str"])
        else:
            a, b = bytes(c["lhs"]), bytes(c["rhs"])
        assert oracle.compute_prefix_len(a, b) == c["expected"]
        assert py.compute_prefix_len(a, b) == c["expected"]
    # uint16 truncation
    big = b"x" * 70000
    assert oracle.compute_prefix_len(big, big) == 70000 & 0xFFFF


def _corrupt(enc: bytes, mutation: str) -> bytes:
    d = bytearray(enc)
    if mutation == "truncate5":
        return bytes(d[:5])
    if mutation == "last_byte_plus_one":
        d[-1] = (d[-1] + 1) & 0xFF
        return bytes(d)
    if mutation == "count_65535_recrc":
        d[-6:-4] = struct.pack(">H", 65535)
    elif mutation == "last_offset_65535_recrc":
        d[-8:-6] = struct.pack(">H", 65535)
    elif mutation == "count_0_recrc":
        d[-6:-4] = struct.pack(">H", 0)
    body = bytes(d[:-4])
    return body + struct.pack(">I", zlib.crc32(body))


def test_corrupt_block(oracle, ref_vectors):
    v = ref_vectors["corrupt_block"]
    bb = oracle.BlockBuilder(v["block_size"])
    for k, val in v["kvs"]:
        assert bb.add_value(k.encode(), val.encode())
    data, offs, _ = bb.build()
    st, enc = oracle.block_encode(data, offs, oracle.NONE)
    for c in v["cases"]:
        bad = _corrupt(enc, c["mutation"])
        meta, _, _ = oracle.block_decode(bad, oracle.NONE)
        assert c["error"] in oracle.status_string(meta["status"]), c["name"]
        assert py.block_decode(bad, oracle.NONE)[0] == meta["status"]
    # detail fields for the %d errors
    meta, _, _ = oracle.block_decode(_corrupt(enc, "count_65535_recrc"), oracle.NONE)
    assert meta["detail"] == len(enc) - 4 - 2 - 2 * 65535
    meta, _, _ = oracle.block_decode(_corrupt(enc, "last_offset_65535_recrc"), oracle.NONE)
    assert (meta["aux"], meta["detail"]) == (1, 65535)


def test_block_roundtrips(oracle, ref_vectors):
    for c in ref_vectors["block_roundtrips"]:
        bb = oracle.BlockBuilder(c["block_size"])
        pb = py.BlockBuilder(c["block_size"])
        for k, val in c["kvs"]:
            v = val.encode() if val is not None else b""
            assert bb.add_value(k.encode(), v)
            assert pb.add_value(k.encode(), v)
        data, offs, fk = bb.build()
        assert (data, offs, fk) == (bytes(pb.data), pb.offsets, pb.first_key)
        assert fk == c["first_key"].encode()
        if c.get("offsets_ascending"):
            assert all(offs[i] > offs[i - 1] for i in range(1, len(offs)))
        for codec in (oracle.NONE, oracle.SNAPPY):
            st, enc = oracle.block_encode(data, offs, codec)
            assert st == 0 and enc == py.block_encode(data, offs, codec)
            meta, buf, rows = oracle.block_decode(enc, codec)
            assert meta["status"] == 0
            assert buf[: meta["data_len"]] == data
            assert list(rows["row_off"]) == offs
            assert meta["aux"] == 0  # FirstKey quirk: v0 row 0 has prefixLen 0 => empty FirstKey
            # rows decode back to the kvs (first key full, rest prefix-compressed)
            for i, (k, val) in enumerate(c["kvs"]):
                r = rows[i]
                assert r["status"] == 0
                suffix = buf[r["row_off"] + 4: r["row_off"] + 4 + r["key_suffix_len"]]
                assert fk[: r["key_prefix_len"]] + suffix == k.encode()
                vs = r["row_off"] + 4 + r["key_suffix_len"] + r["meta_len"]
                if val is None:
                    assert r["flags"] & 1
                else:
                    assert buf[vs: vs + r["value_len"]] == val.encode()


def test_block_builder_cases(oracle, ref_vectors):
    v = ref_vectors["make_blocks_available"]
    b = oracle.SstBuilder(v["block_size"], 0, 10, oracle.NONE)
    for k, val in v["adds1"]:
        assert b.add_value(k.encode(), val.encode()) == 0
    for expect in v["blocks1"]:
        blk = b.next_block()
        _, buf, rows = oracle.block_decode(blk, oracle.NONE)
        assert [buf[r["row_off"] + 4: r["row_off"] + 4 + r["key_suffix_len"]] for r in rows] == \
            [e.encode() for e in expect]
    assert b.next_block() is None
    for k, val in v["adds2"]:
        assert b.add_value(k.encode(), val.encode()) == 0
    blk = b.next_block()
    _, buf, rows = oracle.block_decode(blk, oracle.NONE)
    assert len(rows) == 1 and buf[4:12] == v["blocks2"][0][0].encode()
    assert b.next_block() is None


def _sst_blocks(oracle, sst: bytes, info: dict):
    st, metas = oracle.decode_index(sst[info["index_offset"]: info["index_offset"] + info["index_len"]],
                                    info["codec"])
    assert st == 0
    out = []
    for i, (off, fk) in enumerate(metas):
        end = metas[i + 1][0] if i + 1 < len(metas) else info["filter_offset"]
        meta, buf, rows = oracle.block_decode(sst[off:end], info["codec"])
        assert meta["status"] == 0
        first = None
        keys = []
        for r in rows:
            sfx = buf[r["row_off"] + 4: r["row_off"] + 4 + r["key_suffix_len"]]
            if first is None:
                first = sfx
            keys.append(first[: r["key_prefix_len"]] + sfx)
        assert keys[0] == fk
        out.append(keys)
    return out


@pytest.mark.parametrize("name", ["read_blocks_52", "read_all_blocks"])
def test_read_blocks_layout(oracle, ref_vectors, name):
    v = ref_vectors[name]
    bs = v.get("block_size") or oracle.v0_estimate_block_size(
        [(k.encode(), x.encode()) for k, x in v["estimate_kvs"]])
    b = oracle.SstBuilder(bs, v["min_filter_keys"], 10, oracle.NONE)
    for k, val in v["kvs"]:
        b.add_value(k.encode(), val.encode())
    assert b.build() == 0
    sst = b.encode_table()
    st, info = oracle.sst_read_info(sst)
    assert st == 0 and info == b.info()
    assert _sst_blocks(oracle, sst, info) == [[k.encode() for k in blk] for blk in v["blocks"]]


def test_encode_decode_sst(oracle, ref_vectors):
    v = ref_vectors["encode_decode_sst"]
    bs = oracle.v0_estimate_block_size([(b"key1", b"value1")])
    b = oracle.SstBuilder(bs, v["min_filter_keys"], v["bits_per_key"], oracle.NONE)
    for k, val in v["kvs"]:
        b.add_value(k.encode(), val.encode())
    b.build()
    sst = b.encode_table()
    st, info = oracle.sst_read_info(sst)
    assert st == 0 and info["first_key"] == b"key1"
    assert len(_sst_blocks(oracle, sst, info)) == v["n_blocks"]
    fst, k, bits = oracle.bloom_decode(sst[info["filter_offset"]: info["filter_offset"] + info["filter_len"]],
                                       info["codec"])
    assert fst == 0
    for key, _ in v["kvs"]:
        assert oracle.bloom_has_key(k, bits, key.encode())


def test_dump_layout_derived(oracle, ref_vectors):
    v = ref_vectors["dump_layout_derived"]
    bs = oracle.v0_estimate_block_size([(b"key1", b"value1")])
    assert bs == 35
    b = oracle.SstBuilder(bs, 0, 10, oracle.NONE)
    for k, val in v["kvs"]:
        b.add_value(k.encode(), val.encode())
    b.build()
    info = b.info()
    sst = b.encode_table()
    st, metas = oracle.decode_index(sst[info["index_offset"]: info["index_offset"] + info["index_len"]], 0)
    assert [m[0] for m in metas] == v["block_offsets"]
    assert info["filter_offset"] == v["filter_offset"]
    assert info["filter_len"] == v["filter_len_now"]
    assert info["index_offset"] == v["index_offset_now"]
    k, bits = b.bloom()
    assert k == v["num_probes"] and len(bits) == v["filter_data_len"]
    # The stale docstring predates the index CRC: its "Index Length: 168" is the
    # flatbuffer SsTableIndex alone, which pins the Go-builder layout restated here.
    assert info["index_len"] - 4 == v["dump_stale"]["index_len"]


# ------------------------------------------------------ C vs Python (double entry)
def _rand_kvs(rng, n, klen=(1, 24), vlen=(0, 120), tomb_p=0.1):
    keys = sorted({bytes(rng.getrandbits(8) for _ in range(rng.randint(*klen))) for _ in range(n)})
    kvs = []
    for k in keys:
        if rng.random() < tomb_p:
            kvs.append((k, b""))
        else:
            kvs.append((k, bytes(rng.getrandbits(8) for _ in range(rng.randint(*vlen)))))
    return kvs


@pytest.mark.parametrize("seed", range(6))
def test_c_vs_python_sst(oracle, seed):
    rng = random.Random(seed)
    kvs = _rand_kvs(rng, rng.randint(1, 300))
    for codec in (oracle.NONE, oracle.SNAPPY):
        bs = rng.choice([64, 256, 1024, 4096])
        mfk = rng.choice([0, 10, 1000])
        bpk = rng.choice([1, 10, 20])
        cb = oracle.SstBuilder(bs, mfk, bpk, codec)
        pb = py.SstBuilder(bs, mfk, bpk, codec)
        for k, v in kvs:
            assert cb.add_value(k, v) == 0
            pb.add_value(k, v)
        assert cb.build() == 0
        pb.build()
        assert cb.encode_table() == pb.encode_table()


@pytest.mark.parametrize("seed", range(20))
def test_snappy_c_vs_python(oracle, seed):
    rng = random.Random(100 + seed)
    n = rng.choice([0, 1, 5, 16, 17, 18, 100, 1000, 5000, 70000])
    alphabet = rng.choice([2, 4, 16, 256])
    src = bytes(rng.randrange(alphabet) for _ in range(n))
    if rng.random() < 0.5 and n > 64:
        src = src[: n // 2] * 2
    c = oracle.snappy_encode(src)
    assert c == py.snappy_encode(src)
    st, d = oracle.snappy_decode(c)
    assert st == 0 and d == src
    assert py.snappy_decode(c) == src


def test_snappy_decode_rejects(oracle):
    good = oracle.snappy_encode(b"hello hello hello hello hello hello")
    cases = [b"", b"\xff" * 11, good[:-1], good + b"\x00", b"\x05\x00\x00\x00\x00\x00\x00",
             b"\x04\x01\x05", b"\x10" + b"\x0d\x01", b"\x08\x00a\x09\x00", b"\x08\x04aa\x01\x00"]
    for c in cases:
        st, _ = oracle.snappy_decode(c)
        try:
            py.snappy_decode(c)
            pst = 0
        except py.SnappyCorrupt:
            pst = 11
        assert st == pst, c.hex()


# ------------------------------------------- libsnappy cross-check (non-authoritative)
def _libsnappy():
    for p in ("/opt/conda/lib/libsnappy.so.1", "/opt/conda/lib/libsnappy.so"):
        if os.path.exists(p):
            L = ctypes.CDLL(p)
            L.snappy_compress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                          ctypes.POINTER(ctypes.c_size_t)]
            L.snappy_max_compressed_length.restype = ctypes.c_size_t
            L.snappy_max_compressed_length.argtypes = [ctypes.c_size_t]
            return L
    return None


# Inputs on which the restated golang/snappy v0.0.4 encoder and C++ libsnappy 1.1.8 may
# legitimately differ (an explicit allow-list: none so far; golang/snappy emits the same bytes
# as C++ snappy by design).  Any other difference fails the test.
LIBSNAPPY_ALLOWED_DIFF: set[str] = set()


def test_snappy_cross_libsnappy(oracle):
    """Cross-check (not authority: golang/snappy itself is absent) of the restated encoder's
    bytes against C++ libsnappy on row-shaped inputs, plus random and repetitive buffers."""
    L = _libsnappy()
    if L is None:
        pytest.skip("libsnappy not present")
    rng = np.random.default_rng(7)
    inputs = []
    for i in range(40):
        r = rng.integers(0, 256, 42, dtype=np.uint8).tobytes()
        inputs.append((f"rows{i}", (b"\x00\x0e\x00\x02xy" + b"\x00" * 13 + b"\x54" + r + r) * (1 + i)))
    for i, n in enumerate((0, 1, 16, 17, 100, 4096, 65536, 65537, 200_000)):
        inputs.append((f"rand{i}", rng.integers(0, 256, n, dtype=np.uint8).tobytes()))
        inputs.append((f"rep{i}", bytes(rng.integers(0, 4, n, dtype=np.uint8))))
    diff = []
    for name, src in inputs:
        out = ctypes.create_string_buffer(L.snappy_max_compressed_length(len(src)))
        ol = ctypes.c_size_t(len(out))
        assert L.snappy_compress(src, len(src), out, ctypes.byref(ol)) == 0
        lib_bytes = out.raw[: ol.value]
        st, d = oracle.snappy_decode(lib_bytes)
        assert st == 0 and d == src  # the restated golang decoder accepts C++ snappy output
        if lib_bytes != oracle.snappy_encode(src) and name not in LIBSNAPPY_ALLOWED_DIFF:
            diff.append(name)
    assert not diff, f"restated golang/snappy encoder differs from libsnappy on {diff}"


def test_go_shaped_zlib_stream(oracle):
    """tests/sstgen.go_zlib (the stream shape Go's compress/zlib closes with, used by the GPU
    zlib-par tests): zlib reads it back, its last deflate block is an empty final stored block, and
    the oracle's bloom reader (compression.go:134-140 under bloom.go:70-91) decodes it."""
    from tests import sstgen
    rng = np.random.default_rng(3)
    raw = rng.integers(0, 3, 200_000, dtype=np.uint8).tobytes()
    z = sstgen.go_zlib(raw, 6)
    assert zlib.decompress(z) == raw and z[-8:-4] == b"\x00\x00\xff\xff"
    d = zlib.decompressobj(-15)
    assert d.decompress(z[2:-4]) == raw and d.eof and not d.unused_data  # ends at the stored block
    st, *_ = oracle.bloom_decode(sstgen.crc(z), oracle.ZLIB, cap=1 << 22)
    assert st == 0
