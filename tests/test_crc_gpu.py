"""crc32.ChecksumIEEE of device bytes (slate_crc32_device: the stripe-parallel CRC the SST builder
runs over filter and index payloads, csrc/encode.hip crc_stripes_kernel + crc_join_kernel) against
zlib.crc32 (= Go's crc32.ChecksumIEEE): every alignment of the first byte, lengths around the
16-byte chunk, 4 KiB stripe and 64-stripe boundaries, and a filter-sized 12.5 MB buffer."""
import ctypes as C
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    import slatecodec as sc
    return sc.Context(0)


def _crc(ctx, buf, off, n):
    import slatecodec as sc
    c = C.c_uint32()
    st = sc.lib().slate_crc32_device(ctx.handle, C.c_void_p(buf.ptr + off), n, C.byref(c))
    assert st == 0, st
    return c.value


def test_crc_lengths_and_alignments(ctx):
    import slatecodec as sc
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, 300_000, dtype=np.uint8)
    d = sc.devbuf_from(ctx, data)
    lens = [0, 1, 3, 4, 5, 15, 16, 17, 31, 32, 33, 63, 64, 65, 4095, 4096, 4097, 4111, 8191, 8192, 12288 + 7,
            64 * 4096 - 1, 64 * 4096, 64 * 4096 + 19, 270_000]
    for sh in range(16):
        for n in lens:
            want = zlib.crc32(data[sh:sh + n].tobytes())
            assert _crc(ctx, d, sh, n) == want, (sh, n)


def test_crc_filter_sized(ctx):
    import slatecodec as sc
    rng = np.random.default_rng(6)
    n = 12_500_003
    data = rng.integers(0, 256, n + 16, dtype=np.uint8)
    d = sc.devbuf_from(ctx, data)
    for sh in (0, 5, 13):
        assert _crc(ctx, d, sh, n) == zlib.crc32(data[sh:sh + n].tobytes()), sh
