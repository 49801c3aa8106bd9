"""Profiling aid: opening a CodecZlib SST's index and filter written by a zlib-level encoder (no flush
points: the exact one-wave path) -- a 2 M-KV CodecNone SST's payloads recompressed with zlib level 6."""
import sys, time, zlib
sys.path[:0] = ['/root/repo', '/root/repo/slatedb-go_amd']
import slatecodec as sc
from oracle import binding as ob
from tests import sstgen
from tools.bench_encode import kv_arrays
ctx = sc.Context(0)
keys, key_off, vals, val_off = kv_arrays(2_000_000)
b = sc.SstBuilder(ctx, 4096, 0, 10, ob.NONE)
assert b.add_batch(keys, key_off, vals, val_off) == 0
sst = b.build().encode()
st, info, _ = sc.read_info(sst)
ib = sstgen.crc(zlib.compress(sst[info.index_offset:info.index_offset + info.index_len][:-4], 6))
fb = sstgen.crc(zlib.compress(sst[info.filter_offset:info.filter_offset + info.filter_len][:-4], 6))
for name, buf, fn in (("index", ib, lambda x: ctx.decode_index(x, ob.ZLIB)[0]), ("filter", fb, lambda x: ctx.bloom_decode(x, ob.ZLIB)[0])):
    fn(buf)
    t0 = time.perf_counter()
    s = fn(buf)
    print(f"zlib {name} {len(buf) / 1e6:.2f} MB encoded: status {s}, {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
