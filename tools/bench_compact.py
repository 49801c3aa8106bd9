"""Compaction measurement (tooling): executeCompaction's codec path on the GPU
(slatecodec.compaction: device block decode -> full-key rows -> MergeSort -> gather -> SST
builder) over k L0 SSTs of b"k%015d" keys / 84-byte V-half values sharing a key space.
Inputs are built by the GPU SST builder and handed over as host SST bytes (object-store GET
buffers); outputs are host SST bytes (PUT buffers).  Reports the wall time of the device stages
(decode .. gather, including their host syncs) and of the whole compaction, and checks a smaller
instance bit-exact against the oracle's restatement (tests/compactgen.py), whose time on one core
is the CPU baseline.  usage: python tools/bench_compact.py [--k 4] [--kv 1000000] [--codec snappy]"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "slatedb-go_amd")]


def make_sources(sc, ctx, k, kv, overlap, codec, seed=20250307):
    rng = np.random.default_rng(seed)
    space = int(kv * k * (1 - overlap) + kv)
    srcs = []
    for j in range(k):
        ids = np.sort(rng.choice(space, size=kv, replace=False))
        keys = np.zeros((kv, 16), np.uint8)
        keys[:, 0] = ord("k")
        v = ids.copy()
        for c in range(15, 0, -1):
            keys[:, c] = 48 + v % 10
            v //= 10
        r = rng.integers(0, 256, size=(kv, 42), dtype=np.uint8)
        vals = np.concatenate([r, r], axis=1)
        b = sc.SstBuilder(ctx, 4096, 0, 10, codec)
        assert b.add_batch(keys.reshape(-1), np.arange(kv + 1, dtype=np.uint64) * 16, vals.reshape(-1),
                           np.arange(kv + 1, dtype=np.uint64) * 84) == 0
        srcs.append([b.build().encode()])
    return srcs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--kv", type=int, default=1_000_000)
    ap.add_argument("--overlap", type=float, default=0.3)
    ap.add_argument("--codec", default="snappy", choices=["none", "snappy"])
    ap.add_argument("--max-sst", type=int, default=256 << 20)
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    import slatecodec as sc
    from slatecodec import compaction
    codec = sc.SNAPPY if args.codec == "snappy" else sc.NONE
    ctx = sc.Context(0)
    srcs = make_sources(sc, ctx, args.k, args.kv, args.overlap, codec)
    in_bytes = sum(len(s) for run in srcs for s in run)
    compaction.compact(ctx, srcs, args.max_sst, codec=codec)  # warm-up
    dev_s, all_s, stages = [], [], {}
    for _ in range(args.steps):
        ctx.synchronize()
        t0 = time.perf_counter()
        prof = []
        view, src_start = compaction.decode_rows_kv(ctx, srcs, prof)
        merged = compaction.merge_kv(ctx, view, src_start, prof)
        for (_, a), (lb, b) in zip(prof, prof[1:]):
            stages[lb] = min(stages.get(lb, 1e9), round(b - a, 5))
        ctx.synchronize()
        dev_s.append(time.perf_counter() - t0)
        del view, merged
        t0 = time.perf_counter()
        out = compaction.compact(ctx, srcs, args.max_sst, codec=codec)
        all_s.append(time.perf_counter() - t0)
    n_in = args.k * args.kv
    # parity + CPU baseline on a bounded instance (oracle restatement, one core)
    from tests import compactgen as cg
    rng = random.Random(1)
    small = cg.random_sources(rng, args.k, 20_000, 50_000, codec=codec)
    t0 = time.perf_counter()
    want = cg.oracle_compact(small, args.max_sst, codec=codec)
    cpu_s = time.perf_counter() - t0
    exact = compaction.compact(ctx, small, args.max_sst, codec=codec) == want
    print(json.dumps({
        "metric": "compaction (decode -> merge -> re-encode) input entries/s", "unit": "entries/s",
        "value_device_stages": round(n_in / min(dev_s)), "value_end_to_end": round(n_in / min(all_s)),
        "s_device_stages": round(min(dev_s), 4), "stage_s": stages, "s_end_to_end": round(min(all_s), 4),
        "config": {"sources": args.k, "kv_per_source": args.kv, "overlap": args.overlap, "codec": args.codec,
                   "input_sst_bytes": in_bytes, "output_ssts": len(out), "max_sst_size": args.max_sst},
        "bit_exact_vs_oracle_sample": exact,
        "cpu_baseline": {"value": round(args.k * 20_000 / cpu_s), "unit": "entries/s", "cores": 1, "kind": "port",
                         "sample": f"oracle restatement (tests/compactgen.py: C block decode, Python key "
                                   f"materialisation, C heap merge, C builder) on {args.k} x 20000 KV"},
    }))
    if not exact:
        sys.exit(1)


if __name__ == "__main__":
    main()
