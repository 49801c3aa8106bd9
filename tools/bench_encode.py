"""Encode measurement (tooling; BASELINE.json configs[2]): 10 M x 100 B KV -> SST blocks +
bloom through the GPU sstable.Builder (slate_sst_builder_add_batch + build), bit-exact
against the oracle's C restatement of the Go builder.

Workload: keys b"k%015d" (16 B), V-half values r||r (84 B,
numpy default_rng(20250307)), BlockSize 4096, MinFilterKeys 0, 10 bits per key.
Prints one JSON line: end-to-end KV/s for host-resident KVs (flush: host arrays in, encoded SST
bytes out, including the staging and PCIe copies) and for HBM-resident KVs (compaction's
re-encode), with the add / build / encode split; run under `rocprofv3 --kernel-trace --stats`
for the GPU kernel time of the same command.  usage: python tools/bench_encode.py [--kv N] [--codec none|snappy]
[--steps K] [--check]"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "slatedb-go_amd")]


def kv_arrays(n: int, seed: int = 20250307):
    keys = np.zeros((n, 16), np.uint8)
    keys[:, 0] = ord("k")
    i = np.arange(n, dtype=np.int64)
    for pos in range(15, 0, -1):
        keys[:, pos] = 48 + (i % 10)
        i //= 10
    rng = np.random.default_rng(seed)
    r = rng.integers(0, 256, (n, 42), dtype=np.uint8)
    vals = np.concatenate([r, r], axis=1)
    key_off = (np.arange(n + 1, dtype=np.uint64) * 16)
    val_off = (np.arange(n + 1, dtype=np.uint64) * 84)
    return keys.reshape(-1), key_off, vals.reshape(-1), val_off


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--kv", type=int, default=10_000_000)
    p.add_argument("--codec", choices=["none", "snappy"], default="none")
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--check", action="store_true", help="compare the SST bytes with the oracle")
    args = p.parse_args()
    import torch
    import slatecodec as sc
    codec = sc.NONE if args.codec == "none" else sc.SNAPPY
    t0 = time.time()
    keys, key_off, vals, val_off = kv_arrays(args.kv)
    gen_s = time.time() - t0
    ctx = sc.Context(0)
    dev = torch.device("cuda", 0)
    d_keys, d_vals = torch.from_numpy(keys).to(dev), torch.from_numpy(vals).to(dev)
    d_ko = torch.from_numpy(key_off.view(np.int64)).to(dev)
    d_vo = torch.from_numpy(val_off.view(np.int64)).to(dev)
    torch.cuda.synchronize()
    res = {}
    encs = {}
    sink = np.empty(int(args.kv * 110), np.uint8)  # the caller's output buffer, reused across steps
    sink.fill(0)
    for mode in ("host", "device"):
        times = []
        for step in range(args.steps + 1):  # step 0 warms up
            t0 = time.perf_counter()
            b = sc.SstBuilder(ctx, 4096, 0, 10, codec)
            if mode == "host":
                assert b.add_batch(keys, key_off, vals, val_off) == 0
            else:
                assert b.add_batch_device(d_keys.data_ptr(), d_ko.data_ptr(), d_vals.data_ptr(), d_vo.data_ptr(),
                                          args.kv) == 0
            t1 = time.perf_counter()
            t = b.build()
            t2 = time.perf_counter()
            enc = t.encode_array(sink)
            t3 = time.perf_counter()
            if step:
                times.append((t3 - t0, t1 - t0, t2 - t1, t3 - t2))
            del t, b
        encs[mode] = enc.copy()
        med = lambda k: float(np.median([x[k] for x in times]))  # noqa: E731
        res[mode] = {"end_to_end_s": med(0), "end_to_end_kv_per_s": args.kv / med(0), "add_s": med(1),
                     "build_s": med(2), "encode_s": med(3)}
    out = {"metric": "SST encode (sstable.Builder) KV/s, 100 B KV", "workload": "configs[2]: 10 M x 100 B KV",
           "kv": args.kv, "codec": args.codec, "sst_bytes": int(encs["host"].size), "steps": args.steps,
           "host_input": res["host"], "device_input": res["device"],
           "host_input_path": "slate_sst_builder_add_batch (host arrays) + build + table encode into a host array",
           "device_input_path": "slate_sst_builder_add_batch_device (KVs resident in HBM) + build + table encode",
           "gen_s": gen_s, "data": "synthetic (SURVEY 8d keys k%015d, V-half values)",
           "same_bytes_host_device": bool(np.array_equal(encs["host"], encs["device"]))}
    if args.check:
        from oracle import binding as ob
        t0 = time.time()
        o = ob.SstBuilder(4096, 0, 10, ob.NONE if codec == sc.NONE else ob.SNAPPY)
        assert o.add_batch(keys, key_off, vals, val_off) == 0
        assert o.build() == 0
        ref = o.encode_table()
        out["oracle_s"] = time.time() - t0
        out["bit_exact"] = ref == encs["host"].tobytes()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
