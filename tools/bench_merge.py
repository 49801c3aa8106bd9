"""Compaction-merge measurement (tooling): iter.MergeSort
(internal/iter/merge.go:12-111) over k sorted runs of b"k%015d" keys, device-resident
(slate_merge_sorted_device, inputs already in HBM), timed with HIP events on the context's
stream, checked bit-exact against the oracle's heap restatement, which is also timed on one host
core as the CPU baseline.  Algorithmic bytes per merge: read keys (16 B) + key offsets (8 B) per
input entry, write one u32 index per returned entry.
usage: python tools/bench_merge.py [--k 4] [--n-per 2500000] [--overlap 0.3] [--steps 20]"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "slatedb-go_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--n-per", type=int, default=2_500_000)
    ap.add_argument("--overlap", type=float, default=0.3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()
    import torch
    import slatecodec as sc
    from oracle import binding as ob
    from tests import mergegen as mg

    keys, off, ss = mg.compaction_runs(args.k, args.n_per, args.overlap, seed=args.k)
    n = int(ss[-1])
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)  # torch's HIP runtime first, then the library's context (as bench.py)
    ctx = sc.Context(0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    d_keys = torch.from_numpy(keys).to(dev)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    d_out = torch.zeros(n, dtype=torch.int32, device=dev)
    d_n = torch.zeros(1, dtype=torch.int64, device=dev)
    d_flags = torch.zeros(1, dtype=torch.int32, device=dev)
    scratch = torch.empty(sc.lib().slate_merge_scratch_bytes(n, args.k), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    def run():
        ctx.merge_device(d_keys.data_ptr(), d_off.data_ptr(), ss, d_out.data_ptr(), d_n.data_ptr(),
                         d_flags.data_ptr(), scratch.data_ptr())

    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    for a, b in evs:
        a.record(stream)
        run()  # the device entry synchronises its own stream after launch (host source starts)
        b.record(stream)
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in evs)
    med = ms[len(ms) // 2]
    m = int(d_n.item())
    got = d_out[:m].cpu().numpy().view(np.uint32)
    t0 = time.perf_counter()
    want = ob.merge_arrays(keys, off, ss)
    cpu_s = time.perf_counter() - t0
    exact = bool(np.array_equal(got, want)) and int(d_flags.item()) == 0
    alg = 24 * n + 4 * m
    print(json.dumps({
        "metric": "compaction merge (iter.MergeSort) entries/s, device-resident", "value": round(n / (med / 1e3)),
        "unit": "entries/s", "ms_per_merge": round(med, 4), "ms_min": round(ms[0], 4),
        "config": {"k": args.k, "entries": n, "returned": m, "overlap": args.overlap, "key": "k%015d (16 B)"},
        "bit_exact_vs_oracle": exact,
        "alg_bytes": alg, "alg_GBps": round(alg / (med / 1e3) / 1e9, 1), "hbm_peak_GBps": 8000.0,
        "cpu_baseline": {"value": round(n / cpu_s), "unit": "entries/s", "cores": 1, "kind": "port",
                         "sample": f"oracle/slate_oracle.c or_merge_sort (heap, merge.go restated) on all {n} entries"},
    }))
    if not exact:
        sys.exit(1)


if __name__ == "__main__":
    main()
