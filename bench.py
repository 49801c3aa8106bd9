#!/usr/bin/env python
"""Headline benchmark: device-resident SST block decode GiB/s (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 1 M encoded 4 KiB Snappy blocks
per GPU, keys b"k%015d", 84-byte V-half values (r||r), BlockSize 4096 (38 rows of
100-byte KVs per block), already resident in HBM.  One step = one pass of the
decode path over the batch: plan (decoded sizes + scans) + decode (CRC32 verify,
Snappy decompress, offset checks, row descriptors).  value = decoded bytes of all
ranks per second (GiB = 2^30).  Multi-GPU: one process per GPU, every rank
decodes its own shard (blocks are independent; no collective on the data path),
so scaling is weak.

Run: python bench.py [--gpus N --steps K --warmup W]
     python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "slatedb-go_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "device-resident SST block decode GiB/s, 4 KiB blocks, at 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--blocks", type=int, default=1_000_000, help="blocks per GPU")
    p.add_argument("--codec", choices=["snappy", "none", "lz4", "zstd"], default="snappy",
                   help="zstd runs BASELINE configs[4] (1 KiB values, Zipf-prefixed keys, libzstd level 3 + checksum)")
    p.add_argument("--values", choices=["half", "rand"], default="half")
    p.add_argument("--cpu-seconds", type=float, default=8.0, help="budget per CPU-baseline leg")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cache", default="", help="directory to reuse the generated workload from (profiling runs: "
                   "the zstd generator's libzstd clashes with the profiler's own copy)")
    p.add_argument("--no-host-io", action="store_true")
    p.add_argument("--pmc-json", default=os.path.join(REPO, "profiles", "pmc_decode_latest.json"))
    return p.parse_args()


def main():
    args = parse()
    import torch

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    import slatecodec as sc
    from tools import workload as wl

    codec = {"snappy": sc.SNAPPY, "none": sc.NONE, "lz4": sc.LZ4, "zstd": sc.ZSTD}[args.codec]
    n = args.blocks
    t0 = time.time()
    spec = shard_spec(rank, n)
    cache = (os.path.join(args.cache, f"wl_{args.codec}_{args.values}_{n}_{spec['seed']}_{spec['kv_begin']}")
             if args.cache else "")
    if cache and os.path.exists(cache + "_blob.npy"):
        dec, dec_off, blob, in_off = (np.load(cache + f"_{k}.npy") for k in ("dec", "dec_off", "blob", "in_off"))
    else:
        if args.codec == "zstd":  # configs[4] "mixed"
            dec, dec_off = wl.mixed_blocks(n, seed=spec["seed"])
        else:
            dec, dec_off = wl.decoded_blocks(n, seed=spec["seed"], half=(args.values == "half"),
                                             kv_begin=spec["kv_begin"])
        blob, in_off = wl.encode_blocks(codec, dec, dec_off, threads=min(16, os.cpu_count() or 4))
        if cache:
            os.makedirs(args.cache, exist_ok=True)
            for k, v in (("dec", dec), ("dec_off", dec_off), ("blob", blob), ("in_off", in_off)):
                np.save(cache + f"_{k}.npy", v)
    gen_s = time.time() - t0
    dec_bytes = int(dec_off[-1])
    enc_bytes = int(in_off[-1])

    ctx = sc.Context(local)
    # An explicit (non-null) stream: the C-ABI launches on it and the HIP events
    # that time the decode kernel are recorded on it.
    stream = torch.cuda.Stream(device)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)

    d_in = torch.from_numpy(blob).to(device)
    d_in_off = torch.from_numpy(in_off.view(np.int64)).to(device)
    d_out_off = torch.empty(n + 1, dtype=torch.int64, device=device)
    d_row_base = torch.empty(n + 1, dtype=torch.int64, device=device)
    d_scratch = torch.empty(sc.decode_scratch_bytes(n) + 64, dtype=torch.uint8, device=device)
    ctx.decode_plan_device(codec, d_in.data_ptr(), d_in_off.data_ptr(), n, d_out_off.data_ptr(),
                           d_row_base.data_ptr(), d_scratch.data_ptr())
    torch.cuda.synchronize(device)
    total_out = int(d_out_off[n].item())
    total_rows = int(d_row_base[n].item())
    d_out = torch.empty(total_out + 16, dtype=torch.uint8, device=device)
    d_meta = torch.empty(n * 16, dtype=torch.uint8, device=device)
    d_rows = torch.empty(max(total_rows, 1) * 16, dtype=torch.uint8, device=device)

    def step(ev=None):
        ctx.decode_plan_device(codec, d_in.data_ptr(), d_in_off.data_ptr(), n, d_out_off.data_ptr(),
                               d_row_base.data_ptr(), d_scratch.data_ptr())
        if ev is not None:
            ev[0].record(stream)
        ctx.decode_device(codec, d_in.data_ptr(), d_in_off.data_ptr(), n, d_out.data_ptr(), d_out_off.data_ptr(),
                          d_meta.data_ptr(), d_rows.data_ptr(), d_row_base.data_ptr())
        if ev is not None:
            ev[1].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(device)

    # ---- verify (size-independent properties + sampled bytes against the generator)
    meta = np.frombuffer(d_meta.cpu().numpy().tobytes(), dtype=sc.META_DTYPE)
    assert (meta["status"] == 0).all(), np.unique(meta["status"], return_counts=True)
    out_off = d_out_off.cpu().numpy().view(np.uint64)
    sample = np.arange(0, n, max(1, n // 997))
    out_h = d_out.cpu().numpy()
    for i in sample:
        a = int(out_off[i])
        ln = int(dec_off[i + 1] - dec_off[i])
        assert out_h[a:a + ln].tobytes() == dec[int(dec_off[i]):int(dec_off[i + 1])].tobytes(), f"block {i}"
    n_rows = int(meta["n_rows"].astype(np.int64).sum())
    del out_h

    # ---- timed region
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize(device)
    t_start = time.perf_counter()
    for k in range(args.steps):
        step(evs[k])
    torch.cuda.synchronize(device)
    t_end = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = t_end - t_start
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    elapsed = max_over_ranks(dist, elapsed, device)

    ms_per_step = elapsed * 1e3 / args.steps
    value = world * dec_bytes * args.steps / elapsed / 2**30

    # roofline of the dominant kernel (decode_lpb_kernel for Snappy): algorithmic bytes per launch
    alg_read = enc_bytes + 8 * (n + 1) * 3  # encoded blocks incl. CRC + in_off/out_off/row_base
    alg_write = dec_bytes + 16 * n_rows + 16 * n  # decoded bytes + row descriptors + block meta
    alg = alg_read + alg_write
    achieved = alg / (kern_ms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.pmc_json):
        try:
            pm = json.load(open(args.pmc_json))
            if pm.get("blocks") == n and pm.get("codec") == args.codec:
                traffic = pm.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                "kernel": {"snappy": "decode_lpb2_kernel", "zstd": "decode_fast_kernel<2>"}.get(args.codec, "decode_fast_kernel<0>"),
                "kernel_ms": round(kern_ms, 4),
                "alg_bytes_per_launch": alg, "alg_read_bytes": alg_read, "alg_write_bytes": alg_write,
                "read_only_frac": round(alg_read / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)}

    result = {"metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
              "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
              "scaling": "weak", "vs_baseline": None, "dtype": "u8",
              "data": ("synthetic (SURVEY 8d configs[4]: Zipf-prefixed 8-256 B keys, 1 KiB V-half values, libzstd "
                       "level 3 + checksum frames)" if args.codec == "zstd" else
                       "synthetic (SURVEY 8d keys k%015d, V-half values, " + {"snappy": "libsnappy-encoded)",
                                                                              "lz4": "liblz4 frames)",
                                                                              "none": "CodecNone)"}[args.codec]),
              "config": {"workload": ("configs[1]: 1 M x 4 KiB Snappy blocks, 100 B KV, device-resident decode"
                                      if args.codec == "snappy" and n == 1_000_000 and args.values == "half"
                                      else f"configs[4] mixed: {n} x 4 KiB Zstd blocks, 1 KiB values, skewed key "
                                      "prefixes, device-resident decode (not the headline config)"
                                      if args.codec == "zstd"
                                      else f"{n} x 4 KiB {args.codec} blocks, 100 B KV ({args.values} values), "
                                      "device-resident decode (not the headline config)"),
                         "blocks_per_gpu": n, "codec": args.codec, "values": args.values, "block_size": 4096,
                         "decoded_bytes_per_gpu": dec_bytes, "encoded_bytes_per_gpu": enc_bytes,
                         "rows_per_gpu": n_rows, "parallelism": f"shard{world} (no collective)"},
              "roofline": roofline}

    if rank == 0 and world == 1 and not args.no_host_io:
        result["host_io"] = host_io_rate(torch, sc, ctx, codec, blob, in_off, dec_bytes, device)
        result["host_io_pinned"] = host_io_pinned(torch, sc, codec, blob, in_off, device)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(codec, blob, in_off, args.cpu_seconds)

    if rank == 0:
        result["gen_seconds"] = round(gen_s, 1)
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


def shard_spec(rank: int, blocks_per_rank: int) -> dict:
    """Rank r decodes its own blocks: a disjoint key range (38 keys per block, 40
    reserved) and its own value seed, so every rank's shard is distinct data."""
    return {"seed": 20250307 + rank, "kv_begin": rank * blocks_per_rank * 40}


def max_over_ranks(dist, elapsed: float, device) -> float:
    """Whole-job time = the slowest rank's time (one all-reduce, outside the timed region)."""
    if not dist:
        return elapsed
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def host_io_pinned(torch, sc, codec, blob, in_off, device, n_streams=4, chunk=32768, max_blocks=262144):
    """Host-in/host-out with pinned buffers: per chunk of blocks, H2D of the encoded
    blocks + offsets, plan + decode, D2H of decoded bytes + block meta + row
    descriptors; chunks round-robin over n_streams streams (one slate_ctx each) so
    copies overlap kernels.  For DESIGN.md (PCIe-bound), never `value`."""
    n = min(len(in_off) - 1, max_blocks)
    streams = [torch.cuda.Stream(device) for _ in range(n_streams)]
    ctxs = []
    for s in streams:
        c = sc.Context(device.index)
        c.set_stream(s.cuda_stream)
        ctxs.append(c)
    jobs = []
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        m = b - a
        lo, hi = int(in_off[a]), int(in_off[b])
        h_in = torch.from_numpy(blob[lo:hi].copy()).pin_memory()
        h_off = torch.from_numpy((in_off[a:b + 1] - in_off[a]).astype(np.int64)).pin_memory()
        d_in = torch.empty(hi - lo, dtype=torch.uint8, device=device)
        d_off = torch.empty(m + 1, dtype=torch.int64, device=device)
        d_oo = torch.empty(m + 1, dtype=torch.int64, device=device)
        d_rb = torch.empty(m + 1, dtype=torch.int64, device=device)
        d_sc = torch.empty(sc.decode_scratch_bytes(m) + 64, dtype=torch.uint8, device=device)
        d_in.copy_(h_in)
        d_off.copy_(h_off)
        ctxs[0].set_stream(torch.cuda.current_stream(device).cuda_stream)
        ctxs[0].decode_plan_device(codec, d_in.data_ptr(), d_off.data_ptr(), m, d_oo.data_ptr(), d_rb.data_ptr(),
                                   d_sc.data_ptr())
        torch.cuda.synchronize(device)
        ctxs[0].set_stream(streams[0].cuda_stream)
        tot, rows = int(d_oo[m].item()), int(d_rb[m].item())
        jobs.append(dict(m=m, h_in=h_in, h_off=h_off, d_in=d_in, d_off=d_off, d_oo=d_oo, d_rb=d_rb, d_sc=d_sc,
                         d_out=torch.empty(tot + 16, dtype=torch.uint8, device=device),
                         d_meta=torch.empty(m * 16, dtype=torch.uint8, device=device),
                         d_rows=torch.empty(max(rows, 1) * 16, dtype=torch.uint8, device=device),
                         h_out=torch.empty(tot + 16, dtype=torch.uint8).pin_memory(),
                         h_meta=torch.empty(m * 16, dtype=torch.uint8).pin_memory(),
                         h_rows=torch.empty(max(rows, 1) * 16, dtype=torch.uint8).pin_memory()))

    def run():
        for i, j in enumerate(jobs):
            s, c = streams[i % n_streams], ctxs[i % n_streams]
            with torch.cuda.stream(s):
                j["d_in"].copy_(j["h_in"], non_blocking=True)
                j["d_off"].copy_(j["h_off"], non_blocking=True)
                c.decode_plan_device(codec, j["d_in"].data_ptr(), j["d_off"].data_ptr(), j["m"], j["d_oo"].data_ptr(),
                                     j["d_rb"].data_ptr(), j["d_sc"].data_ptr())
                c.decode_device(codec, j["d_in"].data_ptr(), j["d_off"].data_ptr(), j["m"], j["d_out"].data_ptr(),
                                j["d_oo"].data_ptr(), j["d_meta"].data_ptr(), j["d_rows"].data_ptr(),
                                j["d_rb"].data_ptr())
                j["h_out"].copy_(j["d_out"], non_blocking=True)
                j["h_meta"].copy_(j["d_meta"], non_blocking=True)
                j["h_rows"].copy_(j["d_rows"], non_blocking=True)
        torch.cuda.synchronize(device)

    run()  # warm
    t = time.perf_counter()
    run()
    el = time.perf_counter() - t
    meta = np.concatenate([np.frombuffer(j["h_meta"].numpy().tobytes(), dtype=sc.META_DTYPE) for j in jobs])
    assert (meta["status"] == 0).all()
    dec = int(np.sum(meta["data_len"].astype(np.int64) + 2 * meta["n_rows"].astype(np.int64) + 2))
    h2d = int(in_off[n]) + 8 * (n + len(jobs))
    d2h = sum(j["h_out"].numel() + j["h_meta"].numel() + j["h_rows"].numel() for j in jobs)
    for c in ctxs:
        c.close()
    return {"GiBps_decoded": round(dec / el / 2**30, 2), "blocks": n, "streams": n_streams, "chunk_blocks": chunk,
            "h2d_GBps": round(h2d / el / 1e9, 2), "d2h_GBps": round(d2h / el / 1e9, 2),
            "path": "pinned H2D + plan + decode + D2H (data, meta, rows), overlapped over streams"}


def host_io_rate(torch, sc, ctx, codec, blob, in_off, dec_bytes, device):
    """Host-in/host-out: pinned H2D of the encoded blocks + plan + decode + D2H of
    the decoded blocks, through the C-ABI batch call (for DESIGN.md, never `value`)."""
    n = len(in_off) - 1
    m = min(n, 200_000)
    sub_blob = blob[: int(in_off[m])]
    sub_off = in_off[: m + 1]
    ctx2 = sc.Context(device.index)
    ctx2.decode_batch(codec, sub_blob, sub_off)  # warm (allocations)
    t = time.perf_counter()
    out = ctx2.decode_batch(codec, sub_blob, sub_off)
    el = time.perf_counter() - t
    ctx2.close()
    sub_dec = int(out[1][-1])
    return {"GiBps_decoded": round(sub_dec / el / 2**30, 2), "blocks": m,
            "path": "slate_block_decode_batch (pageable host buffers, one stream, plan sync)"}


CODEC_RESTATEMENT = {0: "no codec", 1: "golang/snappy", 2: "compress/zlib+flate", 3: "LZ4 frame",
                     4: "RFC 8878 zstd (oracle/zstd_oracle.c)"}


def cpu_baseline(codec, blob, in_off, seconds):
    """The oracle (C restatement of the Go path) timed on this host: bounded sample."""
    from oracle import binding as ob
    n = len(in_off) - 1
    chunk = 20_000
    res = {}
    for threads in (1, min(16, os.cpu_count() or 1)):
        done = 0
        dec = 0
        t = time.perf_counter()
        while time.perf_counter() - t < seconds / (1 if threads == 1 else 2) and done < n:
            a, b = done, min(n, done + chunk)
            sub_off = (in_off[a:b + 1] - in_off[a]).astype(np.uint64)
            out, o_off, meta, rows, rb = ob.block_decode_batch(codec, blob[int(in_off[a]):int(in_off[b])], sub_off,
                                                               nthreads=threads)
            assert (meta["status"] == 0).all()
            dec += int(np.sum(meta["data_len"].astype(np.int64) + 2 * meta["n_rows"].astype(np.int64) + 2))
            done = b
        el = time.perf_counter() - t
        res[threads] = (dec / el / 2**30, done)
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    mt = max(res)
    return {"value": round(res[mt][0], 3), "unit": "GiB/s", "cores": mt, "kind": "port",
            "sample": f"first {res[mt][1]} of the same blocks, oracle/slate_oracle.c block decode "
                      f"(CRC32 + {CODEC_RESTATEMENT.get(codec, 'codec')} restatement + offsets + row walk), "
                      f"{mt} threads",
            "single_thread": {"value": round(res[1][0], 3), "cores": 1, "blocks": res[1][1]},
            "cpu_model": cpu_model}


if __name__ == "__main__":
    main()
