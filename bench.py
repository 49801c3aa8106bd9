#!/usr/bin/env python
"""Headline benchmark: device-resident SST block decode GiB/s (BASELINE.json metric).

Workloads (every block is generated on its own by tools/benchgen.c bg_build_set:
keys b"k%015d", 84-byte V-half values r||r, BlockSize 4096 -> 38 rows of 100-byte KVs,
Snappy-encoded by libsnappy + the block CRC32 trailer):
  configs1 (default)  BASELINE configs[1]: 1 M blocks per GPU.  Under torchrun the set has
                      N x 1 M blocks and block i belongs to rank i mod N (round-robin, no
                      collective): weak scaling, N = 1 is exactly configs[1].
  configs3            BASELINE configs[3]: ONE fixed set of 64 GiB of encoded blocks
                      (32,505,856 blocks), block i on rank i mod N: strong scaling.  A rank
                      holds what fits its HBM (outputs + row slots need ~10 KB per block),
                      so N = 1 runs the largest single-GPU slice of the set.
  --codec zstd        BASELINE configs[4] (1 KiB values, Zipf-prefixed keys, libzstd frames).
Inputs are resident in HBM before timing.  One step = plan (decoded sizes + scans) + decode
(CRC32 verify, decompress, offset checks, row descriptors) over the rank's whole shard.
value = decoded bytes of all ranks per second (GiB = 2^30) over the slowest rank's time.

Run: python bench.py [--gpus N --steps K --warmup W] [--workload configs3]
     python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import hashlib
import json
import math
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
SEED = 20250307
CONFIG3_BLOCKS = 32_505_856  # 64 GiB of encoded Snappy V-half blocks (~2,114 B each)
BYTES_PER_BLOCK_HBM = 2114 + 4016 + 268 * 16 + 16 + 24  # input, output slot, row slots, meta, offsets


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", choices=["configs1", "configs3"], default="configs1")
    p.add_argument("--blocks", type=int, default=1_000_000, help="configs1: blocks per GPU")
    p.add_argument("--max-blocks-per-gpu", type=int, default=0, help="configs3: cap a rank's slice (0 = what fits)")
    p.add_argument("--codec", choices=["snappy", "none", "lz4", "zstd"], default="snappy",
                   help="zstd runs BASELINE configs[4] (1 KiB values, Zipf-prefixed keys, libzstd level 3 + checksum)")
    p.add_argument("--values", choices=["half", "rand"], default="half")
    p.add_argument("--verify", choices=["all", "sample", "none"], default="",
                   help="decoded bytes, meta and rows vs the generator (default: all for configs1, sample for configs3)")
    p.add_argument("--cpu-seconds", type=float, default=8.0, help="budget per CPU-baseline leg")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cache", default="", help="configs[4]: directory to reuse the generated workload from")
    p.add_argument("--no-host-io", action="store_true")
    p.add_argument("--no-extras", action="store_true",
                   help="skip the extra legs (codec_none, configs4_zstd, configs2_encode; N=1 only)")
    p.add_argument("--extra-steps", type=int, default=10, help="timed steps of each extra leg")
    p.add_argument("--allow-variant", action="store_true", help="profiling only: accept SLATE_LIB_VARIANT")
    p.add_argument("--pmc-json", default="", help="PMC traffic file (default: profiles/pmc_decode_latest.json, "
                   "CodecNone: profiles/pmc_decode_none_latest.json)")
    return p.parse_args()


def lib_sha256() -> str:
    import slatecodec as sc
    with open(sc.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def host_cpus() -> int:
    """CPUs this process may run on: the affinity mask, capped by a cgroup CPU quota."""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, math.ceil(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return n


def main():
    args = parse()
    if (os.environ.get("SLATE_LIB_VARIANT") or os.environ.get("SLATE_DEBUG_MODE")) and not args.allow_variant:
        sys.exit("bench.py: SLATE_LIB_VARIANT / SLATE_DEBUG_MODE set: profiling variants are not benchmarks")
    import torch

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # rehearsal of the N-rank path on a one-GPU box only (every rank on cuda:0, gloo); the driver's
    # multi-GPU runs leave both unset: one rank per GPU over RCCL
    if os.environ.get("SLATE_BENCH_ONE_DEVICE") == "1":
        local = 0
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(os.environ.get("SLATE_BENCH_BACKEND", "nccl"))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    import slatecodec as sc
    from tools import workload as wl

    codec = {"snappy": sc.SNAPPY, "none": sc.NONE, "lz4": sc.LZ4, "zstd": sc.ZSTD}[args.codec]
    half = args.values == "half"
    threads = max(1, min(16, host_cpus()))
    t0 = time.time()
    shard = None  # (i_begin, stride, count) of the rank's blocks in the generated set
    if args.codec == "zstd":  # configs[4] "mixed": its own sequential generator, one shard per rank
        n = args.blocks
        cache = os.path.join(args.cache, f"wl_zstd_{n}_{SEED + rank}") if args.cache else ""
        dec_ref = None
        if cache and os.path.exists(cache + "_blob.npy"):
            blob, in_off = (np.load(cache + f"_{k}.npy") for k in ("blob", "in_off"))
        else:
            dec, dec_off = wl.mixed_blocks(n, seed=SEED + rank)
            blob, in_off = wl.encode_blocks(codec, dec, dec_off, threads=threads)
            dec_ref = (dec, dec_off)
            if cache:
                os.makedirs(args.cache, exist_ok=True)
                np.save(cache + "_blob.npy", blob)
                np.save(cache + "_in_off.npy", in_off)
        set_blocks, scaling = n * world, "weak"
    else:
        if args.workload == "configs1":
            set_blocks, count, scaling = world * args.blocks, args.blocks, "weak"
        else:
            set_blocks, scaling = CONFIG3_BLOCKS, "strong"
            count = sc.shard_blocks(set_blocks, world, rank)
            free = torch.cuda.mem_get_info(device)[0]
            fit = int(free * 0.92) // BYTES_PER_BLOCK_HBM
            count = min(count, fit, args.max_blocks_per_gpu or count)
        shard = (rank, world, count)
        blob, in_off = wl.block_set(codec, rank, world, count, seed=SEED, half=half, threads=threads)
        n = count
    gen_s = time.time() - t0
    enc_bytes = int(in_off[-1])

    ctx = sc.Context(local)
    # An explicit (non-null) stream: the C-ABI launches on it and the HIP events
    # that time the decode kernel are recorded on it.
    stream = torch.cuda.Stream(device)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)

    # Every device buffer is library-owned HBM (slate_devbuf, include/slatecodec.h): the path timed
    # here is the one a cgo caller reaches (slate_devbuf_ptr -> the *_device entry points).
    leg = DecodeLeg(sc, ctx, codec, blob, in_off)
    n = leg.n

    for _ in range(args.warmup):
        leg.step()
    torch.cuda.synchronize(device)

    # ---- verify, outside the timed region: every block's status; decoded bytes, meta and row
    # descriptors against the generator for every block (configs1) or evenly spread chunks (configs3)
    meta = leg.d_meta.download().view(sc.META_DTYPE)
    assert (meta["status"] == 0).all(), np.unique(meta["status"], return_counts=True)
    dec_bytes = int(np.sum(meta["data_len"].astype(np.int64) + 2 * meta["n_rows"].astype(np.int64) + 2))
    n_rows = int(meta["n_rows"].astype(np.int64).sum())
    verify = args.verify or ("all" if args.workload == "configs1" else "sample")
    verified = 0
    if shard is not None and verify != "none":
        verified = leg.verify_against_generator(wl, shard, verify, meta, threads, half)
    elif args.codec == "zstd" and verify != "none":
        verified = leg.verify_against_decoded(dec_ref, meta)
    # ---- timed region
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize(device)
    t_start = time.perf_counter()
    for k in range(args.steps):
        leg.step(evs[k], stream)
    torch.cuda.synchronize(device)
    t_end = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = t_end - t_start
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    elapsed = max_over_ranks(dist, elapsed, device)
    job_dec_bytes = sum_over_ranks(dist, dec_bytes, device)

    ms_per_step = elapsed * 1e3 / args.steps
    value = job_dec_bytes * args.steps / elapsed / 2**30

    # roofline of the dominant kernel: algorithmic bytes per launch / its event time
    roofline = decode_roofline(enc_bytes, n, dec_bytes, n_rows, kern_ms)
    pmc_json = args.pmc_json or os.path.join(REPO, "profiles", "pmc_decode_none_latest.json" if args.codec == "none"
                                             else "pmc_decode_latest.json")
    traffic, traffic_src = pmc_traffic(pmc_json, n, args.codec)
    roofline["traffic"] = traffic
    roofline["traffic_source"] = traffic_src
    roofline["kernel"] = {"snappy": "decode_lpb2_kernel", "lz4": "decode_lpb2_kernel<true> (+ decode_list_kernel<0>)",
                          "zstd": "zstd decode: zs_fast_parse/crc/build/sum + decode_list_kernel<2> "
                                  "(HIP events around the whole decode)",
                          "none": "decode_none_kernel"}.get(args.codec, "decode_fast_kernel<0>")

    if args.codec == "zstd":
        workload = (f"configs[4] mixed: {n} x 4 KiB Zstd blocks per GPU, 1 KiB values, skewed key prefixes, "
                    "device-resident decode")
        data = ("synthetic (SURVEY 8d configs[4]: Zipf-prefixed 8-256 B keys, 1 KiB V-half values, libzstd "
                "level 3 + checksum frames)")
    else:
        tag = f"{args.codec}, {args.values} values"
        if args.workload == "configs1":
            workload = (f"configs[1]: 1 M x 4 KiB Snappy blocks, 100 B KV, device-resident decode" if
                        (n == 1_000_000 and args.codec == "snappy" and half) else
                        f"{n} x 4 KiB blocks per GPU ({tag}), device-resident decode (not the headline config)")
            if world > 1:
                workload += f"; round-robin shards of one {set_blocks}-block set (block i on GPU i mod {world})"
        else:
            workload = (f"configs[3]: one set of {set_blocks} x 4 KiB Snappy blocks (64 GiB encoded), block i on GPU "
                        f"i mod {world}; this rank decodes {n} of its {sc.shard_blocks(set_blocks, world, rank)}")
        data = ("synthetic (SURVEY 8d keys k%015d, " + ("V-half" if half else "V-rand") + " values, " +
                {"snappy": "libsnappy-encoded", "none": "CodecNone",
                 "lz4": "liblz4 frames as pierrec/lz4's writer defaults"}.get(args.codec, args.codec) +
                ", every block generated on its own: tools/benchgen.c bg_build_set)")
    result = {"metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
              "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
              "scaling": scaling, "vs_baseline": None, "dtype": "u8", "data": data,
              "config": {"workload": workload, "blocks_per_gpu": n, "set_blocks": set_blocks, "codec": args.codec,
                         "values": args.values, "block_size": 4096, "decoded_bytes_per_gpu": dec_bytes,
                         "encoded_bytes_per_gpu": enc_bytes, "rows_per_gpu": n_rows,
                         "parallelism": f"shard{world} round-robin (no collective)"},
              "roofline": roofline,
              "verified": {"blocks": verified, "mode": verify if shard is not None else "status only",
                           "what": "every block's status; decoded bytes, meta and row descriptors vs the generator"}}

    if rank == 0 and world == 1:
        # the kernel's rate against a device-to-device copy measured on this box too
        copy = measured_copy_gbps(device)
        roofline["measured_copy_GBps"] = copy["value"]
        roofline["measured_copy"] = copy
        roofline["frac_of_measured_copy"] = round(roofline["achieved"] / copy["value"], 4)

    if rank == 0 and world == 1 and not args.no_host_io and shard is not None:
        result["host_io"] = host_io_rate(sc, ctx, codec, blob, in_off)

    if rank == 0 and world == 1 and not args.no_extras and args.codec == "snappy" and args.workload == "configs1":
        del leg  # the extra legs get the HBM back
        result["codec_none"] = codec_none_leg(sc, ctx, stream, wl, args, threads)
        result["configs4_zstd"] = zstd_leg(sc, ctx, stream, wl, args, threads)
        # configs[1]'s block shape (100-byte KVs, 4 KiB blocks) written by the Zstd and Zlib writers
        # the reference's other codecs stand for (compression.go:110-121, 88-97)
        result["kv100_zstd"] = kv100_leg(sc, ctx, stream, wl, args, threads, sc.ZSTD)
        result["kv100_zlib"] = kv100_leg(sc, ctx, stream, wl, args, threads, sc.ZLIB)
        result["configs2_encode"] = encode_leg(sc, ctx, args)
        result["compaction"] = compaction_leg(sc, ctx, args)
        # the unchanged per-block reader path (one GPU round trip per 4 KiB block) and BASELINE
        # configs[0] (one 64-block CodecNone SST encoded + decoded), next to the oracle on one thread
        from oracle import binding as ob
        from tools import percall_bench as pb
        result["per_call"] = pb.per_call(ctx, sc, ob, wl, 300)
        result["configs0"] = pb.configs0(ctx, sc, ob)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(codec, blob, in_off, args.cpu_seconds)

    if rank == 0:
        result["gen_seconds"] = round(gen_s, 1)
        result["lib_sha256"] = lib_sha256()[:16]
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


class DecodeLeg:
    """One device-resident decode workload on library-owned HBM (slate_devbuf): inputs uploaded
    once, a step = plan + decode (slate_block_decode_plan_device + slate_block_decode_device)."""

    def __init__(self, sc, ctx, codec, blob, in_off, time_plan=False):
        # time_plan: the kernel-time events bracket the plan too (CodecZlib: the plan is phase Z,
        # the inflate itself, staged for the decode call)
        self.sc, self.ctx, self.codec, self.time_plan = sc, ctx, codec, time_plan
        self.alias = False  # CodecNone: decode without a copy (d_out = NULL: block.go:122's aliasing)
        self.n = n = len(in_off) - 1
        self.d_in = sc.devbuf_from(ctx, blob)
        self.d_in_off = sc.devbuf_from(ctx, np.ascontiguousarray(in_off, np.uint64))
        self.d_out_off, self.d_row_base = sc.DevBuf(ctx, 8 * (n + 1)), sc.DevBuf(ctx, 8 * (n + 1))
        self.d_scratch = sc.DevBuf(ctx, sc.decode_scratch_bytes(n) + 64)
        ctx.decode_plan_device(codec, self.d_in.ptr, self.d_in_off.ptr, n, self.d_out_off.ptr, self.d_row_base.ptr,
                               self.d_scratch.ptr)
        self.total_out, self.total_rows = self.d_out_off.u64(n), self.d_row_base.u64(n)
        self.d_out = sc.DevBuf(ctx, self.total_out + 16)
        self.d_meta = sc.DevBuf(ctx, 16 * n)
        self.d_rows = sc.DevBuf(ctx, 16 * max(self.total_rows, 1))

    def step(self, ev=None, stream=None):
        c = self.ctx
        if ev is not None and self.time_plan:
            ev[0].record(stream)
        c.decode_plan_device(self.codec, self.d_in.ptr, self.d_in_off.ptr, self.n, self.d_out_off.ptr,
                             self.d_row_base.ptr, self.d_scratch.ptr)
        if ev is not None and not self.time_plan:
            ev[0].record(stream)
        c.decode_device(self.codec, self.d_in.ptr, self.d_in_off.ptr, self.n, 0 if self.alias else self.d_out.ptr,
                        0 if self.alias else self.d_out_off.ptr, self.d_meta.ptr, self.d_rows.ptr, self.d_row_base.ptr)
        if ev is not None:
            ev[1].record(stream)

    def timed(self, torch, stream, steps, warmup):
        """Mean decode-kernel ms (HIP events on the context's stream) and wall ms per step."""
        for _ in range(warmup):
            self.step()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k in range(steps):
            self.step(evs[k], stream)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t) * 1e3 / steps
        return float(np.mean([a.elapsed_time(b) for a, b in evs])), wall

    def verify_against_generator(self, wl, shard, verify, meta, threads, half):
        """Decoded bytes, meta and rows of every block (or 16 evenly spread chunks) against the
        per-block generator (tools/benchgen.c): returns the blocks verified."""
        n = self.n
        out_off_h = self.d_out_off.download(dtype=np.uint64)
        rb_h = self.d_row_base.download(dtype=np.uint64)
        meta_u8 = meta.view(np.uint8)
        chunk = 131072
        starts = list(range(0, n, chunk))
        if verify == "sample" and len(starts) > 16:
            starts = [starts[int(j * (len(starts) - 1) / 15)] for j in range(16)]
        verified = 0
        for k0 in starts:
            k1 = min(n, k0 + chunk)
            oa, ob_ = int(out_off_h[k0]), int(out_off_h[k1])
            ra, rb_ = int(rb_h[k0]), int(rb_h[k1])
            out_c = self.d_out.download(ob_ - oa, oa)
            rows_c = self.d_rows.download(16 * (rb_ - ra), 16 * ra)
            bad = wl.verify_set(shard[0] + k0 * shard[1], shard[1], k1 - k0, out_c, out_off_h[k0:k1 + 1] - oa,
                                rows_c, rb_h[k0:k1 + 1] - ra, meta_u8[16 * k0:16 * k1], seed=SEED, half=half,
                                threads=threads)
            assert bad == 0, f"{bad} blocks of [{k0}, {k1}) differ from the generator"
            verified += k1 - k0
        return verified

    def verify_against_decoded(self, dec_ref, meta):
        """configs[4]: every block's decoded bytes against the blocks before encoding."""
        if dec_ref is None:
            return 0
        from tools import workload as wl
        dec, dec_off = dec_ref
        dl = (meta["data_len"].astype(np.int64) + 2 * meta["n_rows"].astype(np.int64) + 2)
        assert np.array_equal(dl, np.diff(dec_off.astype(np.int64))), "decoded lengths differ"
        bad = wl.compare_blocks(self.d_out.download(), self.d_out_off.download(dtype=np.uint64), dec, dec_off)
        assert bad == 0, f"{bad} blocks differ from the blocks before encoding"
        return self.n

    def free(self):
        for b in (self.d_in, self.d_in_off, self.d_out_off, self.d_row_base, self.d_scratch, self.d_out, self.d_meta,
                  self.d_rows):
            b.free()


def decode_roofline(enc_bytes, n, dec_bytes, n_rows, kern_ms):
    """SURVEY 8d algorithmic bytes of one decode launch: R = encoded blocks incl. CRC + in_off /
    out_off / row_base reads, W = decoded bytes + 16 B per row descriptor + 16 B per block meta."""
    alg_read = enc_bytes + 8 * (n + 1) * 3
    alg_write = dec_bytes + 16 * n_rows + 16 * n
    alg = alg_read + alg_write
    achieved = alg / (kern_ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": None, "kernel_ms": round(kern_ms, 4),
            "alg_bytes_per_launch": alg, "alg_read_bytes": alg_read, "alg_write_bytes": alg_write,
            "read_only_frac": round(alg_read / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)}


def _decode_leg_result(sc, leg, torch, stream, steps, warmup, enc_bytes):
    kern_ms, wall_ms = leg.timed(torch, stream, steps, warmup)
    meta = leg.d_meta.download().view(sc.META_DTYPE)
    assert (meta["status"] == 0).all(), np.unique(meta["status"], return_counts=True)
    dec_bytes = int(np.sum(meta["data_len"].astype(np.int64) + 2 * meta["n_rows"].astype(np.int64) + 2))
    n_rows = int(meta["n_rows"].astype(np.int64).sum())
    return meta, {"value": round(dec_bytes / (wall_ms * 1e-3) / 2**30, 2), "unit": "GiB/s",
                  "ms_per_step": round(wall_ms, 4), "steps": steps,
                  "roofline": decode_roofline(enc_bytes, leg.n, dec_bytes, n_rows, kern_ms),
                  "blocks": leg.n, "decoded_bytes": dec_bytes, "encoded_bytes": enc_bytes, "rows": n_rows}


def codec_none_leg(sc, ctx, stream, wl, args, threads):
    """CodecNone decode (the DB's default codec, slatedb/config/config.go:85) of the configs[1] keys
    and values: 1 M blocks, every block verified against the generator outside the timed region."""
    import torch
    n = args.blocks
    blob, in_off = wl.block_set(sc.NONE, 0, 1, n, seed=SEED, half=True, threads=threads)
    leg = DecodeLeg(sc, ctx, sc.NONE, blob, in_off)
    meta, res = _decode_leg_result(sc, leg, torch, stream, args.extra_steps, 2, int(in_off[-1]))
    res["roofline"]["kernel"] = "decode_none_kernel (+ decode_large_kernel<0> over an empty list)"
    res["roofline"]["traffic"], res["roofline"]["traffic_source"] = pmc_traffic(
        os.path.join(REPO, "profiles", "pmc_decode_none_latest.json"), n, "none")
    res["verified"] = leg.verify_against_generator(wl, (0, 1, n), "all", meta, threads, True)
    # the same blocks decoded as Go decodes CodecNone, without a copy (block.go:122: Data aliases the
    # input; d_out = NULL): metas and rows only, checked equal to the copying decode's
    leg.alias = True
    rows_copy = leg.d_rows.download()
    leg.d_meta.memset(0)
    kern_a, wall_a = leg.timed(torch, stream, args.extra_steps, 2)
    meta_a = leg.d_meta.download().view(sc.META_DTYPE)
    same = meta_a.tobytes() == meta.tobytes() and np.array_equal(leg.d_rows.download(), rows_copy)
    assert same, "CodecNone aliased decode: metas / rows differ from the copying decode"
    alg_a = int(in_off[-1]) + 16 * int(meta["n_rows"].astype(np.int64).sum()) + 16 * n
    res["aliased"] = {"ms_per_step": round(wall_a, 4), "kernel_ms": round(kern_a, 4),
                      "GiBps_decoded": round(res["decoded_bytes"] / (wall_a * 1e-3) / 2**30, 1),
                      "alg_bytes_per_launch": alg_a, "GBps_alg": round(alg_a / (kern_a * 1e-3) / 1e9, 1),
                      "same_metas_and_rows": same,
                      "what": "slate_block_decode_device with d_out = NULL (block.Decode's aliasing for CodecNone, "
                              "block.go:122): CRC32, offsets and rows checked and described, no decoded copy written; "
                              "alg bytes = the blocks read + the row descriptors and metas written. The leg's value "
                              "and roofline above are the copying decode's"}
    leg.alias = False
    res["workload"] = f"{n} x 4 KiB CodecNone blocks (configs[1] keys and V-half values), device-resident decode"
    leg.free()
    return res


def zstd_leg(sc, ctx, stream, wl, args, threads):
    """BASELINE configs[4]: Zstd 4 KiB blocks (libzstd level 3 + checksum frames), 1 KiB values,
    Zipf-prefixed 8-256 B keys; every block's decoded bytes checked against the blocks before
    encoding, and the first 4096 blocks' metas and rows against the oracle."""
    import torch
    from oracle import binding as ob
    n = args.blocks
    t0 = time.time()
    dec, dec_off = wl.mixed_blocks(n, seed=SEED)
    blob, in_off = wl.encode_blocks(sc.ZSTD, dec, dec_off, threads=threads)
    gen_s = time.time() - t0
    leg = DecodeLeg(sc, ctx, sc.ZSTD, blob, in_off)
    meta, res = _decode_leg_result(sc, leg, torch, stream, args.extra_steps, 2, int(in_off[-1]))
    res["roofline"]["kernel"] = "zs_fast_parse/crc/build/sum + decode_list_kernel<2> (+ plan)"
    res["verified"] = leg.verify_against_decoded((dec, dec_off), meta)
    m = min(4096, n)
    sub_off = np.ascontiguousarray(in_off[:m + 1], np.uint64)
    o_out, o_off, o_meta, o_rows, o_rb = ob.block_decode_batch(ob.ZSTD, blob[:int(sub_off[m])], sub_off, nthreads=threads)
    assert o_meta.tobytes() == meta[:m].tobytes(), "configs4 metas differ from the oracle"
    rows = leg.d_rows.download(16 * int(o_rb[m])).view(sc.ROW_DTYPE)
    used = np.concatenate([np.arange(int(o_rb[i]), int(o_rb[i]) + int(o_meta["n_rows"][i])) for i in range(m)])
    assert rows[used].tobytes() == o_rows[used].tobytes(), "configs4 rows differ from the oracle"
    res["oracle_checked_blocks"] = m
    res["roofline"]["traffic"], res["roofline"]["traffic_source"] = pmc_traffic(
        os.path.join(REPO, "profiles", "pmc_decode_zstd_latest.json"), n, "zstd")
    if not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(sc.ZSTD, blob, in_off, args.cpu_seconds / 2)
    res["gen_seconds"] = round(gen_s, 1)
    res["workload"] = f"configs[4] mixed: {n} x 4 KiB Zstd blocks, 1 KiB values, skewed key prefixes"
    leg.free()
    return res


def kv100_leg(sc, ctx, stream, wl, args, threads, codec):
    """configs[1]'s blocks (1 M x 4 KiB, 100-byte V-half KVs) in CodecZstd (libzstd level 3 + checksum
    + content size: ~112 sequences and FSE_Compressed tables per block) or CodecZlib (zlib level 6
    closed as Go's compress/zlib closes a stream: tools/benchgen.c go_zlib6), device-resident decode.
    Every block's bytes are checked against the blocks before encoding, the first 4096 blocks'
    metas and rows against the oracle; `handbacks` = blocks a fast path left to the exact decoder in
    one step (slate_ctx_handbacks)."""
    import torch
    from oracle import binding as ob
    n = args.blocks
    t0 = time.time()
    dec, dec_off = wl.decoded_blocks(n, seed=SEED, half=True)
    blob, in_off = wl.encode_blocks(codec, dec, dec_off, threads=threads)
    gen_s = time.time() - t0
    leg = DecodeLeg(sc, ctx, codec, blob, in_off, time_plan=codec == sc.ZLIB)
    ctx.handbacks(reset=True)
    leg.step()
    handbacks = ctx.handbacks(reset=True)
    meta, res = _decode_leg_result(sc, leg, torch, stream, max(2, args.extra_steps // (1 if codec == sc.ZSTD else 5)), 1,
                                   int(in_off[-1]))
    name = {sc.ZSTD: "zstd", sc.ZLIB: "zlib"}[codec]
    res["roofline"]["kernel"] = ("zs_fast_parse + zs_fse_parse/crc/build/sum + decode_list_kernel<2> (+ plan)"
                                 if codec == sc.ZSTD else
                                 "zl_fast_kernel<stage> (the plan: phase Z once) + plan_zlib/scans + zs_fast_crc/build "
                                 "+ decode_list_kernel<1>, plan and decode timed together")
    res["handbacks"] = int(handbacks)
    res["verified"] = leg.verify_against_decoded((dec, dec_off), meta)
    m = min(4096, n)
    sub_off = np.ascontiguousarray(in_off[:m + 1], np.uint64)
    obc = {sc.ZSTD: ob.ZSTD, sc.ZLIB: ob.ZLIB}[codec]
    o_out, o_off, o_meta, o_rows, o_rb = ob.block_decode_batch(obc, blob[:int(sub_off[m])], sub_off, nthreads=threads)
    assert o_meta.tobytes() == meta[:m].tobytes(), f"kv100 {name} metas differ from the oracle"
    rows = leg.d_rows.download(16 * int(o_rb[m])).view(sc.ROW_DTYPE)
    used = np.concatenate([np.arange(int(o_rb[i]), int(o_rb[i]) + int(o_meta["n_rows"][i])) for i in range(m)])
    assert rows[used].tobytes() == o_rows[used].tobytes(), f"kv100 {name} rows differ from the oracle"
    res["oracle_checked_blocks"] = m
    res["gen_seconds"] = round(gen_s, 1)
    res["workload"] = (f"{n} x 4 KiB {name} blocks of configs[1]'s 100-byte V-half KVs, "
                       + ("libzstd level 3 + checksum + content size" if codec == sc.ZSTD else
                          "zlib level 6 + Go's empty final stored block"))
    leg.free()
    return res


def encode_leg(sc, ctx, args):
    """BASELINE configs[2]: 10 M x 100 B KV through the GPU sstable.Builder from HBM-resident KVs
    (slate_sst_builder_add_batch_device, compaction's re-encode path; flush's host-array path too),
    SST bytes compared with the oracle's C restatement of the Go builder at full size once.
    roofline: SURVEY 8d encode bytes (R = 100 B KV + 16 B descriptor per KV, W = encoded SST bytes +
    6 bloom-bit byte RMWs of 2 B per key) over the builder's device busy time (the union of HIP-event
    spans around every device pass, the library's measurement switch); `wall_frac` over the
    device-input build's wall time instead."""
    from oracle import binding as ob
    from tools import bench_encode as be
    n = 10_000_000
    keys, key_off, vals, val_off = be.kv_arrays(n)
    d_keys, d_vals = sc.devbuf_from(ctx, keys), sc.devbuf_from(ctx, vals)
    d_ko, d_vo = sc.devbuf_from(ctx, key_off), sc.devbuf_from(ctx, val_off)
    sink = np.empty(int(n * 110), np.uint8)
    sink.fill(0)
    pcie = pinned_copy_gbps()
    res = {"pcie": pcie}
    for codec, name in ((sc.NONE, "none"), (sc.SNAPPY, "snappy")):
        times, gpu, enc = [], [], None
        for k in range(4):  # the first warms the context
            ctx.set_timing(k > 0)
            ctx.gpu_busy_ms(reset=True)
            t0 = time.perf_counter()
            b = sc.SstBuilder(ctx, 4096, 0, 10, codec)
            assert b.add_batch_device(d_keys.ptr, d_ko.ptr, d_vals.ptr, d_vo.ptr, n) == 0
            t = b.build()
            t1 = time.perf_counter()
            enc = t.encode_array(sink)
            if k:
                times.append(t1 - t0)
                gpu.append(ctx.gpu_busy_ms(reset=True))
            del t, b
        ctx.set_timing(False)
        th = []
        hsink = np.empty_like(sink)  # the PUT buffer: caller-owned, reused like the device path's
        hsink.fill(0)
        for k in range(3):  # flush's path: host arrays in (staging + PCIe included)
            t0 = time.perf_counter()
            b = sc.SstBuilder(ctx, 4096, 0, 10, codec)
            assert b.add_batch(keys, key_off, vals, val_off) == 0
            t = b.build()
            host = t.encode_array(hsink)
            th.append(time.perf_counter() - t0)
            del t, b
        t0 = time.perf_counter()
        o = ob.SstBuilder(4096, 0, 10, ob.NONE if codec == sc.NONE else ob.SNAPPY)
        assert o.add_batch(keys, key_off, vals, val_off) == 0
        assert o.build() == 0
        ref = o.encode_table()
        oracle_s = time.perf_counter() - t0
        oracle_mt = oracle_threads_encode(ob, keys, key_off, vals, val_off,
                                          ob.NONE if codec == sc.NONE else ob.SNAPPY, host_cpus())
        exact = ref == enc.tobytes() and ref == host.tobytes()
        assert exact, f"configs[2] {name}: SST bytes differ from the oracle"
        s_dev = float(np.median(times))
        k_ms = float(np.median([g[0] for g in gpu]))
        k_sum = float(np.median([g[1] for g in gpu]))
        alg = n * (100 + 16) + len(ref) + n * 6 * 2
        # the link's bound for the host-input build: the KVs in, the SST out, at the pinned copy rates
        # measured here (one direction at a time, as the build moves them)
        kv_in = int(keys.nbytes + vals.nbytes + key_off.nbytes + val_off.nbytes)
        pcie_s = kv_in / (pcie["h2d_GBps"] * 1e9) + len(ref) / (pcie["d2h_GBps"] * 1e9)
        res[name] = {"value": round(n / s_dev, 1), "unit": "KV/s", "s_device_input": round(s_dev, 4),
                     "s_host_input": round(float(np.median(th)), 4),
                     "pcie_bound_s": round(pcie_s, 4), "host_input_over_pcie_bound": round(float(np.median(th)) / pcie_s, 2),
                     "pcie_bound_note": f"{kv_in} B of KVs + offsets in, {len(ref)} B of SST out, at pinned "
                                        f"hipMemcpy rates measured in this run ({pcie['h2d_GBps']} / "
                                        f"{pcie['d2h_GBps']} GB/s)",
                     "sst_bytes": len(ref), "bit_exact": exact,
                     "kernel_ms": round(k_ms, 3), "kernel_ms_summed": round(k_sum, 3),
                     "roofline": {"bound": "hbm", "achieved": round(alg / (k_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBPS,
                                  "unit": "GB/s", "frac": round(alg / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 5),
                                  "alg_bytes": alg,
                                  "time": "device busy time per build: the union of HIP-event spans around every "
                                          "device pass of add_batch_device and build, on the context's stream and the "
                                          "filter's side stream (slate_ctx_gpu_busy; overlap counted once; "
                                          "kernel_ms_summed adds the spans up). Excluded: the blocks' and payloads' "
                                          "device-to-host copies and small result reads",
                                  "wall_frac": round(alg / s_dev / 1e9 / HBM_PEAK_GBPS, 5)},
                     "cpu_baseline": {"value": round(n / oracle_s, 1), "unit": "KV/s", "cores": 1, "kind": "port",
                                      "sample": "the same 10 M KV through oracle/slate_oracle.c's sstable.Builder",
                                      "n_threads": oracle_mt}}
    for x in (d_keys, d_vals, d_ko, d_vo):
        x.free()
    res["workload"] = "configs[2]: 10 M x 100 B KV (keys k%015d, V-half values) -> SST blocks + bloom, BlockSize 4096"
    return res


def compaction_leg(sc, ctx, args, kv_per_sst=2_500_000, k=4, max_sst=256 << 20):
    """executeCompaction (slatedb/compaction/executor.go:92-151) end to end: k L0 SSTs of kv_per_sst
    KV each (keys k%015d over a shared key space with 30 % overlap, 84 B V-half values), host SST
    bytes in (the object-store GET buffers) -> slate_compact (decode -> row views -> MergeSort ->
    gather -> SST builders cut at MaxSSTSize) -> host SST bytes out, per codec (CodecNone = the DB's
    default, CodecSnappy).  Outputs bit-exact against the oracle's C restatement of the same loop
    (oracle/compact_oracle.c), which is also the CPU baseline, on one thread and on every CPU."""
    from oracle import binding as ob
    from tools import bench_compact as bc
    res = {"workload": f"{k} L0 SSTs x {kv_per_sst} KV (100 B: k%015d keys, 84 B V-half values, 30 % key overlap), "
                       f"MaxSSTSize {max_sst >> 20} MiB, output codec = input codec",
           "unit": "input KV/s"}
    threads = host_cpus()
    for codec, name in ((sc.NONE, "none"), (sc.SNAPPY, "snappy")):
        srcs = bc.make_sources(sc, ctx, k, kv_per_sst, 0.3, codec)
        # the GET buffers as a cgo caller holds them: one host array, SST offsets, source ranges
        ssts = [x for run in srcs for x in run]
        blob = np.frombuffer(b"".join(ssts), np.uint8)
        sst_off = np.zeros(len(ssts) + 1, np.uint64)
        sst_off[1:] = np.cumsum([len(x) for x in ssts])
        src_sst = np.arange(len(srcs) + 1, dtype=np.uint32)
        in_bytes = int(blob.size)
        sink = np.empty(in_bytes + (1 << 20), np.uint8)  # the PUT buffers, reused
        sink.fill(0)
        sc.compact_arrays(ctx, blob, sst_off, src_sst, max_sst, codec=codec, sink=sink)  # warm-up
        walls, busy, out = [], [], None
        for _ in range(3):
            ctx.synchronize()
            ctx.set_timing(True)
            ctx.gpu_busy_ms(reset=True)
            t0 = time.perf_counter()
            out = sc.compact_arrays(ctx, blob, sst_off, src_sst, max_sst, codec=codec, sink=sink)
            walls.append(time.perf_counter() - t0)
            busy.append(ctx.gpu_busy_ms(reset=True))
            ctx.set_timing(False)
        # the oracle: the same inputs, the same loop, one thread and every CPU
        oc = ob.NONE if codec == sc.NONE else ob.SNAPPY
        t0 = time.perf_counter()
        st, ref, ref_off = ob.compact_arrays(blob, sst_off, src_sst, max_sst, oc, 1)
        cpu1 = time.perf_counter() - t0
        assert st == 0, ob.status_string(st)
        t0 = time.perf_counter()
        st, ref_mt, _ = ob.compact_arrays(blob, sst_off, src_sst, max_sst, oc, threads)
        cpu_mt = time.perf_counter() - t0
        assert st == 0, ob.status_string(st)
        got = b"".join(o.tobytes() for o in out)
        exact = (len(out) == len(ref_off) - 1 and got == ref.tobytes() and ref.tobytes() == ref_mt.tobytes() and
                 all(len(o) == int(ref_off[i + 1] - ref_off[i]) for i, o in enumerate(out)))
        assert exact, f"compaction {name}: output SSTs differ from the oracle"
        n_in = k * kv_per_sst
        wall = float(np.median(walls))
        res[name] = {"value": round(n_in / wall, 1), "s_wall": round(wall, 4),
                     "device_busy_ms": round(float(np.median([b[0] for b in busy])), 3),
                     "device_busy_ms_summed": round(float(np.median([b[1] for b in busy])), 3),
                     "input_sst_bytes": in_bytes, "output_ssts": len(out), "output_sst_bytes": len(got),
                     "bit_exact": exact,
                     "cpu_baseline": {"value": round(n_in / cpu1, 1), "unit": "input KV/s", "cores": 1, "kind": "port",
                                      "s": round(cpu1, 3), "value_all_threads": round(n_in / cpu_mt, 1),
                                      "threads": threads, "s_all_threads": round(cpu_mt, 3),
                                      "sample": "the same inputs through oracle/compact_oracle.c (or_compact: "
                                                "block.Decode + block.Iterator keys, iter.MergeSort, the MaxSSTSize "
                                                "writer loop); all-threads: blocks decoded and outputs built in "
                                                "parallel, the merge serial"}}
        del srcs, blob, ref, ref_mt, out
    res["time"] = ("s_wall: the slate_compact call from host SST bytes to host SST bytes (uploads, every device "
                   "stage, the output builders) plus slate_sst_table_encode of every output into a reused PUT "
                   "buffer; device_busy_ms: the union of HIP-event spans around its kernel groups "
                   "(slate_ctx_gpu_busy)")
    return res


def oracle_threads_encode(ob, keys, key_off, vals, val_off, codec, threads):
    """The oracle's sstable.Builder on every CPU this process may use: the 10 M KV cut into one
    contiguous slice per thread, each slice its own SST (the reference builds one SST per flush /
    compaction output serially: independent builders are how N cores serve N SSTs)."""
    from concurrent.futures import ThreadPoolExecutor
    n = len(key_off) - 1
    bounds = [n * t // threads for t in range(threads + 1)]

    def one(t):
        a, b = bounds[t], bounds[t + 1]
        ko = (key_off[a:b + 1] - key_off[a]).astype(np.uint64)
        vo = (val_off[a:b + 1] - val_off[a]).astype(np.uint64)
        o = ob.SstBuilder(4096, 0, 10, codec)
        assert o.add_batch(keys[int(key_off[a]):int(key_off[b])], ko, vals[int(val_off[a]):int(val_off[b])], vo) == 0
        assert o.build() == 0
        return len(o.encode_table())

    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(one, range(threads)))
    s = time.perf_counter() - t0
    return {"value": round(n / s, 1), "unit": "KV/s", "cores": threads,
            "sample": f"the same 10 M KV as {threads} SSTs of contiguous slices, one oracle builder per thread"}


def pinned_copy_gbps(nbytes: int = 256 << 20, reps: int = 5) -> dict:
    """Host<->device rates of page-locked hipMemcpy (torch pinned tensors), each direction alone."""
    import torch
    h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    res = {}
    for name, fn in (("h2d_GBps", lambda: d.copy_(h, non_blocking=True)), ("d2h_GBps", lambda: h.copy_(d, non_blocking=True))):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        res[name] = round(nbytes * reps / (time.perf_counter() - t) / 1e9, 1)
    del h, d
    return res


def measured_copy_gbps(device, nbytes: int = 2 << 30, reps: int = 10) -> dict:
    """Read + write bytes per second of a large device-to-device copy, outside the timed region:
    the best of the hand-written streaming copy shapes in tools/copy_kernel.hip (16 B per lane;
    grid-stride with 4 or 8 loads in flight, plain or nontemporal, at 4 / 8 / 16 workgroups per CU,
    and one-pass grids covering the buffer), and torch's copy_."""
    import ctypes
    import torch
    a = torch.empty(nbytes, dtype=torch.uint8, device=device)
    b = torch.empty_like(a)
    a.fill_(1)
    stream = torch.cuda.current_stream(device)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def timed(fn):
        fn()
        ev[0].record(stream)
        for _ in range(reps):
            fn()
        ev[1].record(stream)
        ev[1].synchronize()
        return 2 * nbytes / (ev[0].elapsed_time(ev[1]) / reps * 1e-3) / 1e9

    res = {"torch_copy_GBps": round(timed(lambda: b.copy_(a)), 1)}
    so = os.path.join(REPO, "tools", "build", "libcopykernel.so")
    if os.path.exists(so):
        lib = ctypes.CDLL(so)
        fn = getattr(lib, "slate_probe_stream_copy_v", None)
        cus = torch.cuda.get_device_properties(device).multi_processor_count
        shapes = {}
        if fn is None:  # an older build: the round-4 kernel only
            lib.slate_probe_stream_copy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                                    ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
            for g in (4, 8, 16):
                shapes[f"v0_g{g}"] = timed(lambda: lib.slate_probe_stream_copy(a.data_ptr(), b.data_ptr(), nbytes,
                                                                               stream.cuda_stream, cus, g))
        else:
            fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int,
                           ctypes.c_int, ctypes.c_int]
            for v in range(8):
                for g in ((4, 8, 16) if v < 5 else (8,)):
                    b.zero_()
                    shapes[f"v{v}_g{g}" if v < 5 else f"v{v}"] = timed(
                        lambda: fn(a.data_ptr(), b.data_ptr(), nbytes, stream.cuda_stream, cus, g, v))
                    assert torch.equal(a[:4096], b[:4096]) and torch.equal(a[-4096:], b[-4096:]), f"copy kernel v{v}"
        best = max(shapes, key=shapes.get)
        res["stream_copy_GBps"] = round(shapes[best], 1)
        res["stream_copy_shape"] = best
        res["stream_copy_shapes"] = {k: round(v, 1) for k, v in shapes.items()}
    del a, b
    res["value"] = res.get("stream_copy_GBps", res["torch_copy_GBps"])
    return res


def pmc_traffic(path: str, n: int, codec: str):
    """HBM bytes per launch from the PMC passes (tools/traffic.sh), only when they were taken on
    this very library build and workload."""
    if not os.path.exists(path):
        return None, "no PMC file"
    try:
        pm = json.load(open(path))
    except (OSError, ValueError):
        return None, "unreadable PMC file"
    if pm.get("blocks") != n or pm.get("codec") != codec:
        return None, "PMC file is for another workload"
    if pm.get("lib_sha256") != lib_sha256():
        return None, "PMC file is for another library build"
    return pm.get("hbm_bytes_per_launch"), os.path.relpath(path, REPO)


def shard_spec(rank: int, blocks_per_rank: int) -> dict:
    """configs[4] (sequential generator): rank r gets its own seed and key range."""
    return {"seed": SEED + rank, "kv_begin": rank * blocks_per_rank * 40}


def max_over_ranks(dist, elapsed: float, device) -> float:
    """Whole-job time = the slowest rank's time (one all-reduce, outside the timed region)."""
    if not dist:
        return elapsed
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(dist, v: int, device) -> int:
    if not dist:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def host_io_rate(sc, ctx, codec, blob, in_off, max_blocks=262144):
    """Host-in/host-out through the C-ABI itself (slate_block_decode_batch: page-locked staging,
    chunks over two stream lanes), into caller buffers sized once from a plan-only call, and the
    same batch sharded over two contexts (slate_block_decode_sharded).  PCIe-bound: for
    DESIGN.md, never `value`."""
    n = min(len(in_off) - 1, max_blocks)
    sub_off = np.ascontiguousarray(in_off[: n + 1], np.uint64)
    sub = np.ascontiguousarray(blob[: int(sub_off[n])])
    ctx2 = sc.Context(ctx.device)
    out_off = np.zeros(n + 1, np.uint64)
    row_base = np.zeros(n + 1, np.uint64)
    meta = np.zeros(n, sc.META_DTYPE)
    st = ctx2.decode_batch_into(codec, sub, sub_off, np.zeros(1, np.uint8), np.zeros(1, sc.ROW_DTYPE), meta, out_off,
                                row_base)
    assert st == sc.E_CAPACITY, st
    out = np.zeros(int(out_off[n]) + 16, np.uint8)
    rows = np.zeros(int(row_base[n]) + 1, sc.ROW_DTYPE)
    out.fill(0)
    rows.fill(0)
    for _ in range(2):  # the first call warms the context's staging and device buffers
        t = time.perf_counter()
        st = ctx2.decode_batch_into(codec, sub, sub_off, out, rows, meta, out_off, row_base)
        el = time.perf_counter() - t
        assert st == sc.OK and (meta["status"] == 0).all()
    dec = int(np.sum(meta["data_len"].astype(np.int64) + 2 * meta["n_rows"].astype(np.int64) + 2))
    res = {"GiBps_decoded": round(dec / el / 2**30, 2), "blocks": n,
           "h2d_GBps": round(int(sub_off[n]) / el / 1e9, 2),
           # what crosses the link back: decoded bytes, the rows densely (slate_row, 16 B, of decoded
           # blocks only: rows_pack) and the metas
           "d2h_GBps": round((dec + 16 * int(np.sum(np.where(meta["status"] == 0, meta["n_rows"], 0).astype(np.int64)))
                              + 16 * n) / el / 1e9, 2),
           "path": "slate_block_decode_batch: pageable caller buffers, page-locked staging, 2 stream lanes"}
    ctx3 = sc.Context(ctx.device)
    for _ in range(2):  # the same caller buffers; the first call warms the second context
        t = time.perf_counter()
        st = sc.decode_sharded_into([ctx2, ctx3], codec, sub, sub_off, out, rows, meta, out_off, row_base)
        el = time.perf_counter() - t
        assert st == sc.OK and (meta["status"] == 0).all()
    res["sharded_2ctx_GiBps_decoded"] = round(dec / el / 2**30, 2)
    ctx3.close()
    # eight contexts on this one GPU (the in-process path of an 8-GPU node), each with its share of
    # this process's CPUs as copy threads: what the host gather / scatter sustains through one link
    cpus = host_cpus()
    ctxs = [sc.Context(ctx.device) for _ in range(8)]
    for c in ctxs:
        c.set_copy_threads(max(1, cpus // 8))
    for _ in range(2):
        t = time.perf_counter()
        st = sc.decode_sharded_into(ctxs, codec, sub, sub_off, out, rows, meta, out_off, row_base)
        el = time.perf_counter() - t
        assert st == sc.OK and (meta["status"] == 0).all()
    res["sharded_8ctx_GiBps_decoded"] = round(dec / el / 2**30, 2)
    res["sharded_8ctx_copy_threads"] = max(1, cpus // 8)
    # the same calls with page-locked outputs (slate_hostbuf): the GPU writes decoded bytes and rows
    # straight into the caller's buffers, so no staging copy and no host memcpy of the output
    hb_o, hb_r = sc.HostBuf(ctx2, out.nbytes), sc.HostBuf(ctx2, rows.nbytes)
    out_h, rows_h = hb_o.view[: out.nbytes], hb_r.view[: rows.nbytes].view(sc.ROW_DTYPE)
    for name, cs in (("pinned_out_1ctx_GiBps_decoded", None), ("pinned_out_sharded_8ctx_GiBps_decoded", ctxs)):
        for _ in range(2):
            t = time.perf_counter()
            if cs is None:
                st = ctx2.decode_batch_into(codec, sub, sub_off, out_h, rows_h, meta, out_off, row_base)
            else:
                st = sc.decode_sharded_into(cs, codec, sub, sub_off, out_h, rows_h, meta, out_off, row_base)
            el = time.perf_counter() - t
            assert st == sc.OK and (meta["status"] == 0).all()
        res[name] = round(dec / el / 2**30, 2)
    assert out_h[: int(out_off[n])].tobytes() == out[: int(out_off[n])].tobytes(), "pinned output bytes"
    out_h = rows_h = None
    hb_o.free()
    hb_r.free()
    for c in ctxs:
        c.close()
    ctx2.close()
    res["host_memcpy_GBps"] = host_memcpy_rate(cpus)
    return res


def host_memcpy_rate(threads, nbytes=1 << 30, piece=64 << 20):
    """Host memory bandwidth of plain copies over `threads` threads (numpy releases the GIL):
    the ceiling of the host pipelines' staging copies on this box's CPU share."""
    import concurrent.futures as cf
    src = np.ones(nbytes, np.uint8)
    dst = np.zeros(nbytes, np.uint8)
    pieces = [(o, min(nbytes, o + piece)) for o in range(0, nbytes, piece)]
    with cf.ThreadPoolExecutor(max_workers=threads) as ex:
        best = 0.0
        for _ in range(3):
            t = time.perf_counter()
            list(ex.map(lambda ab: np.copyto(dst[ab[0]:ab[1]], src[ab[0]:ab[1]]), pieces))
            best = max(best, nbytes / (time.perf_counter() - t) / 1e9)
    return round(best, 1)


CODEC_RESTATEMENT = {0: "no codec", 1: "golang/snappy", 2: "compress/zlib+flate", 3: "LZ4 frame",
                     4: "RFC 8878 zstd (oracle/zstd_oracle.c)"}


def cpu_baseline(codec, blob, in_off, seconds):
    """The oracle (C restatement of the Go path) timed on this host: bounded sample, on one
    thread and on every CPU this process may use (affinity mask and cgroup quota)."""
    from oracle import binding as ob
    n = len(in_off) - 1
    chunk = 20_000
    res = {}
    for threads in sorted({1, min(64, host_cpus())}):
        done = 0
        dec = 0
        t = time.perf_counter()
        while time.perf_counter() - t < seconds / (1 if threads == 1 else 2) and done < n:
            a, b = done, min(n, done + chunk * max(1, threads // 8))
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
                      f"{mt} threads = every CPU this process may use, at most 64 (affinity/cgroup; os.cpu_count() = "
                      f"{os.cpu_count()})",
            "single_thread": {"value": round(res[1][0], 3), "cores": 1, "blocks": res[1][1]},
            "cpu_model": cpu_model}


if __name__ == "__main__":
    main()
