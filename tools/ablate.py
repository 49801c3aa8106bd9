"""Profiling aid: times the decode kernel with parts switched off
(SLATE_DEBUG_MODE bits: wave-per-block kernel 1 skip CRC, 2 skip Snappy, 4 skip rows, 8 skip
write-back, 16 use it for Snappy; lane-per-block kernel 32 v1 kernel, 64 skip CRC, 128 skip rows,
256 far copies from the ring, 512 record per-round iterations/cycles, 1024 drop output stores,
2048 skip the flush LDS read, 4096 skip the copy-source LDS read, 8192 no holes, 16384 drop row
stores, 32768 drop far-copy loads, 65536 skip the row verification),
interleaved rounds in one process.  Results are wrong by design; timing only."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "slatedb-go_amd")]
import slatecodec as sc  # noqa: E402
from tools import workload as wl  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    modes = [int(x, 0) for x in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "1", "2", "4", "8", "15"])]
    codec = int(os.environ.get("SLATE_ABLATE_CODEC", sc.SNAPPY))  # 3: LZ4 frames
    if codec == sc.ZSTD:  # configs[4] mixed; zstd bits: 2 skip decompression, 1<<17 Huffman streams,
        dec, doff = wl.mixed_blocks(n)  # 1<<18 XXH64, 1<<19 sequence copies
        blob, in_off = wl.encode_blocks(codec, dec, doff)
        dec_bytes = int(doff[-1])
    else:
        blob, in_off, dec_bytes = wl.snappy_vhalf(n, codec=codec)
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    ctx = sc.Context(0)
    ctx.set_stream(s.cuda_stream)
    with torch.cuda.stream(s):
        d_in = torch.from_numpy(blob).to(dev)
        d_off = torch.from_numpy(in_off.view(np.int64)).to(dev)
        d_oo = torch.empty(n + 1, dtype=torch.int64, device=dev)
        d_rb = torch.empty(n + 1, dtype=torch.int64, device=dev)
        d_sc = torch.empty(sc.decode_scratch_bytes(n) + 64, dtype=torch.uint8, device=dev)
        ctx.decode_plan_device(codec, d_in.data_ptr(), d_off.data_ptr(), n, d_oo.data_ptr(), d_rb.data_ptr(),
                               d_sc.data_ptr())
        s.synchronize()
        d_out = torch.empty(int(d_oo[n].item()) + 16, dtype=torch.uint8, device=dev)
        d_meta = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        d_rows = torch.empty(int(d_rb[n].item()) * 16 + 16, dtype=torch.uint8, device=dev)
        res = {m: [] for m in modes}
        for rnd in range(5):
            for m in modes:
                os.environ["SLATE_DEBUG_MODE"] = str(m)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(s)
                ctx.decode_device(codec, d_in.data_ptr(), d_off.data_ptr(), n, d_out.data_ptr(), d_oo.data_ptr(),
                                  d_meta.data_ptr(), d_rows.data_ptr(), d_rb.data_ptr())
                b.record(s)
                b.synchronize()
                if rnd:
                    res[m].append(a.elapsed_time(b))
    os.environ.pop("SLATE_DEBUG_MODE", None)
    stats = None
    if any(m & 512 for m in modes):  # per-round loop iterations and cycles (LPB kernel, last 512-mode run)
        m512 = [m for m in modes if m & 512][-1]
        os.environ["SLATE_DEBUG_MODE"] = str(m512)
        ctx.decode_device(codec, d_in.data_ptr(), d_off.data_ptr(), n, d_out.data_ptr(), d_oo.data_ptr(),
                          d_meta.data_ptr(), d_rows.data_ptr(), d_rb.data_ptr())
        s.synchronize()
        os.environ.pop("SLATE_DEBUG_MODE", None)
        meta = np.frombuffer(d_meta.cpu().numpy().tobytes(), dtype=sc.META_DTYPE)
        it = meta["detail"][0::64].astype(np.float64)
        cyc = meta["detail"][1::64].astype(np.uint32).astype(np.float64)
        post = meta["detail"][2::64].astype(np.uint32).astype(np.float64)
        waited = meta["detail"][3::64].astype(np.uint32).astype(np.float64)
        stats = {"mode": m512, "iters_median": float(np.median(it)), "iters_max": float(it.max()),
                 "cycles_median": float(np.median(cyc)), "cycles_per_iter": float(np.median(cyc / np.maximum(it, 1))),
                 "final_cycles_median": float(np.median(post)), "rows_wait_median": float(np.median(waited))}
    out = {str(m): {"ms_median": float(np.median(v)), "ms_min": float(np.min(v)),
                    "GiBps": dec_bytes / (np.median(v) * 1e-3) / 2**30} for m, v in res.items()}
    print(json.dumps({"blocks": n, "decoded_bytes": dec_bytes, "modes": out, "round_stats": stats}, indent=1))


if __name__ == "__main__":
    main()
