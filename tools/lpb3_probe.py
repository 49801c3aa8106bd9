"""Profiling aid (tooling): decode_lpb3 per-round P/M cycles, M rounds and P iterations from a
SLATE_PROFILING_BUILD variant (SLATE_DEBUG_MODE 512 stamps them into meta.detail), and kernel
times with parts switched off (1<<22 P only, 1<<23 no rows).  Results are wrong by design."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "slatedb-go_amd")]
import slatecodec as sc  # noqa: E402
from tools import workload as wl  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    modes = [int(x, 0) for x in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "512", "0x400000", "0x800000", "32"])]
    blob, in_off = wl.block_set(sc.SNAPPY, 0, 1, n, threads=16)
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
        ctx.decode_plan_device(sc.SNAPPY, d_in.data_ptr(), d_off.data_ptr(), n, d_oo.data_ptr(), d_rb.data_ptr(),
                               d_sc.data_ptr())
        torch.cuda.synchronize()
        d_out = torch.empty(int(d_oo[n].item()) + 16, dtype=torch.uint8, device=dev)
        d_meta = torch.empty(n * 16, dtype=torch.uint8, device=dev)
        d_rows = torch.empty(int(d_rb[n].item()) * 16 + 16, dtype=torch.uint8, device=dev)
    for m in modes:
        os.environ["SLATE_DEBUG_MODE"] = str(m)
        ts = []
        for rep in range(6):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            ctx.decode_device(sc.SNAPPY, d_in.data_ptr(), d_off.data_ptr(), n, d_out.data_ptr(), d_oo.data_ptr(),
                              d_meta.data_ptr(), d_rows.data_ptr(), d_rb.data_ptr())
            e1.record(s)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        line = f"mode {m:#x}: {np.median(ts[1:]):.3f} ms"
        if m & 512:
            det = np.frombuffer(d_meta.cpu().numpy().tobytes(), dtype=sc.META_DTYPE)["detail"]
            r0 = np.arange(0, n - 3, 64)
            line += (f"  P cycles/round {np.mean(det[r0]):.0f}  M cycles/round {np.mean(det[r0 + 1]):.0f}"
                     f"  M rounds/round {np.mean(det[r0 + 2]):.1f}  P iters/round {np.mean(det[r0 + 3]):.1f}")
        print(line, flush=True)
    os.environ.pop("SLATE_DEBUG_MODE", None)


if __name__ == "__main__":
    main()
