"""Profiling aid (tooling): per-kernel times of the CodecZstd decode with parts switched off
(SLATE_DEBUG_MODE bits, profiling variant only: see zstd_fast.hip).  Results are wrong by design.
  python tools/zstd_ablate.py gen FILE N        # configs[4] blocks -> FILE (outside the profiler)
  python tools/zstd_ablate.py run FILE MODE     # 5 plan + decode calls (under rocprofv3)"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "slatedb-go_amd")]
import slatecodec as sc  # noqa: E402
from tools import workload as wl  # noqa: E402


def main():
    what, path = sys.argv[1], sys.argv[2]
    if what == "gen":
        n = int(sys.argv[3])
        dec, doff = wl.mixed_blocks(n)
        blob, in_off = wl.encode_blocks(sc.ZSTD, dec, doff)
        np.savez(path, blob=blob, in_off=in_off)
        return
    z = np.load(path)
    blob, in_off = z["blob"], z["in_off"]
    n = len(in_off) - 1
    os.environ["SLATE_DEBUG_MODE"] = sys.argv[3]
    dev = torch.device("cuda", 0)
    ctx = sc.Context(0)
    d_in = torch.from_numpy(blob).to(dev)
    d_off = torch.from_numpy(in_off.view(np.int64)).to(dev)
    d_oo = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d_rb = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d_sc = torch.empty(sc.decode_scratch_bytes(n) + 64, dtype=torch.uint8, device=dev)
    ctx.decode_plan_device(sc.ZSTD, d_in.data_ptr(), d_off.data_ptr(), n, d_oo.data_ptr(), d_rb.data_ptr(),
                           d_sc.data_ptr())
    ctx.synchronize()
    d_out = torch.empty(int(d_oo[n].item()) + 16, dtype=torch.uint8, device=dev)
    d_meta = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    d_rows = torch.empty(int(d_rb[n].item()) * 16 + 16, dtype=torch.uint8, device=dev)
    for _ in range(5):
        ctx.decode_device(sc.ZSTD, d_in.data_ptr(), d_off.data_ptr(), n, d_out.data_ptr(), d_oo.data_ptr(),
                          d_meta.data_ptr(), d_rows.data_ptr(), d_rb.data_ptr())
    ctx.synchronize()


if __name__ == "__main__":
    main()
