"""Host pipeline probe (tooling): slate_block_decode_batch on the configs[1] block set from host
buffers, 262 k blocks, with SLATE_HOST_TRACE phase times; plus raw host memcpy and pinned
H2D/D2H rates of this box for reference."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "slatedb-go_amd")]
import torch  # noqa: E402
import slatecodec as sc  # noqa: E402
from tools import workload as wl  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
    blob, off = wl.block_set(sc.SNAPPY, 1, 0, n, threads=16)
    a = np.ones(1 << 28, np.uint8)
    b = np.empty_like(a)
    t = time.perf_counter(); np.copyto(b, a); el = time.perf_counter() - t
    print(f"numpy memcpy 1 thread: {a.nbytes / el / 1e9:.1f} GB/s", file=sys.stderr)
    pin = torch.empty(1 << 28, dtype=torch.uint8).pin_memory()
    dev = torch.empty(1 << 28, dtype=torch.uint8, device="cuda")
    for name, f in (("H2D pinned", lambda: dev.copy_(pin, non_blocking=True)),
                    ("D2H pinned", lambda: pin.copy_(dev, non_blocking=True))):
        f(); torch.cuda.synchronize()
        t = time.perf_counter(); f(); torch.cuda.synchronize(); el = time.perf_counter() - t
        print(f"{name}: {pin.numel() / el / 1e9:.1f} GB/s", file=sys.stderr)
    ctx = sc.Context(0)
    out_off = np.zeros(n + 1, np.uint64); row_base = np.zeros(n + 1, np.uint64); meta = np.zeros(n, sc.META_DTYPE)
    ctx.decode_batch_into(sc.SNAPPY, blob, off, np.zeros(1, np.uint8), np.zeros(1, sc.ROW_DTYPE), meta, out_off, row_base)
    out = np.zeros(int(out_off[n]) + 16, np.uint8); rows = np.zeros(int(row_base[n]) + 1, sc.ROW_DTYPE)
    out.fill(0); rows.fill(0)
    for i in range(3):
        t = time.perf_counter()
        st = ctx.decode_batch_into(sc.SNAPPY, blob, off, out, rows, meta, out_off, row_base)
        el = time.perf_counter() - t
        assert st == 0
        print(f"call {i}: {el * 1e3:.1f} ms, {int(out_off[n]) / el / 2**30:.2f} GiB/s (out_off basis)", file=sys.stderr)


if __name__ == "__main__":
    main()
