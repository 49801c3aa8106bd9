"""Profiling aid (tooling): how many configs[4] Zstd blocks the fast path (zstd_fast.hip) takes,
and why the others went to the exact path.  Reads the decode scratch after a plan + decode
(layout of decode.hip carve()) and re-parses the handed-back blocks on the host."""
import collections
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "slatedb-go_amd")]
import slatecodec as sc  # noqa: E402
from tools import workload as wl  # noqa: E402

SEQS = 16


def a16(x):
    return (x + 15) & ~15


def offsets(n):
    tiles = (n + 1 + 1023) // 1024
    p = a16(2 * tiles * 8) + 16 + a16(n * 4) + 16
    cnt = p
    p += 16
    lst = p
    p += a16(n * 4)
    rec = p
    return cnt, lst, rec


def shape(f: bytes):
    """(literal type, nseq, modes, sequences-section bytes) of a one-block frame, or a reason."""
    if f[:4] != b"\x28\xb5\x2f\xfd":
        return "magic"
    fhd = f[4]
    p = 5 + (0 if (fhd >> 5) & 1 else 1) + [0, 1, 2, 4][fhd & 3] + [1 if (fhd >> 5) & 1 else 0, 2, 4, 8][fhd >> 6]
    bh = int.from_bytes(f[p:p + 3], "little")
    p += 3
    if not bh & 1:
        return "multi-block"
    if (bh >> 1) & 3 != 2:
        return f"block type {(bh >> 1) & 3}"
    bs = bh >> 3
    b0 = f[p]
    lt, sf = b0 & 3, (b0 >> 2) & 3
    if lt > 1:
        return f"literals type {lt}"
    hs = 2 if sf == 1 else 3 if sf == 3 else 1
    nl = (b0 >> 4) + (f[p + 1] << 4) if sf == 1 else ((b0 >> 4) + (f[p + 1] << 4) + (f[p + 2] << 12) if sf == 3 else b0 >> 3)
    q = p + hs + (nl if lt == 0 else 1)
    c0 = f[q]
    ns = c0 if c0 < 128 else (((c0 - 128) << 8) + f[q + 1] if c0 < 255 else f[q + 1] + (f[q + 2] << 8) + 0x7F00)
    if ns > SEQS:
        return f"nseq {ns}"
    return f"fast shape (nseq {ns}, seq section {p + bs - q} B, modes {f[q + 1 + (c0 >= 128)] if ns else 0:#x})"


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    dec, doff = wl.mixed_blocks(n)
    blob, in_off = wl.encode_blocks(sc.ZSTD, dec, doff)
    dev = torch.device("cuda", 0)
    ctx = sc.Context(0)
    d_in = torch.from_numpy(blob).to(dev)
    d_off = torch.from_numpy(in_off.view(np.int64)).to(dev)
    d_oo = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d_rb = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d_sc = torch.zeros(sc.decode_scratch_bytes(n) + 64, dtype=torch.uint8, device=dev)
    cnt, _, _ = offsets(n)
    ctx.decode_plan_device(sc.ZSTD, d_in.data_ptr(), d_off.data_ptr(), n, d_oo.data_ptr(), d_rb.data_ptr(),
                           d_sc.data_ptr())
    ctx.synchronize()
    plan_list = int(d_sc[cnt:cnt + 4].cpu().numpy().view(np.uint32)[0])
    d_out = torch.empty(int(d_oo[n].item()) + 16, dtype=torch.uint8, device=dev)
    d_meta = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    d_rows = torch.empty(int(d_rb[n].item()) * 16 + 16, dtype=torch.uint8, device=dev)
    ctx.decode_device(sc.ZSTD, d_in.data_ptr(), d_off.data_ptr(), n, d_out.data_ptr(), d_oo.data_ptr(),
                      d_meta.data_ptr(), d_rows.data_ptr(), d_rb.data_ptr())
    ctx.synchronize()
    meta = np.frombuffer(d_meta.cpu().numpy().tobytes(), dtype=sc.META_DTYPE)
    lines = open(os.environ["SLATE_ZF_STATS"]).read().split("\n")
    nb, fast, count, sum_fail = (int(x) for x in lines[0].split())
    handed = [tuple(int(x) for x in l.split()) for l in lines[1:] if l.strip()]
    print(f"blocks {nb}: plan handed to the wave plan {plan_list}; fast after parse {fast}; decode handed to the "
          f"exact path {count} (checksum mismatch {sum_fail}); statuses "
          f"{dict(collections.Counter(int(s) for s in meta['status']))}")
    why = collections.Counter()
    for b, was_fast in handed[:4000]:
        f = bytes(blob[int(in_off[b]):int(in_off[b + 1]) - 4])
        why[("C " if was_fast else "A ") + shape(f).split(" (")[0]] += 1
    print(why.most_common(10))
    for b, was_fast in handed[:6]:
        f = bytes(blob[int(in_off[b]):int(in_off[b + 1]) - 4])
        print(b, "checksum" if was_fast else "parse", shape(f), "frame", len(f), "shift", int(in_off[b]) & 15)


if __name__ == "__main__":
    main()
