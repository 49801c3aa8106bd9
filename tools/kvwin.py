"""The kv100 Zstd blocks' sequences-section shape, for phase A's LDS window sizes (zstd_fast.hip
zs_fse_parse_kernel): table accuracy logs, header bytes, and the 16-byte chunks each block's section
needs from the chunk holding its first byte and from the one holding its bitstream's first byte
(tests/zsection.py).  CPU only: python3 tools/kvwin.py [blocks]."""
import collections
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import workload as wl  # noqa: E402
from tests.zsection import section_shape  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
dec, dec_off = wl.decoded_blocks(N, seed=20250307, half=True)
blob, off = wl.encode_blocks(4, dec, dec_off, threads=8)
logs, hdr, nseq, from_sec, from_bits = collections.Counter(), [], [], [], []
other = 0
for i in range(N):
    z = section_shape(bytes(blob[int(off[i]):int(off[i + 1])]), int(off[i]) & 15)
    if z is None:
        other += 1
        continue
    logs[z["logs"]] += 1
    hdr.append(z["hdr"])
    nseq.append(z["nseq"])
    from_sec.append(z["chunks_from_section"])
    from_bits.append(z["chunks_from_bitstream"])


def over(x):
    x = np.array(x)
    return {k: int((x > k).sum()) for k in (8, 9, 10, 11, 12)}


print("blocks", N, "other shapes", other, "sequences mean", np.mean(nseq), "max", max(nseq))
print("table logs (LL, OF, ML)", logs.most_common(8))
print("header bytes mean", np.mean(hdr), "max", max(hdr))
print("chunks from the section's first: blocks over k", over(from_sec), "max", max(from_sec))
print("chunks from the bitstream's first: blocks over k", over(from_bits), "max", max(from_bits))
