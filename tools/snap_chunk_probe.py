"""Profiling aid (tooling): the golang/snappy chunk encoder (encode.hip snappy_chunks_kernel, one wave
per 64 KiB chunk) timed on different data (random like a bloom filter, zeros, text-like), through
the library's internal launcher."""
import ctypes as C
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "slatedb-go_amd")]
import slatecodec as sc  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 12_500_002
    L = sc.lib()
    fn = getattr(L, "_ZN5slate20launch_snappy_chunksEP12ihipStream_tPKhmPhPji")
    fn.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_int]
    fn.restype = C.c_int
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev)
    rng = np.random.default_rng(1)
    keys = b"".join(b"k%015d" % i for i in range(n // 16 + 1))[:n]
    data = {"random": rng.integers(0, 256, n, dtype=np.uint8),
            "zeros": np.zeros(n, np.uint8),
            "keys": np.frombuffer(keys, np.uint8).copy(),
            "bloom45": (rng.random(n * 8) < 0.45).astype(np.uint8).reshape(-1, 8) @ (1 << np.arange(8)).astype(np.uint8)}
    nch = (n + 65535) // 65536
    dst = torch.empty(nch * 80 * 1024, dtype=torch.uint8, device=dev)
    lens = torch.empty(nch, dtype=torch.int32, device=dev)
    for name, arr in data.items():
        src = torch.from_numpy(np.ascontiguousarray(arr, np.uint8)).to(dev)
        ts = []
        for rep in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            assert fn(s.cuda_stream, src.data_ptr(), n, dst.data_ptr(), lens.data_ptr(), 256) == 0
            b.record(s)
            b.synchronize()
            ts.append(a.elapsed_time(b))
        tot = int(lens.cpu().numpy().astype(np.int64).sum())
        print(f"{name:8s} {n} B: {min(ts):.3f} ms, encoded {tot} B")


if __name__ == "__main__":
    main()
