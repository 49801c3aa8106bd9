"""DMA probe (tooling): pinned H2D and D2H alone and concurrently on two streams, and a
device->pinned-host copy done by a kernel (torch copy_ between cuda and pinned with
non_blocking)."""
import sys
import time

import torch


def rate(f, nbytes, reps=5):
    f(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    return nbytes * reps / (time.perf_counter() - t) / 1e9


def main():
    n = 1 << 28
    ph = torch.empty(n, dtype=torch.uint8).pin_memory()
    ph2 = torch.empty(n, dtype=torch.uint8).pin_memory()
    d1 = torch.empty(n, dtype=torch.uint8, device="cuda")
    d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    print("H2D alone", rate(lambda: d1.copy_(ph, non_blocking=True), n))
    print("D2H alone", rate(lambda: ph2.copy_(d2, non_blocking=True), n))

    def both():
        with torch.cuda.stream(s1):
            d1.copy_(ph, non_blocking=True)
        with torch.cuda.stream(s2):
            ph2.copy_(d2, non_blocking=True)
    print("H2D+D2H concurrent (GB/s total)", rate(both, 2 * n))
    # a kernel writing pinned host memory directly (zero-copy view of the pinned buffer)
    hv = ph2  # torch cannot map host memory into a kernel; emulate with a device copy for reference
    print("D2D", rate(lambda: d1.copy_(d2), n))
    sys.stdout.flush()


if __name__ == "__main__":
    main()
