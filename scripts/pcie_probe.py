"""Host <-> device copy rates for one 4K RGB frame (24.9 MB) on this box:
pageable vs pinned sources, a warm (cached) vs cold (8 distinct) source, and the
host memcpy into a pinned buffer -- the ceiling of the PCIe-inclusive path.
  python scripts/pcie_probe.py"""
import time

import numpy as np
import torch

N = 3840 * 2160 * 3
dev = torch.device("cuda", 0)
d = torch.empty(N, dtype=torch.uint8, device=dev)
pinned = torch.empty(N, dtype=torch.uint8).pin_memory()
srcs = [np.random.default_rng(i).integers(0, 256, N, dtype=np.uint8) for i in range(8)]
tsrc = [torch.from_numpy(s) for s in srcs]


def rate(fn, reps=20):
    fn(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        fn(i)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    return f"{dt * 1e3:.3f} ms  {N / dt / 1e9:.1f} GB/s"


print("H2D pageable, same source  ", rate(lambda i: d.copy_(tsrc[0])))
print("H2D pageable, 8 sources    ", rate(lambda i: d.copy_(tsrc[i % 8])))
print("H2D pinned                 ", rate(lambda i: d.copy_(pinned, non_blocking=True)))
print("D2H pinned                 ", rate(lambda i: pinned.copy_(d, non_blocking=True)))
print("host memcpy -> pinned, 8 sources", rate(lambda i: pinned.numpy().__setitem__(slice(None), srcs[i % 8])))
