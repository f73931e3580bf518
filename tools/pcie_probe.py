"""PCIe copy probe (dev tool): H2D alone, D2H alone, both at once on two
streams, pinned host buffers. Prints GB/s per leg."""
import time

import torch

N = 512 << 20
dev = torch.device("cuda", 0)
h_a = torch.empty(N, dtype=torch.uint8, pin_memory=True)
h_b = torch.empty(N, dtype=torch.uint8, pin_memory=True)
d_a = torch.empty(N, dtype=torch.uint8, device=dev)
d_b = torch.empty(N, dtype=torch.uint8, device=dev)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def h2d():
    with torch.cuda.stream(s1):
        d_a.copy_(h_a, non_blocking=True)


def d2h():
    with torch.cuda.stream(s2):
        h_b.copy_(d_b, non_blocking=True)


def both():
    h2d()
    d2h()


def chunked_both(k=8):
    for i in range(k):
        sl = slice(i * N // k, (i + 1) * N // k)
        with torch.cuda.stream(s1):
            d_a[sl].copy_(h_a[sl], non_blocking=True)
        with torch.cuda.stream(s2):
            h_b[sl].copy_(d_b[sl], non_blocking=True)


for name, fn, nbytes in [("h2d", h2d, N), ("d2h", d2h, N), ("both", both, 2 * N),
                         ("both_chunked", chunked_both, 2 * N)]:
    dt = t(fn)
    print(f"{name:14s} {dt * 1e3:8.2f} ms  {nbytes / dt / 1e9:6.1f} GB/s", flush=True)
