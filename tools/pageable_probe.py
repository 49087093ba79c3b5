#!/usr/bin/env python3
"""Host-buffer staging floor of snappy_compress_buffer / snappy_decompress_buffer:
pageable <-> HBM through the runtime (hipMemcpy of a pageable buffer), and a
pageable <-> pinned memcpy split over 1..16 threads (ctypes memmove releases the
GIL), i.e. what a multi-threaded staging copy in front of a pinned DMA could
reach.  256 MiB, best of 3."""
import ctypes
import threading
import time

import numpy as np
import torch

N = 256 << 20


def best(f, reps=3):
    t = float("inf")
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        t = min(t, time.perf_counter() - t0)
    return N / t / 1e9


def par_copy(dst, src, threads):
    part = (N + threads - 1) // threads

    def w(i):
        o = i * part
        m = min(part, N - o)
        if m > 0:
            ctypes.memmove(dst + o, src + o, m)

    ts = [threading.Thread(target=w, args=(i,)) for i in range(1, threads)]
    for t in ts:
        t.start()
    w(0)
    for t in ts:
        t.join()


page = np.random.default_rng(1).integers(0, 255, N, dtype=np.uint8)
page2 = np.empty(N, dtype=np.uint8)
page2[:] = 0
pin = torch.empty(N, dtype=torch.uint8, pin_memory=True)
pin.fill_(1)
dev = torch.empty(N, dtype=torch.uint8, device="cuda")
pt = torch.from_numpy(page)
pt2 = torch.from_numpy(page2)
print(f"runtime pageable h2d: {best(lambda: dev.copy_(pt)):6.1f} GB/s", flush=True)
print(f"runtime pageable d2h: {best(lambda: pt2.copy_(dev)):6.1f} GB/s", flush=True)
print(f"pinned h2d:           {best(lambda: dev.copy_(pin)):6.1f} GB/s", flush=True)
print(f"pinned d2h:           {best(lambda: pin.copy_(dev)):6.1f} GB/s", flush=True)
for th in (1, 2, 4, 8, 16):
    r_in = best(lambda: par_copy(pin.data_ptr(), page.ctypes.data, th))
    r_out = best(lambda: par_copy(page2.ctypes.data, pin.data_ptr(), th))
    print(f"memcpy {th:2d} threads: pageable->pinned {r_in:6.1f} GB/s  pinned->pageable {r_out:6.1f} GB/s", flush=True)
# sizes and offsets that are not multiples of 4 KiB (a compressed stream's length):
# does the runtime still take the DMA path?
for off, m in ((0, N - 3), (0, 145000001), (1, 145000000), (0, 145000000 - 145000000 % 4096)):
    src = pt[off:off + m]
    dst = dev[:m]
    t = float("inf")
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dst.copy_(src)
        torch.cuda.synchronize()
        t = min(t, time.perf_counter() - t0)
    t2 = float("inf")
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pt2[off:off + m].copy_(dev[:m])
        torch.cuda.synchronize()
        t2 = min(t2, time.perf_counter() - t0)
    print(f"pageable offset {off} size {m}: h2d {m / t / 1e9:6.1f} GB/s  d2h {m / t2 / 1e9:6.1f} GB/s", flush=True)
