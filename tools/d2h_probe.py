#!/usr/bin/env python3
"""Host <-> HBM copy rates in 64 MiB chunks into pinned buffers (what the FILE*
pipelines do), one chunk after another and with three in flight: the PCIe
floor of snappy_decompress(FILE*) / snappy_compress(FILE*)."""
import time

import torch

CH = 64 << 20
n = 4 << 30
x = torch.empty(n, dtype=torch.uint8, device="cuda")
x.fill_(7)
hs = [torch.empty(CH, dtype=torch.uint8, pin_memory=True) for _ in range(3)]
s = torch.cuda.Stream()
for mode in ("d2h serial", "d2h 3 in flight", "h2d serial", "h2d 3 in flight"):
    for rep in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        evs = []
        with torch.cuda.stream(s):
            for k in range(n // CH):
                h = hs[k % 3]
                if "3 in flight" in mode and len(evs) >= 3:
                    evs[k - 3].synchronize()
                if mode.startswith("d2h"):
                    h.copy_(x[k * CH:(k + 1) * CH], non_blocking=True)
                else:
                    x[k * CH:(k + 1) * CH].copy_(h, non_blocking=True)
                e = torch.cuda.Event()
                e.record(s)
                evs.append(e)
                if "serial" in mode:
                    e.synchronize()
        s.synchronize()
        dt = time.perf_counter() - t
        print(f"{mode:18s} rep {rep}: {n / dt / 1e9:6.1f} GB/s", flush=True)
