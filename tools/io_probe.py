#!/usr/bin/env python3
"""Host I/O floor of the FILE* pipelines (no GPU): positional writes and reads
of a 4 GiB file in /dev/shm (tmpfs = the page cache the bench's file API
uses), 64 MiB chunks, 1-8 threads, into a new file and into one whose pages
were allocated first (posix_fallocate).  (Linux serialises writes to one file
on its inode lock: extra writer threads only add contention.)  GB/s = bytes / wall second.
Usage: tools/io_probe.py [GiB]"""
import os
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

N = int(float(sys.argv[1] if len(sys.argv) > 1 else 4) * (1 << 30))
CH = 64 << 20
buf = np.random.default_rng(1).integers(0, 256, CH, dtype=np.uint8).tobytes()


def pwrite_all(fd, threads):
    def one(k):
        os.pwrite(fd, buf, k * CH)
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(one, range(N // CH)))


def pread_all(fd, threads):
    bufs = [bytearray(CH) for _ in range(threads)]

    def one(k):  # into a preallocated buffer per thread slot (no allocation in the loop)
        return os.preadv(fd, [bufs[k % threads]], k * CH)
    with ThreadPoolExecutor(threads) as ex:
        return sum(ex.map(one, range(N // CH)))


with tempfile.TemporaryDirectory(dir="/dev/shm", prefix="io_probe_") as d:
    for threads in (1, 2, 4, 8):
        for pre in (False, True):
            p = os.path.join(d, f"f{threads}{int(pre)}")
            fd = os.open(p, os.O_CREAT | os.O_WRONLY | os.O_TRUNC, 0o600)
            t0 = time.perf_counter()
            if pre:
                os.posix_fallocate(fd, 0, N)
            t1 = time.perf_counter()
            pwrite_all(fd, threads)
            t2 = time.perf_counter()
            os.close(fd)
            print(f"write {threads} thread(s){' after fallocate' if pre else ''}: "
                  f"{N / (t2 - t0) / 1e9:6.2f} GB/s total"
                  + (f" (fallocate {t1 - t0:.2f} s, writes {N / (t2 - t1) / 1e9:.2f} GB/s)" if pre else ""), flush=True)
            fd = os.open(p, os.O_RDONLY)
            t0 = time.perf_counter()
            got = pread_all(fd, threads)
            t1 = time.perf_counter()
            os.close(fd)
            assert got == N
            print(f"read  {threads} thread(s): {N / (t1 - t0) / 1e9:6.2f} GB/s", flush=True)
            os.unlink(p)
