"""Seeded synthetic inputs (csrc/datagen.c): text 'T', random 'R', 64-byte
repeat 'P', zeros 'Z', Appendix-B LCG 'L' and period-k repeats.  Used by the
tests and bench.py; regenerates bit-identical bytes on the GPU box."""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "libsnappy_datagen.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run make -C lightweight-snappy_amd")
        l = ctypes.CDLL(path)
        l.snappy_gen_fill_at.restype = ctypes.c_int
        l.snappy_gen_fill_at.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int,
                                         ctypes.c_uint64, ctypes.c_int]
        _lib = l
    return _lib


GEN_CHUNK = 1 << 20  # the generators are counter-based per 1 MiB (csrc/datagen.c)


def fill(out: np.ndarray, kind: str, seed: int, offset: int = 0, threads: int = 8) -> np.ndarray:
    """Fill a contiguous uint8 array with bytes [offset, offset+len) of a generator."""
    assert out.dtype == np.uint8 and out.flags["C_CONTIGUOUS"]
    lead = offset % GEN_CHUNK
    if lead and kind != "L" and out.size:  # unaligned start: the first chunk through a bounce buffer
        head = min(out.size, GEN_CHUNK - lead)
        tmp = np.empty(lead + head, dtype=np.uint8)
        fill(tmp, kind, seed, offset - lead, threads)
        out[:head] = tmp[lead:]
        if head < out.size:
            fill(out[head:], kind, seed, offset + head, threads)
        return out
    rc = lib().snappy_gen_fill_at(out.ctypes.data_as(ctypes.c_void_p), out.size, offset, ord(kind), seed, threads)
    if rc != 0:
        raise ValueError(f"datagen kind={kind!r} offset={offset}: rc={rc}")
    return out


def make(kind: str, n: int, seed: int = 0, period: int = 0) -> np.ndarray:
    """kind in T/R/P/Z/L, or 'K' = `period` random bytes (seed) tiled."""
    out = np.empty(n, dtype=np.uint8)
    if n == 0:
        return out
    if kind == "K":
        base = np.empty(period, dtype=np.uint8)
        fill(base, "R", seed)
        reps = (n + period - 1) // period
        out[:] = np.tile(base, reps)[:n]
        return out
    return fill(out, kind, seed)
