"""ctypes wrapper of the CPU restatement (liboracle.so) and of the compiled
reference (_ref/libsnappy_ref.so).  TEST INFRASTRUCTURE ONLY: imported by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the
product package."""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_orc = None
_ref = None


def orc():
    global _orc
    if _orc is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run make -C oracle")
        l = ctypes.CDLL(path)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        l.oracle_compress.restype = sz
        l.oracle_compress.argtypes = [vp, sz, vp]
        l.oracle_compress_block.restype = sz
        l.oracle_compress_block.argtypes = [vp, ctypes.c_uint32, vp]
        l.oracle_max_compressed_length.restype = sz
        l.oracle_max_compressed_length.argtypes = [sz]
        l.oracle_decompress.restype = ctypes.c_int
        l.oracle_decompress.argtypes = [vp, sz, vp, sz, ctypes.POINTER(sz)]
        l.oracle_compress_streams.restype = sz
        l.oracle_compress_streams.argtypes = [vp, sz, ctypes.c_uint32, vp, vp, ctypes.c_int]
        l.oracle_compress_threaded.restype = sz
        l.oracle_compress_threaded.argtypes = [vp, sz, vp, ctypes.c_int]
        l.oracle_compress_streams_strided.restype = None
        l.oracle_compress_streams_strided.argtypes = [vp, sz, ctypes.c_uint32, vp, sz, vp, ctypes.c_int]
        l.oracle_decompress_streams.restype = ctypes.c_int
        l.oracle_decompress_streams.argtypes = [vp, vp, sz, ctypes.c_uint32, vp, ctypes.c_int]
        l.oracle_varint_encode.restype = ctypes.c_uint32
        l.oracle_varint_encode.argtypes = [ctypes.c_uint64, vp]
        l.oracle_max_block_bytes.restype = sz
        l.oracle_max_block_bytes.argtypes = [ctypes.c_uint32]
        _orc = l
    return _orc


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _arr(data) -> np.ndarray:
    return np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else np.ascontiguousarray(data)


def compress(data) -> bytes:
    a = _arr(data)
    out = np.empty(orc().oracle_max_compressed_length(a.size) + 16, dtype=np.uint8)
    n = orc().oracle_compress(_ptr(a), a.size, _ptr(out))
    return out[:n].tobytes()


def compress_parallel(a: np.ndarray, threads: int = 16) -> np.ndarray:
    """compress() of one whole stream with its 65,536-byte blocks spread over
    `threads` threads (blocks are independent); same bytes, as an array."""
    a = _arr(a)
    out = np.empty(orc().oracle_max_compressed_length(a.size) + 16, dtype=np.uint8)
    n = orc().oracle_compress_threaded(_ptr(a), a.size, _ptr(out), threads)
    return out[:n]


def decompress(data, cap: int | None = None) -> bytes:
    a = _arr(data)
    if a.size == 0:
        return b""
    # declared length from the varint
    v, sh = 0, 0
    for b in a[:10]:
        v |= (int(b) & 0x7F) << sh
        sh += 7
        if not b & 0x80:
            break
    out = np.empty(max(v, 1), dtype=np.uint8)
    got = ctypes.c_size_t(0)
    rc = orc().oracle_decompress(_ptr(a), a.size, _ptr(out), v, ctypes.byref(got))
    if rc != 0:
        raise ValueError(f"oracle_decompress rc={rc}")
    return out[: got.value].tobytes()


def compress_streams(a: np.ndarray, chunk: int, threads: int = 8):
    """Independent snappy_compress() streams of each `chunk` bytes ->
    (payload uint8 array, offsets uint64 array)."""
    ns = (a.size + chunk - 1) // chunk
    out = np.empty(a.size + ns * (chunk // 32 + 48) + 16, dtype=np.uint8)
    offs = np.empty(ns + 1, dtype=np.uint64)
    n = orc().oracle_compress_streams(_ptr(a), a.size, chunk, _ptr(out), _ptr(offs), threads)
    return out[:n], offs


def decompress_streams(payload: np.ndarray, offs: np.ndarray, n: int, chunk: int, threads: int = 8) -> np.ndarray:
    out = np.empty(max(n, 1), dtype=np.uint8)
    rc = orc().oracle_decompress_streams(_ptr(payload), _ptr(offs), n, chunk, _ptr(out), threads)
    if rc != 0:
        raise ValueError(f"oracle_decompress_streams rc={rc}")
    return out[:n]


# ---- the compiled reference (this container only) --------------------------
def ref():
    global _ref
    if _ref is None:
        path = os.path.join(HERE, "_ref", "libsnappy_ref.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run make -C oracle ref (needs /root/reference)")
        l = ctypes.CDLL(path)
        for name in ("ref_compress_mem", "ref_decompress_mem", "ref_compress_bst_mem"):
            fn = getattr(l, name)
            fn.restype = ctypes.c_longlong
            fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
        _ref = l
    return _ref


def _ref_call(name: str, data, cap: int) -> bytes:
    a = _arr(data)
    out = np.empty(max(cap, 1), dtype=np.uint8)
    n = getattr(ref(), name)(_ptr(a), a.size, _ptr(out), cap)
    if n < 0:
        raise RuntimeError(f"{name} failed: {n}")
    return out[:n].tobytes()


def ref_compress(data) -> bytes:
    return _ref_call("ref_compress_mem", data, len(data) + len(data) // 32 + 4096)


def ref_compress_bst(data) -> bytes:
    return _ref_call("ref_compress_bst_mem", data, len(data) + len(data) // 32 + 4096)


def ref_decompress(data, n_out: int) -> bytes:
    return _ref_call("ref_decompress_mem", data, n_out + 16)
