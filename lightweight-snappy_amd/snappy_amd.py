"""Python mirror of the reference codec interface, bound to libsnappy_amd.so.

The reference (tturturiello/lightweight-snappy) exposes two C entry points,
``snappy_compress(FILE*, unsigned long long, FILE*)`` (src/snappy_compression.h:8)
and ``snappy_decompress(FILE*, FILE*)`` (src/snappy_decompression.h:15).  This
module offers the same two calls over Python binary file objects, the
in-memory buffer API, and the device-resident batch API (HBM pointers, used by
bench.py and the GPU parity tests).  Everything goes through the C ABI of
libsnappy_amd.so (include/snappy_amd.h), whose kernels run on the MI355X.
There is no CPU fallback: if the library is missing, every call raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import BinaryIO, Optional, Tuple

try:  # share torch's HIP runtime (same SONAME) when torch is present
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is always present in this image
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SNAPPY_AMD_LIB") or os.path.join(HERE, "libsnappy_amd.so")

OK = 0
ERR_ARG = -1
ERR_HEADER = -2
ERR_TRUNCATED = -3
ERR_OFFSET = -4
ERR_OVERRUN = -5
ERR_CAPACITY = -6
ERR_DEVICE = -7
ERR_IO = -8
ERR_UNSUPPORTED = -9
ERR_TIMEOUT = -10
ERR_INDEX = -11
IDX_MAGIC = 0x3158444941504E53  # b"SNPAIDX1" as a little-endian u64

BLOCK = 65536
SINGLE = 0
STREAMS = 1
NO_PREAMBLE = 1
OPT_SERIAL_INDEX = 1    # snappy_amd_set_option: one-wave index walk instead of K5p
OPT_K1R_EXTRA_LDS = 2   # extra dynamic LDS bytes per K1r unit (occupancy experiments)

_NAMES = {
    ERR_ARG: "bad argument",
    ERR_HEADER: "bad varint preamble",
    ERR_TRUNCATED: "truncated element",
    ERR_OFFSET: "copy offset out of range",
    ERR_OVERRUN: "element overruns declared length",
    ERR_CAPACITY: "output buffer too small",
    ERR_DEVICE: "HIP device error",
    ERR_IO: "I/O error",
    ERR_UNSUPPORTED: "unsupported",
    ERR_TIMEOUT: "block dependency wait timed out",
    ERR_INDEX: "sidecar index does not fit the stream",
}

# every function include/*.h declares, with its ctypes signature
_c = ctypes
_SIGS = {
    "snappy_compress": (None, [_c.c_void_p, _c.c_ulonglong, _c.c_void_p]),
    "snappy_decompress": (_c.c_int, [_c.c_void_p, _c.c_void_p]),
    "snappy_compress_bst": (_c.c_int, [_c.c_void_p, _c.c_ulonglong, _c.c_void_p]),
    "snappy_compress_file_indexed": (_c.c_int, [_c.c_void_p, _c.c_ulonglong, _c.c_void_p, _c.c_void_p]),
    "snappy_decompress_file_indexed": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p]),
    "snappy_amd_last_status": (_c.c_int, []),
    "snappy_varint_encode": (_c.c_uint32, [_c.c_uint64, _c.c_void_p]),
    "snappy_varint_decode": (_c.c_uint32, [_c.c_void_p, _c.c_size_t, _c.POINTER(_c.c_uint64)]),
    "snappy_max_compressed_length": (_c.c_size_t, [_c.c_size_t]),
    "snappy_compress_buffer": (_c.c_int, [_c.c_void_p, _c.c_size_t, _c.c_void_p, _c.POINTER(_c.c_size_t)]),
    "snappy_amd_build_config": (_c.c_char_p, []),
    "snappy_amd_bst_compress_file": (_c.c_int, [_c.c_void_p, _c.c_uint64, _c.c_void_p]),
    "snappy_compress_bst_buffer": (_c.c_int, [_c.c_void_p, _c.c_size_t, _c.c_void_p, _c.c_size_t,
                                              _c.POINTER(_c.c_size_t)]),
    "snappy_decompress_buffer": (_c.c_int, [_c.c_void_p, _c.c_size_t, _c.c_void_p, _c.c_size_t,
                                            _c.POINTER(_c.c_size_t)]),
    "snappy_uncompressed_length": (_c.c_int, [_c.c_void_p, _c.c_size_t, _c.POINTER(_c.c_uint64)]),
    "snappy_amd_create": (_c.c_int, [_c.c_int, _c.POINTER(_c.c_void_p)]),
    "snappy_amd_destroy": (None, [_c.c_void_p]),
    "snappy_amd_set_stream": (_c.c_int, [_c.c_void_p, _c.c_void_p]),
    "snappy_amd_get_stream": (_c.c_void_p, [_c.c_void_p]),
    "snappy_amd_device_bytes": (_c.c_size_t, [_c.c_void_p]),
    "snappy_amd_trim": (_c.c_int, [_c.c_void_p]),
    "snappy_amd_num_units": (_c.c_size_t, [_c.c_size_t, _c.c_uint32, _c.c_int]),
    "snappy_amd_max_output": (_c.c_size_t, [_c.c_size_t, _c.c_uint32, _c.c_int]),
    "snappy_amd_compress_device": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_size_t, _c.c_uint32, _c.c_int,
                                              _c.c_void_p, _c.c_void_p, _c.POINTER(_c.c_size_t)]),
    "snappy_amd_decompress_device": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_size_t,
                                                _c.c_uint32, _c.c_int, _c.c_void_p]),
    "snappy_amd_decompress_device_async": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_size_t,
                                                      _c.c_uint32, _c.c_int, _c.c_void_p]),
    "snappy_amd_decompress_status": (_c.c_int, [_c.c_void_p]),
    "snappy_amd_compress_device_ex": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_size_t, _c.c_uint32, _c.c_int,
                                                 _c.c_uint32, _c.c_uint64, _c.c_void_p, _c.c_void_p,
                                                 _c.POINTER(_c.c_size_t)]),
    "snappy_amd_decompress_device_ex": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_void_p, _c.c_size_t, _c.c_uint32,
                                                   _c.c_int, _c.c_uint32, _c.c_uint64, _c.c_void_p, _c.c_int]),
    "snappy_amd_index_device": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_size_t, _c.c_void_p, _c.c_size_t,
                                           _c.POINTER(_c.c_size_t)]),
    "snappy_amd_last_timings": (_c.c_int, [_c.c_void_p, _c.POINTER(_c.c_float), _c.POINTER(_c.c_float),
                                           _c.POINTER(_c.c_float)]),
    "snappy_amd_enable_timing": (_c.c_int, [_c.c_void_p, _c.c_int]),
    "snappy_amd_set_option": (_c.c_int, [_c.c_void_p, _c.c_int, _c.c_int64]),
    "snappy_amd_host_set_device": (_c.c_int, [_c.c_int]),
    "snappy_amd_host_get_device": (_c.c_int, []),
    "snappy_amd_host_release": (_c.c_int, []),
    "snappy_amd_host_pool_size": (_c.c_size_t, []),
    "snappy_compress_buffer_multi": (_c.c_int, [_c.POINTER(_c.c_int), _c.c_int, _c.c_void_p, _c.c_size_t, _c.c_void_p,
                                                _c.POINTER(_c.c_size_t)]),
    "snappy_decompress_buffer_multi": (_c.c_int, [_c.POINTER(_c.c_int), _c.c_int, _c.c_void_p, _c.c_size_t,
                                                  _c.c_void_p, _c.c_size_t, _c.POINTER(_c.c_size_t)]),
    "snappy_amd_host_compress": (_c.c_int, [_c.c_void_p, _c.c_size_t, _c.c_uint64, _c.c_void_p, _c.c_size_t,
                                            _c.POINTER(_c.c_size_t)]),
    "snappy_amd_host_decompress": (_c.c_int, [_c.c_void_p, _c.c_size_t, _c.c_void_p, _c.c_size_t,
                                              _c.POINTER(_c.c_size_t)]),
    "snappy_amd_host_decompress_idx": (_c.c_int, [_c.c_void_p, _c.c_size_t, _c.c_void_p, _c.c_size_t, _c.c_void_p,
                                                  _c.c_size_t, _c.POINTER(_c.c_size_t)]),
    # FILE* in, header value, FILE* out, FILE* sidecar (or NULL), bytes read (C stdio streams; the C host layer)
    "snappy_amd_host_compress_file": (_c.c_int, [_c.c_void_p, _c.c_uint64, _c.c_void_p, _c.c_void_p,
                                                 _c.POINTER(_c.c_uint64)]),
    # FILE* in, sidecar entries (or NULL) and their count, FILE* out
    "snappy_amd_host_decompress_file": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_size_t, _c.c_void_p]),
}
# the reference Buffer cursor helpers, in libsnappy_amd_compat.so (Buffer* is a
# struct of two pointers and a u32)
_COMPAT_SIGS = {
    "init_Buffer": (None, [_c.c_void_p, _c.c_uint]),
    "move_current": (None, [_c.c_void_p, _c.c_uint]),
    "reset": (None, [_c.c_void_p]),
}
COMPAT_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsnappy_amd_compat.so")

_lib: Optional[ctypes.CDLL] = None


class SnappyError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        super().__init__(f"{what}: error {code} ({_NAMES.get(code, 'unknown')})" if what else
                         f"error {code} ({_NAMES.get(code, 'unknown')})")


def lib() -> ctypes.CDLL:
    """Load libsnappy_amd.so (raises loudly if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: run __graft_entry__.build() (make -C lightweight-snappy_amd)")
        l = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(l, name)
            fn.restype = res
            fn.argtypes = args
        _lib = l
    return _lib


def compat_lib() -> ctypes.CDLL:
    """Load libsnappy_amd_compat.so (the reference's Buffer cursor helpers)."""
    if not os.path.exists(COMPAT_PATH):
        raise RuntimeError(f"{COMPAT_PATH} is missing: run __graft_entry__.build()")
    l = ctypes.CDLL(COMPAT_PATH)
    for name, (res, args) in _COMPAT_SIGS.items():
        fn = getattr(l, name)
        fn.restype = res
        fn.argtypes = args
    return l


def _check(rc: int, what: str) -> None:
    if rc != OK:
        raise SnappyError(rc, what)


def _buf(data) -> Tuple[ctypes.c_void_p, int, object]:
    mv = memoryview(data).cast("B")
    n = mv.nbytes
    if n == 0:
        return ctypes.c_void_p(0), 0, None
    if mv.readonly:
        keep = ctypes.create_string_buffer(bytes(mv), n)
    else:
        keep = (ctypes.c_uint8 * n).from_buffer(mv)
    return ctypes.cast(keep, ctypes.c_void_p), n, keep


def build_config() -> str:
    """The kernels' compile-time knobs (snappy_amd_build_config); a product
    library reports measurement=0 for both halves."""
    return lib().snappy_amd_build_config().decode()


# ---- varint (src/varint.c) ------------------------------------------------
def varint_encode(n: int) -> bytes:
    out = ctypes.create_string_buffer(16)
    k = lib().snappy_varint_encode(n, out)
    return out.raw[:k]


def varint_decode(data: bytes) -> Tuple[int, int]:
    """Returns (value, bytes consumed); consumed 0 means malformed."""
    v = ctypes.c_uint64(0)
    p, n, keep = _buf(data)
    k = lib().snappy_varint_decode(p, n, ctypes.byref(v))
    return v.value, k


# ---- in-memory API --------------------------------------------------------
def max_compressed_length(n: int) -> int:
    return lib().snappy_max_compressed_length(n)


def compress(data, header_value: Optional[int] = None) -> bytes:
    """One stream, byte-identical to the reference snappy_compress()."""
    p, n, keep = _buf(data)
    cap = max_compressed_length(n)
    out = ctypes.create_string_buffer(max(cap, 1))
    got = ctypes.c_size_t(0)
    hv = n if header_value is None else header_value
    _check(lib().snappy_amd_host_compress(p, n, hv, out, cap, ctypes.byref(got)), "compress")
    return out.raw[: got.value]


def compress_bst(data) -> bytes:
    """The -b stream, byte-identical to the reference snappy_compress_bst()
    (src/snappy_compression_tree.c:291-306): host threads, no GPU."""
    p, n, keep = _buf(data)
    cap = max_compressed_length(n)
    out = ctypes.create_string_buffer(max(cap, 1))
    got = ctypes.c_size_t(0)
    _check(lib().snappy_compress_bst_buffer(p, n, out, cap, ctypes.byref(got)), "compress_bst")
    return out.raw[: got.value]


def uncompressed_length(data) -> int:
    p, n, keep = _buf(data)
    v = ctypes.c_uint64(0)
    _check(lib().snappy_uncompressed_length(p, n, ctypes.byref(v)), "uncompressed_length")
    return v.value


def _declared_length(data, n: int) -> int:
    """The preamble's N, refused (as the library refuses it) when n bytes of
    stream cannot expand to it: at most 64 output bytes per 3-byte element."""
    N = uncompressed_length(data)
    if N // 22 > n:
        raise SnappyError(ERR_TRUNCATED, "decompress")
    return N


def decompress(data) -> bytes:
    p, n, keep = _buf(data)
    if n == 0:
        return b""
    N = _declared_length(data, n)
    out = ctypes.create_string_buffer(max(N, 1))
    got = ctypes.c_size_t(0)
    _check(lib().snappy_decompress_buffer(p, n, out, N, ctypes.byref(got)), "decompress")
    return out.raw[: got.value]


def compress_multi(data, devices) -> bytes:
    """snappy_compress_buffer_multi: one stream (== compress(data)) made on
    several devices, each compressing a contiguous range of blocks."""
    p, n, keep = _buf(data)
    devs = (ctypes.c_int * len(devices))(*devices)
    out = ctypes.create_string_buffer(max(max_compressed_length(n), 1))
    got = ctypes.c_size_t(0)
    _check(lib().snappy_compress_buffer_multi(devs, len(devices), p, n, out, ctypes.byref(got)), "compress_multi")
    return out.raw[: got.value]


def decompress_multi(data, devices) -> bytes:
    """snappy_decompress_buffer_multi: decompress(data) over several devices."""
    p, n, keep = _buf(data)
    if n == 0:
        return b""
    N = _declared_length(data, n)
    devs = (ctypes.c_int * len(devices))(*devices)
    out = ctypes.create_string_buffer(max(N, 1))
    got = ctypes.c_size_t(0)
    _check(lib().snappy_decompress_buffer_multi(devs, len(devices), p, n, out, N, ctypes.byref(got)),
           "decompress_multi")
    return out.raw[: got.value]


def read_index(data: bytes):
    """Sidecar index file (snappy_amd.h) -> (N, [entries])."""
    import struct
    if len(data) < 24:
        raise SnappyError(ERR_INDEX, "read_index")
    magic, n, count = struct.unpack_from("<QQQ", data, 0)
    # exactly `count` entries, no trailing bytes (the C reader refuses them too)
    if magic != IDX_MAGIC or len(data) != 24 + 8 * count:
        raise SnappyError(ERR_INDEX, "read_index")
    return n, list(struct.unpack_from(f"<{count}Q", data, 24))


def decompress_indexed(data, index_file: bytes) -> bytes:
    """decompress() with a sidecar index instead of the GPU index pass."""
    p, n, keep = _buf(data)
    if n == 0:
        return b""
    _, ent = read_index(index_file)
    arr = (ctypes.c_uint64 * max(len(ent), 1))(*ent)
    N = _declared_length(data, n)
    out = ctypes.create_string_buffer(max(N, 1))
    got = ctypes.c_size_t(0)
    _check(lib().snappy_amd_host_decompress_idx(p, n, arr, len(ent), out, N, ctypes.byref(got)), "decompress_indexed")
    return out.raw[: got.value]


# ---- the reference's FILE*-level calls over Python binary files -------------
def snappy_compress(file_input: BinaryIO, input_size: int, file_compressed: BinaryIO) -> None:
    """snappy_compress (src/snappy_compression.c:414): reads file_input from its
    current position to EOF, writes varint(input_size) ++ blocks; an empty
    read writes nothing."""
    data = file_input.read()
    if not data:
        return
    file_compressed.write(compress(data, header_value=input_size))


def snappy_decompress(file_input: BinaryIO, file_decompressed: BinaryIO) -> int:
    """snappy_decompress (src/snappy_decompression.c:345); returns 0."""
    data = file_input.read()
    file_decompressed.write(decompress(data))
    return 0


# ---- device-resident batch API ------------------------------------------------
class Codec:
    """A device context: kernels run on `device`, on the current torch stream
    of that device when torch tensors are passed (or on the context stream)."""

    def __init__(self, device: int = 0):
        h = ctypes.c_void_p(0)
        _check(lib().snappy_amd_create(device, ctypes.byref(h)), "snappy_amd_create")
        self._h = h
        self.device = device

    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().snappy_amd_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_ptr: int) -> None:
        _check(lib().snappy_amd_set_stream(self._h, ctypes.c_void_p(stream_ptr)), "set_stream")

    def device_bytes(self) -> int:
        """HBM bytes held as scratch by this context (grows to the largest call)."""
        return lib().snappy_amd_device_bytes(self._h)

    def trim(self) -> None:
        """Free the context's scratch (the next call allocates it again)."""
        _check(lib().snappy_amd_trim(self._h), "trim")

    def set_option(self, option: int, value: int) -> None:
        """snappy_amd_set_option: OPT_SERIAL_INDEX (1: one-wave index walk),
        OPT_K1R_EXTRA_LDS (extra dynamic LDS bytes per K1r unit)."""
        _check(lib().snappy_amd_set_option(self._h, option, value), "set_option")

    def enable_timing(self, on: bool = True) -> None:
        _check(lib().snappy_amd_enable_timing(self._h, 1 if on else 0), "enable_timing")

    def last_timings(self) -> Tuple[float, float, float]:
        a, b, c = ctypes.c_float(), ctypes.c_float(), ctypes.c_float()
        _check(lib().snappy_amd_last_timings(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)), "timings")
        return a.value, b.value, c.value

    @staticmethod
    def num_units(n: int, chunk: int, layout: int) -> int:
        return lib().snappy_amd_num_units(n, chunk, layout)

    @staticmethod
    def max_output(n: int, chunk: int, layout: int) -> int:
        return lib().snappy_amd_max_output(n, chunk, layout)

    # raw-pointer forms ---------------------------------------------------
    def compress_ptr(self, d_in: int, n: int, chunk: int, layout: int, d_out: int, d_offsets: int,
                     want_len: bool = True) -> Optional[int]:
        got = ctypes.c_size_t(0)
        rc = lib().snappy_amd_compress_device(self._h, ctypes.c_void_p(d_in), n, chunk, layout,
                                              ctypes.c_void_p(d_out), ctypes.c_void_p(d_offsets),
                                              ctypes.byref(got) if want_len else None)
        _check(rc, "compress_device")
        return got.value if want_len else None

    def decompress_ptr(self, d_comp: int, d_offsets: int, n: int, chunk: int, layout: int, d_out: int,
                       check: bool = True) -> None:
        if check:
            rc = lib().snappy_amd_decompress_device(self._h, ctypes.c_void_p(d_comp), ctypes.c_void_p(d_offsets),
                                                    n, chunk, layout, ctypes.c_void_p(d_out))
        else:
            rc = lib().snappy_amd_decompress_device_async(self._h, ctypes.c_void_p(d_comp),
                                                          ctypes.c_void_p(d_offsets), n, chunk, layout,
                                                          ctypes.c_void_p(d_out))
        _check(rc, "decompress_device")

    def compress_ptr_ex(self, d_in: int, n: int, chunk: int, layout: int, flags: int, header_value: int,
                        d_out: int, d_offsets: int, want_len: bool = True) -> Optional[int]:
        got = ctypes.c_size_t(0)
        rc = lib().snappy_amd_compress_device_ex(self._h, ctypes.c_void_p(d_in), n, chunk, layout, flags,
                                                 header_value, ctypes.c_void_p(d_out), ctypes.c_void_p(d_offsets),
                                                 ctypes.byref(got) if want_len else None)
        _check(rc, "compress_device_ex")
        return got.value if want_len else None

    def decompress_ptr_ex(self, d_comp: int, d_offsets: int, n: int, chunk: int, layout: int, flags: int,
                          header_value: int, d_out: int, check: bool = True) -> None:
        rc = lib().snappy_amd_decompress_device_ex(self._h, ctypes.c_void_p(d_comp), ctypes.c_void_p(d_offsets), n,
                                                   chunk, layout, flags, header_value, ctypes.c_void_p(d_out),
                                                   1 if check else 0)
        _check(rc, "decompress_device_ex")

    def decompress_status(self) -> int:
        return lib().snappy_amd_decompress_status(self._h)

    def index_ptr(self, d_comp: int, clen: int, d_offsets: int, max_units: int) -> int:
        n = ctypes.c_size_t(0)
        _check(lib().snappy_amd_index_device(self._h, ctypes.c_void_p(d_comp), clen, ctypes.c_void_p(d_offsets),
                                             max_units, ctypes.byref(n)), "index_device")
        return n.value

    # torch-tensor forms ----------------------------------------------------
    def _bind_stream(self):
        # torch's default stream is the legacy null stream (cuda_stream 0): set_stream(0)
        # selects the context's own stream, a blocking one, so it is ordered after it too
        self.set_stream(torch.cuda.current_stream(self.device).cuda_stream)

    def compress_tensor(self, x, chunk: int = BLOCK, layout: int = SINGLE):
        """x: contiguous uint8 CUDA tensor -> (payload tensor, offsets tensor)."""
        assert x.is_cuda and x.dtype == torch.uint8 and x.is_contiguous()
        n = x.numel()
        units = self.num_units(n, chunk, layout)
        out = torch.empty(max(self.max_output(n, chunk, layout), 16), dtype=torch.uint8, device=x.device)
        offs = torch.empty(units + 1, dtype=torch.int64, device=x.device)
        self._bind_stream()
        length = self.compress_ptr(x.data_ptr(), n, chunk, layout, out.data_ptr(), offs.data_ptr())
        return out[:length], offs

    def decompress_tensor(self, comp, offsets, n: int, chunk: int = BLOCK, layout: int = SINGLE, out=None):
        assert comp.is_cuda and comp.dtype == torch.uint8
        if out is None:
            out = torch.empty(max(n, 1), dtype=torch.uint8, device=comp.device)
        self._bind_stream()
        self.decompress_ptr(comp.data_ptr(), offsets.data_ptr(), n, chunk, layout, out.data_ptr())
        return out[:n]

    def index_tensor(self, comp):
        """Block index of a SINGLE-layout stream (e.g. a reference .snp)."""
        units_max = (1 << 20)
        offs = torch.empty(units_max + 1, dtype=torch.int64, device=comp.device)
        self._bind_stream()
        n = self.index_ptr(comp.data_ptr(), comp.numel(), offs.data_ptr(), units_max + 1)
        units = (n + BLOCK - 1) // BLOCK
        return n, offs[: units + 1]
