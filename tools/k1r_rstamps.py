#!/usr/bin/env python3
"""Window-refresh share of K1r / K1r64 with the asm round loop in place
(SNAPPY_K1R_RSTAMPS build): loop cycles per unit, token-flush and window-move
cycles per refresh.  Usage: tools/k1r_rstamps.py BYTES CHUNK [VARIANT]"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lightweight-snappy_amd"))
os.environ["SNAPPY_AMD_LIB"] = os.path.join(ROOT, "lightweight-snappy_amd", "variants",
                                            "libsnappy_amd_" + (sys.argv[3] if len(sys.argv) > 3 else "rst") + ".so")
import numpy as np, torch
import datagen, snappy_amd
n = int(sys.argv[1]) if len(sys.argv) > 1 else 256 << 20
chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
layout = snappy_amd.SINGLE if chunk == 65536 else snappy_amd.STREAMS
a = datagen.make("T", n, 1234)
x = torch.from_numpy(a).cuda()
c = snappy_amd.Codec(0)
comp, offs = c.compress_tensor(x, chunk=chunk, layout=layout)
torch.cuda.synchronize()
class Ctx(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("own", ctypes.c_void_p), ("stream", ctypes.c_void_p),
                ("sizes", ctypes.c_void_p), ("sizes_cap", ctypes.c_size_t),
                ("tokens", ctypes.c_void_p), ("tokens_cap", ctypes.c_size_t)]
ctx = ctypes.cast(c._h, ctypes.POINTER(Ctx)).contents
units = n // chunk
tok_cap = chunk // 4 + 2
hip = ctypes.CDLL("libamdhip64.so")
buf = np.empty(units * 4, dtype=np.uint64)
hip.hipMemcpy(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(ctx.tokens + units * tok_cap * 8),
              ctypes.c_size_t(buf.nbytes), 2)
raw = buf.reshape(units, 4)
f = lambda v: v.astype(np.float64).mean()
loop = f(raw[:, 0])
fl, asm = f(raw[:, 1] & ((1 << 24) - 1)), f(raw[:, 1] >> 24)
win, nasm = f(raw[:, 2] & ((1 << 40) - 1)), f(raw[:, 2] >> 40)
nref, nfl = f(raw[:, 3] & 0xFFFF), f((raw[:, 3] >> 16) & 0xFFFF)
c3, c45 = f((raw[:, 3] >> 32) & 0xFFFF), f(raw[:, 3] >> 48)
print(f"chunk {chunk}: loop {loop:.0f} cycles/unit; refreshes {nref:.0f}/unit ({nfl:.0f} with a token flush)")
print(f"  asm round loop {asm/loop*100:5.1f}%  {nasm:.0f} entries/unit, {asm/max(nasm,1):.0f} cycles/entry; exits to the C++ round: code 3 {c3:.0f}, codes 4-5 {c45:.0f}")
print(f"  window move    {win/loop*100:5.1f}%  {win/max(nref,1):6.0f} cycles/refresh (s_memtime clock)")
print(f"  token flush    {fl/loop*100:5.1f}%  {fl/max(nfl,1):6.0f} cycles/flush")
print(f"  rest (C++ rounds, W-probe rounds, stamps) {(loop-asm-win-fl)/loop*100:5.1f}%")
