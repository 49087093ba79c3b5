#!/usr/bin/env python3
"""Per-segment cycle shares of the K1r round (SNAPPY_K1R_STAMPS build)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lightweight-snappy_amd"))
os.environ["SNAPPY_AMD_LIB"] = os.path.join(ROOT, "lightweight-snappy_amd", "variants", "libsnappy_amd_" + (sys.argv[3] if len(sys.argv) > 3 else "stamps") + ".so")
import numpy as np, torch
import datagen, snappy_amd
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8 << 20
chunk = int(os.environ.get("K1R_CHUNK", "32768"))  # 65536: one SINGLE stream (K1r64)
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
hip.hipMemcpy(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(ctx.tokens + units * tok_cap * 8), ctypes.c_size_t(buf.nbytes), 2)
st = buf.reshape(units, 4)
loop = st[:, 0].astype(float)
seg0, seg1 = (st[:, 1] & 0xFFFFFFFF).astype(float), (st[:, 1] >> 32).astype(float)
seg2, seg3 = (st[:, 3] & 0xFFFFFFFF).astype(float), (st[:, 3] >> 32).astype(float)
seg4, seg5 = (st[:, 2] & 0xFFFFFFFF).astype(float), (st[:, 2] >> 32).astype(float)
rounds = int(os.environ.get("K1R_ROUNDS", "3937"))
names = sys.argv[2].split(",") if len(sys.argv) > 2 and sys.argv[2] else ["head", "verify_issue", "verify_wait", "tail", "lane-space total", "window refresh"]
tot = loop.sum()
for nm, v in zip(names, [seg0, seg1, seg2, seg3, seg4, seg5]):
    print(f"{nm:24s} {v.sum()/tot*100:5.1f}%  {v.mean()/rounds:7.1f} cycles/round")
print(f"loop cycles/unit {loop.mean():.0f} ({loop.mean()/rounds:.0f}/round)")
