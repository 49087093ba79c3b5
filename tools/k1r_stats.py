#!/usr/bin/env python3
"""Run the SNAPPY_K1R_STATS variant and summarise per-unit cycles/probe."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lightweight-snappy_amd"))
os.environ["SNAPPY_AMD_LIB"] = os.path.join(ROOT, "lightweight-snappy_amd", "variants", "libsnappy_amd_" + os.environ.get("K1R_VARIANT", "stats") + ".so")
import numpy as np, torch
import datagen, snappy_amd
kind = sys.argv[1] if len(sys.argv) > 1 else "T"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 256 << 20
chunk = int(sys.argv[3]) if len(sys.argv) > 3 else 32768  # 65536: one SINGLE stream (K1r64)
layout = snappy_amd.SINGLE if chunk == 65536 else snappy_amd.STREAMS
a = datagen.make(kind, n, 1234 if kind == "T" else 1)
x = torch.from_numpy(a).cuda()
c = snappy_amd.Codec(0)
if os.environ.get("SNAPPY_K1R_DYNLDS"):  # occupancy experiments: extra dynamic LDS per unit
    c.set_option(snappy_amd.OPT_K1R_EXTRA_LDS, int(os.environ["SNAPPY_K1R_DYNLDS"]))
comp, offs = c.compress_tensor(x, chunk=chunk, layout=layout)
comp, offs = c.compress_tensor(x, chunk=chunk, layout=layout)
torch.cuda.synchronize()
lib = snappy_amd.lib()
# the context's token buffer pointer is private: re-run through a probe kernel is overkill; read via hipMemcpy of ctx->tokens
class Ctx(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("own", ctypes.c_void_p), ("stream", ctypes.c_void_p),
                ("sizes", ctypes.c_void_p), ("sizes_cap", ctypes.c_size_t),
                ("tokens", ctypes.c_void_p), ("tokens_cap", ctypes.c_size_t)]
ctx = ctypes.cast(c._h, ctypes.POINTER(Ctx)).contents
units = n // chunk
tok_cap = chunk // 4 + 2
hip = ctypes.CDLL("libamdhip64.so")
buf = np.empty(units * 4, dtype=np.uint64)
rc = hip.hipMemcpy(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(ctx.tokens + units * tok_cap * 8), ctypes.c_size_t(buf.nbytes), 2)
st = buf.reshape(units, 4)
loop, pr, matches, refresh = st[:, 0], st[:, 2], st[:, 3] & 0xFFFFFFFF, st[:, 3] >> 32
farc, reload = st[:, 1] & 0xFFFFFFFF, st[:, 1] >> 32
tmatch = np.zeros_like(loop)
probes, rounds = pr & 0xFFFFFFFF, pr >> 32
print(f"{kind}: units {units} probes/unit {probes.mean():.0f} rounds/unit {rounds.mean():.0f} matches/unit {matches.mean():.0f} window refreshes/unit {refresh.mean():.0f}")
print(f"loop cycles/unit {loop.mean():.0f} cycles/probe {loop.sum() / probes.sum():.1f} cycles/round {loop.sum()/rounds.sum():.1f}"
      f" match-path cycles/match {tmatch.sum()/max(matches.sum(),1):.1f} non-match cycles/round {(loop.sum()-tmatch.sum())/rounds.sum():.1f}")
print(f"64 KiB blocks: candidate gathers from global memory/unit {farc.mean():.1f}, ring segments loaded synchronously/unit {reload.mean():.1f}")
if chunk <= 32768:
    print(f"W-probe rounds (steps > 1) per unit {farc.mean():.0f} of {rounds.mean():.0f} rounds")
