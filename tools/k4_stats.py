#!/usr/bin/env python3
"""Cycles per element of K4 (SNAPPY_K4_STATS build).
Usage: tools/k4_stats.py KIND BYTES [VARIANT]  (variants/libsnappy_amd_<VARIANT>.so, default k4stats)"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lightweight-snappy_amd"))
os.environ["SNAPPY_AMD_LIB"] = os.path.join(ROOT, "lightweight-snappy_amd", "variants", f"libsnappy_amd_{sys.argv[3] if len(sys.argv) > 3 else 'k4stats'}.so")
import numpy as np, torch
import datagen, snappy_amd
kind = sys.argv[1]; n = int(sys.argv[2]); chunk = 32768
a = datagen.make(kind, n, 1234 if kind == "T" else 1)
x = torch.from_numpy(a).cuda()
c = snappy_amd.Codec(0)
comp, offs = c.compress_tensor(x, chunk=chunk, layout=snappy_amd.STREAMS)
back = c.decompress_tensor(comp, offs, n, chunk=chunk, layout=snappy_amd.STREAMS)
assert torch.equal(back, x)
units = n // chunk
buf = np.zeros(units * 16, dtype=np.uint64)
lib = snappy_amd.lib()
lib.snappy_amd_debug_k4_stats.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert lib.snappy_amd_debug_k4_stats(buf.ctypes.data_as(ctypes.c_void_p), units * 16) == 0
st = buf.reshape(units, 16)
far = (st[:, 1] >> 32).astype(np.float64)
st = st.astype(np.float64)
st[:, 1] = (buf.reshape(units, 16)[:, 1] & 0xFFFFFFFF).astype(np.float64)
m = st.mean(axis=0)
print(f"{kind} units {units}: elements/unit {m[1]:.0f} batches {m[2]:.0f} passes {m[3]:.0f} pass steps {m[4]:.0f} (passes + pointer-jump steps)"
      f" passes reading HBM (copies beyond the ring) {far.mean():.0f}")
print(f"cycles/unit {m[0]:.0f}  cycles/element {m[0]/m[1]:.1f}  cycles/batch {m[0]/m[2]:.0f}")
for i, nm in ((5, "window+candidate parse"), (6, "doubling+gather+scans+validate"), (7, "execute (passes)")):
    print(f"  {nm:32s} {m[i]/m[2]:7.0f} cycles/batch  {100*m[i]/m[0]:5.1f}%")
print(f"  per pass {m[7]/max(m[3],1):.0f} cycles")
b = max(m[2], 1)
print(f"batch shape: halves/batch {m[8]/b:.2f}  parsed elements/batch {m[9]/b:.1f}  executed {m[1]/b:.1f}  "
      f"E == 64 {100*m[13]/b:.1f}%  halves stopped at the window {100*m[15]/b:.1f}%  after a span cut {100*m[14]/b:.1f}%")
print(f"cut before E by: a bad/tail element {100*m[10]/b:.1f}%  a literal leaving the window {100*m[11]/b:.1f}%  "
      f"the output span {100*m[12]/b:.1f}%")
