#!/usr/bin/env python3
"""One compress + decompress of N bytes of a workload (for rocprofv3 counter passes)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lightweight-snappy_amd"))
import torch, datagen, snappy_amd
kind = sys.argv[1] if len(sys.argv) > 1 else "T"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 256 << 20
chunk = int(sys.argv[3]) if len(sys.argv) > 3 else 32768
layout = snappy_amd.STREAMS if chunk <= 32768 else snappy_amd.SINGLE
x = torch.from_numpy(datagen.make(kind, n, 1234 if kind == "T" else 1)).cuda()
c = snappy_amd.Codec(0)
comp, offs = c.compress_tensor(x, chunk=chunk, layout=layout)
back = c.decompress_tensor(comp, offs, n, chunk=chunk, layout=layout)
assert torch.equal(back, x)
print("ok", comp.numel())
