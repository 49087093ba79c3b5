#!/usr/bin/env python3
"""Does splitting a 1 GiB round trip into two halves on two streams (the first
at high priority) fill K1r's last, partly empty round of units?  Times the
whole compress + decompress of one GiB both ways; outputs checked equal."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lightweight-snappy_amd"))
import datagen  # noqa: E402
import snappy_amd as sa  # noqa: E402

kind, chunk, layout = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
n = 1 << 30
x = torch.from_numpy(datagen.make(kind, n, 1234)).cuda()
unit = chunk if layout == sa.STREAMS else 65536
half = (n // 2 // unit) * unit
parts = [(0, half), (half, n - half)]
ca, cb = sa.Codec(0), sa.Codec(0)
sA, sB = torch.cuda.Stream(priority=-1), torch.cuda.Stream(priority=0)
ca.set_stream(sA.cuda_stream)
cb.set_stream(sB.cuda_stream)
cap = [sa.Codec.max_output(m, chunk, layout) for _, m in parts]
out = torch.empty(sum(cap), dtype=torch.uint8, device="cuda")
offs = [torch.empty(sa.Codec.num_units(m, chunk, layout) + 1, dtype=torch.int64, device="cuda") for _, m in parts]
back = torch.empty(n, dtype=torch.uint8, device="cuda")
one_out = torch.empty(sa.Codec.max_output(n, chunk, layout), dtype=torch.uint8, device="cuda")
one_offs = torch.empty(sa.Codec.num_units(n, chunk, layout) + 1, dtype=torch.int64, device="cuda")
torch.cuda.synchronize()


def one():
    ca.compress_ptr(x.data_ptr(), n, chunk, layout, one_out.data_ptr(), one_offs.data_ptr(), want_len=False)
    ca.decompress_ptr(one_out.data_ptr(), one_offs.data_ptr(), n, chunk, layout, back.data_ptr(), check=False)


def halves(two_streams=True):
    pos = 0
    for i, ((o, m), c) in enumerate(zip(parts, (ca, cb if two_streams else ca))):
        flags = sa.NO_PREAMBLE if (layout == sa.SINGLE and o) else 0
        c.compress_ptr_ex(x.data_ptr() + o, m, chunk, layout, flags, n, out.data_ptr() + pos, offs[i].data_ptr(),
                          want_len=False)
        pos += cap[i]
    pos = 0
    for i, ((o, m), c) in enumerate(zip(parts, (ca, cb if two_streams else ca))):
        flags = sa.NO_PREAMBLE if (layout == sa.SINGLE and o) else 0
        c.decompress_ptr_ex(out.data_ptr() + pos, offs[i].data_ptr(), m, chunk, layout, flags, n,
                            back.data_ptr() + o, check=False)
        pos += cap[i]


for name, fn in (("one piece", one), ("halves, one stream", lambda: halves(False)), ("halves, two streams", halves)):
    for rep in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / 5
        ok = bool(torch.equal(back, x))
        back.zero_()
        print(f"{kind} {chunk} {name:20s} rep {rep}: {dt * 1e3:7.3f} ms per GiB round trip ({n / dt / 1e9:5.1f} GB/s) ok {ok}",
              flush=True)
