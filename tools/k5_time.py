#!/usr/bin/env python3
"""K5p (block index of a foreign SINGLE stream) timing: compress N bytes of a
workload as one 64 KiB-block stream on the GPU, then time index_tensor on it
(HIP events on the codec's stream) and check the index equals the one the
compressor wrote.  Run under rocprofv3 --kernel-trace --stats for per-kernel
times (k5a_chunk_walk, k5b_carry, k5c_mark, k5d_result)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lightweight-snappy_amd"))
import torch  # noqa: E402

import datagen  # noqa: E402
import snappy_amd  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "T"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 256 << 20
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
x = torch.from_numpy(datagen.make(kind, n, 1234)).cuda()
codec = snappy_amd.Codec(0)
comp, offs = codec.compress_tensor(x, chunk=65536, layout=snappy_amd.SINGLE)
stream = torch.cuda.Stream()
codec.set_stream(stream.cuda_stream)
ms = []
with torch.cuda.stream(stream):
    for r in range(reps + 1):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        got_n, got = codec.index_tensor(comp)
        b.record(stream)
        b.synchronize()
        if r:
            ms.append(a.elapsed_time(b))
ok = got_n == n and torch.equal(got.cpu(), offs.cpu())
back = codec.decompress_tensor(comp, got, got_n, chunk=65536, layout=snappy_amd.SINGLE)
ok = ok and torch.equal(back, x)
codec.close()
print(json.dumps({"kind": kind, "n": n, "clen": int(comp.numel()), "k5_ms": sorted(ms)[len(ms) // 2],
                  "k5_GBps_out": n / (sorted(ms)[len(ms) // 2] * 1e-3) / 1e9, "index_ok": bool(ok)}))
