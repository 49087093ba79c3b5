#!/usr/bin/env python3
"""A/B the kernel variants built by tools/variants.sh in ONE process each,
interleaved rounds: K1/K3/K4 HIP-event times on the same seeded workload,
output bytes checked identical across variants (sha256)."""
import argparse
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import os, sys, json, hashlib
sys.path.insert(0, os.path.join(ROOT, "lightweight-snappy_amd"))
import numpy as np, torch
import datagen, snappy_amd
kind, n, chunk, layout, reps = KIND, N, CHUNK, LAYOUT, REPS
a = datagen.make(kind, n, 1234 if kind == "T" else (1 if kind == "R" else 2))
x = torch.from_numpy(a).cuda()
c = snappy_amd.Codec(0); c.enable_timing(True)
c.set_stream(torch.cuda.current_stream().cuda_stream)
units = c.num_units(n, chunk, layout)
out = torch.empty(c.max_output(n, chunk, layout), dtype=torch.uint8, device="cuda")
offs = torch.empty(units + 1, dtype=torch.int64, device="cuda")
back = torch.empty(n, dtype=torch.uint8, device="cuda")
k1 = []; k3 = []; k4 = []
for r in range(reps + 1):
    L = c.compress_ptr(x.data_ptr(), n, chunk, layout, out.data_ptr(), offs.data_ptr())
    c.decompress_ptr(out.data_ptr(), offs.data_ptr(), n, chunk, layout, back.data_ptr())
    t = c.last_timings()
    if r: k1.append(t[0]); k3.append(t[1]); k4.append(t[2])
ok = bool(torch.equal(back, x))
h = hashlib.sha256(out[:L].cpu().numpy().tobytes()).hexdigest()
print(json.dumps({"k1": sorted(k1)[len(k1)//2], "k1min": min(k1), "k3": min(k3), "k4": sorted(k4)[len(k4)//2], "k4min": min(k4), "len": L, "sha": h[:16], "rt": ok}))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--kind", default="T")
    ap.add_argument("--n", type=int, default=256 << 20)
    ap.add_argument("--chunk", type=int, default=32768)
    ap.add_argument("--layout", type=int, default=1)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    code = CHILD.replace("ROOT", repr(ROOT)).replace("KIND", repr(args.kind)).replace("REPS", str(args.reps))
    code = code.replace("CHUNK", str(args.chunk)).replace("LAYOUT", str(args.layout)).replace(", N,", f", {args.n},")
    res = {}
    for rnd in range(args.rounds):
        for v in args.variants:
            name, _, envs = v.partition("+")
            lib = os.path.join(ROOT, "lightweight-snappy_amd", "variants", f"libsnappy_amd_{name}.so") if name != "default" else ""
            env = dict(os.environ, SNAPPY_AMD_LIB=lib)
            for kv in filter(None, envs.split(",")):
                k, _, val = kv.partition("=")
                env[k] = val or "1"
            r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=600)
            if r.returncode != 0:
                print(v, "FAILED", r.stderr[-2000:], flush=True)
                sys.exit(1)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            res.setdefault(v, []).append(d)
            gbs = args.n / (d["k1"] * 1e-3) / 1e9
            print(f"round {rnd} {v:10s} k1 {d['k1']:8.3f} ms ({gbs:6.2f} GB/s in) k3 {d['k3']:.3f} k4 {d['k4']:8.3f} ms "
                  f"({args.n / (d['k4'] * 1e-3) / 1e9:6.2f} GB/s) len {d['len']} sha {d['sha']} rt {d['rt']}", flush=True)
    shas = {d["sha"] for v in res for d in res[v]}
    print("ALL OUTPUTS IDENTICAL" if len(shas) == 1 else f"OUTPUTS DIFFER: {shas}")


if __name__ == "__main__":
    main()
