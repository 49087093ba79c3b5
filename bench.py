#!/usr/bin/env python3
"""bench.py -- MI355X Snappy codec benchmark (BASELINE.json metric).

One step = one compress (K1 block compress + K3 scan/gather) and one
decompress (K4) of the per-GPU batch, inputs already resident in HBM.
Default workload = BASELINE.json configs[1]: 1 GiB of synthetic enwik8-like
text as 32,768 independent 32 KiB streams (each == the reference's
snappy_compress() of its chunk), per GPU (weak scaling: every rank gets its
own 1 GiB shard of the generator; the only exchange is the 8-byte size
all-gather that places each shard in the global stream).  --assemble adds
the RCCL all-gather of the compressed shards (timed separately).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--workload text32k|text64k|random|repeat]
Multi-GPU: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "lightweight-snappy_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import datagen  # noqa: E402
import snappy_amd  # noqa: E402

METRIC = "compress + decompress MB/s at 1/2/4/8 MI355X; % HBM roofline; ratio vs ref"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

WORKLOADS = {
    # name: (generator kind, seed, layout, chunk, description)
    "text32k": ("T", 1234, snappy_amd.STREAMS, 32768,
                "1 GiB/GPU synthetic enwik8-like text as 32,768 independent 32 KiB snappy_compress() streams"),
    "text64k": ("T", 1234, snappy_amd.SINGLE, 65536,
                "1 GiB/GPU synthetic text as one snappy_compress() stream of 65,536-byte blocks"),
    "random": ("R", 1, snappy_amd.SINGLE, 65536, "1 GiB/GPU random bytes (all-literal), one stream"),
    "repeat": ("P", 2, snappy_amd.SINGLE, 65536, "1 GiB/GPU 64-byte-period repeat (all-copy), one stream"),
    # BASELINE configs[4]: decode only, a ~10 GB pre-compressed stream (compressed once, untimed)
    "decode10g": ("T", 1234, snappy_amd.SINGLE, 65536,
                  "decode-only: 1 GiB/GPU of text pre-compressed (untimed) into one stream of 65,536-byte blocks"),
}
DECODE_ONLY = {"decode10g"}
DECODE10G_BYTES = (18_500_000_000 // 65536) * 65536  # ratio ~1.85 -> ~10 GB of compressed stream


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="text32k", choices=sorted(WORKLOADS))
    ap.add_argument("--bytes-per-gpu", type=int, default=1 << 30)
    ap.add_argument("--assemble", action="store_true", help="also time the RCCL all-gather of shards")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-e2e", action="store_true", help="skip the PCIe-inclusive host API sample")
    ap.add_argument("--keep-size", action="store_true", help="decode10g: use --bytes-per-gpu as given")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="nccl (= RCCL, the real path) or gloo (CPU collectives; rehearsal with ranks sharing a GPU)")
    ap.add_argument("--cpu-sample-bytes", type=int, default=1 << 30)
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_latest.json"),
                    help="rocprofv3 PMC summary giving HBM traffic per launch (see profiles/README.md)")
    return ap.parse_args()


def cpu_baseline(kind: str, seed: int, chunk: int, layout: int, sample: int, decode_only: bool = False):
    """The oracle (CPU restatement, fixture-verified bit-exact with the
    reference) timed on this host, 1 thread like the reference, wall clock."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg only

    a = datagen.make(kind, sample, seed)
    t0 = time.perf_counter()
    if layout == snappy_amd.STREAMS:
        payload, offs = oracle.compress_streams(a, chunk, threads=1)
    else:
        payload = np.frombuffer(oracle.compress(a), dtype=np.uint8)
    t1 = time.perf_counter()
    if layout == snappy_amd.STREAMS:
        back = oracle.decompress_streams(payload, offs, a.size, chunk, threads=1)
    else:
        back = np.frombuffer(oracle.decompress(payload.tobytes()), dtype=np.uint8)
    t2 = time.perf_counter()
    assert np.array_equal(back, a)
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    base = {"value": round(a.size / ((t2 - t1) if decode_only else (t2 - t0)) / 1e6, 2), "unit": "MB/s",
            "cores": 1, "kind": "port",
            "sample": f"{a.size / 2**20:.0f} MiB of the same workload, compress {a.size / (t1 - t0) / 1e6:.1f} MB/s"
                      f" + decompress {a.size / (t2 - t1) / 1e6:.1f} MB/s, oracle/snappy_oracle.c -O2, 1 thread,"
                      f" {cpu_model}"}
    # all host cores of this box's share over independent units
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "16")), os.cpu_count() or 1))
    t0 = time.perf_counter()
    if layout == snappy_amd.STREAMS:
        payload, offs = oracle.compress_streams(a, chunk, threads=threads)
        t1 = time.perf_counter()
        back = oracle.decompress_streams(payload, offs, a.size, chunk, threads=threads)
    else:  # independent 64 KiB blocks: the all-core upper bound of the reference algorithm
        payload, offs = oracle.compress_streams(a, 65536, threads=threads)
        t1 = time.perf_counter()
        back = oracle.decompress_streams(payload, offs, a.size, 65536, threads=threads)
    t2 = time.perf_counter()
    assert np.array_equal(back, a)
    allc = {"value": round(a.size / ((t2 - t1) if decode_only else (t2 - t0)) / 1e6, 2), "unit": "MB/s",
            "cores": threads, "kind": "port",
            "compress_MBps": round(a.size / (t1 - t0) / 1e6, 1),
            "decompress_MBps": round(a.size / (t2 - t1) / 1e6, 1)}
    return base, allc


def cpu_reference(kind: str, seed: int, chunk: int, layout: int, sample: int, decode_only: bool = False):
    """The compiled reference itself (oracle/_ref/libsnappy_ref.so, built from
    /root/reference/src by oracle/Makefile; its FILE* API through tmpfiles, as
    cmd.c drives it), 1 thread, on a sample of the same workload.  None when the
    library is absent."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg only

    if not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "libsnappy_ref.so")):
        return None
    a = datagen.make(kind, sample, seed)
    step = chunk if layout == snappy_amd.STREAMS else a.size
    t0 = time.perf_counter()
    comp = [oracle.ref_compress(a[i:i + step]) for i in range(0, a.size, step)]
    t1 = time.perf_counter()
    back = [oracle.ref_decompress(c, min(step, a.size - i * step)) for i, c in enumerate(comp)]
    t2 = time.perf_counter()
    assert b"".join(back) == a.tobytes()
    return {"value": round(a.size / ((t2 - t1) if decode_only else (t2 - t0)) / 1e6, 2), "unit": "MB/s",
            "cores": 1, "kind": "reference",
            "sample": f"{a.size / 2**20:.0f} MiB, compress {a.size / (t1 - t0) / 1e6:.1f} MB/s + decompress "
                      f"{a.size / (t2 - t1) / 1e6:.1f} MB/s, reference src/*.c -O2 through its FILE* API (tmpfiles)"}


def host_end_to_end(kind: str, seed: int, sample: int) -> dict:
    """PCIe-inclusive rate of the drop-in host API (snappy_compress_buffer /
    snappy_decompress_buffer: one SINGLE stream of 64 KiB blocks, pageable
    host buffers in and out).  Reported beside `value`, never as it."""
    import ctypes
    lib = snappy_amd.lib()
    a = datagen.make(kind, sample, seed)
    cap = snappy_amd.max_compressed_length(a.size)
    comp = np.empty(cap, dtype=np.uint8)
    back = np.empty(a.size, dtype=np.uint8)
    got = ctypes.c_size_t(0)
    vp = ctypes.c_void_p
    best_c = best_d = float("inf")
    for _ in range(3):
        t0 = time.perf_counter()
        rc = lib.snappy_compress_buffer(vp(a.ctypes.data), a.size, vp(comp.ctypes.data), ctypes.byref(got))
        t1 = time.perf_counter()
        assert rc == 0, rc
        clen = got.value
        rc = lib.snappy_decompress_buffer(vp(comp.ctypes.data), clen, vp(back.ctypes.data), a.size,
                                          ctypes.byref(got))
        t2 = time.perf_counter()
        assert rc == 0 and got.value == a.size, rc
        best_c, best_d = min(best_c, t1 - t0), min(best_d, t2 - t1)
    assert np.array_equal(back, a)
    return {"bytes": int(a.size), "layout": "SINGLE 64 KiB blocks", "compress_MBps": round(a.size / best_c / 1e6, 1),
            "decompress_MBps": round(a.size / best_d / 1e6, 1), "note": "pageable host buffers, H2D+D2H included"}


def hbm_copy_gbps(dev, nbytes: int = 1 << 30) -> float:
    """Device-to-device copy (read + write bytes) as the box's HBM check."""
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize(dev)
    best = float("inf")
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        b.copy_(a)
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e-3)
    del a, b
    return round(2 * nbytes / best / 1e9, 1)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gloo = args.dist_backend == "gloo"
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # gloo: rehearsal of the multi-rank path (ranks may share a GPU)
        local = local % torch.cuda.device_count() if gloo else local
        torch.cuda.set_device(local)
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)
    cdev = torch.device("cpu") if gloo else dev  # where collective tensors live

    kind, seed, layout, chunk, desc = WORKLOADS[args.workload]
    decode_only = args.workload in DECODE_ONLY
    n = args.bytes_per_gpu
    if decode_only and n == 1 << 30 and not args.keep_size:
        n = DECODE10G_BYTES
    host = np.empty(n, dtype=np.uint8)
    datagen.fill(host, kind, seed, offset=rank * n, threads=16)
    x = torch.from_numpy(host).to(dev)
    codec = snappy_amd.Codec(dev.index)
    codec.enable_timing(True)
    stream = torch.cuda.current_stream(dev)
    codec.set_stream(stream.cuda_stream)
    units = codec.num_units(n, chunk, layout)
    out = torch.empty(codec.max_output(n, chunk, layout), dtype=torch.uint8, device=dev)
    offs = torch.empty(units + 1, dtype=torch.int64, device=dev)
    back = torch.empty(n, dtype=torch.uint8, device=dev)
    # SINGLE layout sharded over ranks: rank 0 carries the global preamble
    flags = snappy_amd.NO_PREAMBLE if (layout == snappy_amd.SINGLE and rank > 0) else 0
    header_value = n * world if layout == snappy_amd.SINGLE else n
    sizes_t = torch.zeros(world, dtype=torch.int64, device=cdev)

    def allgather(dst, src):
        if gloo:
            parts = list(dst.chunk(world))
            dist.all_gather(parts, src)
            if parts[0].data_ptr() != dst.data_ptr():
                dst.copy_(torch.cat(parts))
        else:
            dist.all_gather_into_tensor(dst, src)

    pre_clen = None
    if decode_only:  # the stream exists before the timed region
        pre_clen = codec.compress_ptr_ex(x.data_ptr(), n, chunk, layout, flags, header_value, out.data_ptr(),
                                         offs.data_ptr())

    def step():
        if decode_only:
            codec.decompress_ptr_ex(out.data_ptr(), offs.data_ptr(), n, chunk, layout, flags, header_value,
                                    back.data_ptr(), check=False)
            return pre_clen
        clen = codec.compress_ptr_ex(x.data_ptr(), n, chunk, layout, flags, header_value, out.data_ptr(),
                                     offs.data_ptr())
        if world > 1:  # C1: shard sizes -> global stream offsets
            mine = torch.tensor([clen], dtype=torch.int64, device=cdev)
            allgather(sizes_t, mine)
        codec.decompress_ptr_ex(out.data_ptr(), offs.data_ptr(), n, chunk, layout, flags, header_value,
                                back.data_ptr(), check=False)
        return clen

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    k1, k3, k4 = [], [], []
    t0 = time.perf_counter()
    clen = 0
    for _ in range(args.steps):
        clen = step()
        a, b, c = codec.last_timings()
        k1.append(a), k3.append(b), k4.append(c)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    st = codec.decompress_status()
    ok = st == 0 and bool(torch.equal(back, x))
    if world > 1:
        t = torch.tensor([elapsed, 0.0 if ok else 1.0], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, bad = float(t[0]), float(t[1])
        ok = bad == 0.0
        tot = torch.tensor([clen], dtype=torch.int64, device=cdev)
        dist.all_reduce(tot)
        total_comp = int(tot)
    else:
        total_comp = clen

    assemble = None
    if args.assemble and world > 1:  # C2: every rank receives the whole stream
        torch.cuda.synchronize(dev)
        dist.barrier()
        ta = time.perf_counter()
        mx = int(sizes_t.max())
        pad = torch.zeros(mx, dtype=torch.uint8, device=cdev)
        pad[:clen] = out[:clen].to(cdev)
        full = torch.empty(world * mx, dtype=torch.uint8, device=cdev)
        allgather(full, pad)
        torch.cuda.synchronize(dev)
        dist.barrier()
        tb = time.perf_counter() - ta
        assemble = {"allgather_ms": round(tb * 1e3, 3), "bytes": int(world * mx),
                    "GBps_per_rank_in": round((world - 1) * mx / tb / 1e9, 2)}

    hbm_gbps = hbm_copy_gbps(dev) if rank == 0 else None
    total_in = n * world
    ms_step = elapsed / args.steps * 1e3
    value = total_in / (elapsed / args.steps) / 1e6
    k1m, k3m, k4m = (float(np.mean(v)) for v in (k1, k3, k4))
    comp_bytes = clen  # this rank's compressed output
    # dominant kernel (longest average launch) and its algorithmic bytes per
    # launch: compress = N_in + N_out, decompress = N_comp + N_out
    k1_name = "k1r_match_units" if chunk <= 32768 else "k1r_match_units64"
    if os.environ.get("SNAPPY_AMD_FORCE_LDS_K1"):
        k1_name = "k1_compress_units"
    cands = [(k1m, k1_name, n + comp_bytes), (k4m, "k4_decompress_units", comp_bytes + n)]
    if decode_only:
        cands = cands[1:]
    dom_ms, dom_name, dom_bytes = max(cands)
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    traffic = None
    try:
        pm = json.load(open(args.pmc))
        if pm.get("workload") == args.workload and pm.get("bytes_per_gpu") == n:
            traffic = pm["kernels"].get(dom_name, {}).get("hbm_bytes")
    except (OSError, ValueError, KeyError):
        pass

    if rank == 0:
        cpu = cpu_all = cpu_ref = e2e = None
        if world == 1 and not args.no_cpu_baseline:
            cpu, cpu_all = cpu_baseline(kind, seed, chunk, layout, min(args.cpu_sample_bytes, n), decode_only)
            cpu_ref = cpu_reference(kind, seed, chunk, layout, min(128 << 20, n), decode_only)
        if world == 1 and not args.no_host_e2e and not decode_only:
            e2e = host_end_to_end(kind, seed, min(n, 256 << 20))
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "MB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": f"{args.workload}: {desc.replace('1 GiB/GPU', f'{n / 2**30:.4g} GiB/GPU')}; one step = "
                                   + ("one decode of the stream" if decode_only else "compress + decompress round trip"),
                       "bytes_per_gpu": n, "chunk": chunk, "layout": "STREAMS" if layout else "SINGLE",
                       "units_per_gpu": units, "parallelism": f"dp{world} (block shards)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "kernel": dom_name, "kernel_ms": round(dom_ms, 3),
                         "algorithmic_bytes_per_launch": dom_bytes},
            "cpu_baseline": cpu,
            "cpu_baseline_all_cores": cpu_all,
            "cpu_reference": cpu_ref,
            "ratio": round(total_in / total_comp, 4),
            "compress_MBps": None if decode_only else round(n / ((k1m + k3m) * 1e-3) / 1e6, 1),
            "decompress_MBps": round(n / (k4m * 1e-3) / 1e6, 1),
            # src/result.c:40 defines decompress speed over the compressed bytes
            "decompress_MBps_ref_definition": round(comp_bytes / (k4m * 1e-3) / 1e6, 1),
            "hbm_copy_GBps_measured": hbm_gbps,
            "host_end_to_end": e2e,
            "kernel_ms": {"k1_match": round(k1m, 3), "k3_scan_k2_emit": round(k3m, 3),
                          "k4_decode": round(k4m, 3)},
            "hbm_frac": {"compress_k1": round((n + comp_bytes) / (k1m * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                         "decompress_k4": round((n + comp_bytes) / (k4m * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)},
            "round_trip_ok": ok,
        }
        if assemble:
            line["assemble"] = assemble
        print(json.dumps(line), flush=True)
    codec.close()
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
