#!/usr/bin/env python3
"""bench.py -- MI355X Snappy codec benchmark (BASELINE.json metric).

One step = one compress (K1r match finder + K3 scan + K2 emit) and one
decompress (K4) of the rank's batch, inputs already resident in HBM.
Default workload = BASELINE.json configs[1]: 1 GiB of synthetic enwik8-like
text as 32,768 independent 32 KiB streams (each == the reference's
snappy_compress() of its chunk), per GPU (weak scaling: every rank gets its
own 1 GiB shard of the generator).  --total-bytes T instead fixes the job
size (strong scaling, configs[3]: 64 GiB over 1/2/4/8 GPUs): rank r owns
the unit-aligned range dist.shard_range(T, N, r) of the generator.

Exchange steps: C1, the all-gather of the shard sizes, is part
of every step; with N > 1 the run then times, outside the steps, C2 (the
RCCL all-gather that reassembles the compressed stream on every rank) and
C3 (the all-gather of the decoded shards), each verified by checksums.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
                       [--workload text32k|text64k|random|repeat|decode10g] [--total-bytes T]
--gpus N without a torch.distributed launcher spawns the N ranks itself
(python -m torch.distributed.run, 127.0.0.1); this parent process never
touches the GPU.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "lightweight-snappy_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import datagen  # noqa: E402
import snappy_amd  # noqa: E402
from dist import shard_range  # noqa: E402

METRIC = "compress + decompress MB/s at 1/2/4/8 MI355X; % HBM roofline; ratio vs ref"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

WORKLOADS = {
    # name: (generator kind, seed, layout, chunk, description)
    "text32k": ("T", 1234, snappy_amd.STREAMS, 32768,
                "synthetic enwik8-like text as independent 32 KiB snappy_compress() streams"),
    "text64k": ("T", 1234, snappy_amd.SINGLE, 65536,
                "synthetic text as one snappy_compress() stream of 65,536-byte blocks"),
    "random": ("R", 1, snappy_amd.SINGLE, 65536, "random bytes (all-literal), one stream"),
    "repeat": ("P", 2, snappy_amd.SINGLE, 65536, "64-byte-period repeat (all-copy), one stream"),
    # BASELINE configs[4]: decode only, a ~10 GB pre-compressed stream (compressed once, untimed)
    "decode10g": ("T", 1234, snappy_amd.SINGLE, 65536,
                  "decode-only: synthetic text pre-compressed (untimed) into one stream of 65,536-byte blocks"),
}
DECODE_ONLY = {"decode10g"}
DECODE10G_BYTES = (18_500_000_000 // 65536) * 65536  # ratio ~1.85 -> ~10 GB of compressed stream
GiB = 1 << 30


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="text32k", choices=sorted(WORKLOADS))
    ap.add_argument("--bytes-per-gpu", type=int, default=GiB, help="weak scaling: input bytes per rank")
    ap.add_argument("--total-bytes", type=int, default=0,
                    help="strong scaling: fixed job size sharded over the ranks (e.g. 68719476736 = configs[3])")
    ap.add_argument("--piece-bytes", type=int, default=16 * GiB,
                    help="a rank compresses its range in pieces of at most this many bytes (bounds token scratch)")
    ap.add_argument("--no-assemble", action="store_true", help="N > 1: skip the timed C2/C3 all-gathers")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-e2e", action="store_true", help="skip the PCIe-inclusive host API sample")
    ap.add_argument("--keep-size", action="store_true", help="decode10g: use --bytes-per-gpu as given")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="nccl (= RCCL, the real path) or gloo (CPU collectives; rehearsal with ranks sharing a GPU)")
    ap.add_argument("--cpu-sample-bytes", type=int, default=GiB)
    ap.add_argument("--pmc", default=None,
                    help="rocprofv3 PMC summary giving HBM traffic per launch (default profiles/pmc_<workload>.json, "
                         "written by tools/pmc_summary.py)")
    a = ap.parse_args()
    if a.pmc is None:
        a.pmc = os.path.join(ROOT, "profiles", f"pmc_{a.workload}.json")
    return a


def spawn_ranks(n: int) -> int:
    """--gpus N outside a launcher: run N ranks under torch.distributed.run
    (a child process; nothing here has touched the GPU)."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, env=env).returncode


def cpu_share() -> tuple:
    """(threads to use, note): the GPU box's CPU share for one GPU is what its
    environment sets OMP_NUM_THREADS to (16); the affinity mask and
    os.cpu_count() show the whole machine, which other jobs share."""
    try:
        visible = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        visible = os.cpu_count() or 1
    lease = os.environ.get("OMP_NUM_THREADS")
    if lease and lease.isdigit() and 0 < int(lease) <= visible:
        return int(lease), (f"{lease} threads = this GPU's CPU share on the box (OMP_NUM_THREADS); "
                            f"the machine shows {visible} CPUs, shared with the other GPUs' jobs")
    return visible, f"every CPU in this process's affinity mask ({visible})"


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def cpu_baseline(kind: str, seed: int, chunk: int, layout: int, sample: int, decode_only: bool = False):
    """The oracle (CPU restatement, fixture-verified bit-exact with the
    reference) timed on this host, 1 thread like the reference, wall clock;
    then over every core of this process's CPU share."""
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
    base = {"value": round(a.size / ((t2 - t1) if decode_only else (t2 - t0)) / 1e6, 2), "unit": "MB/s",
            "cores": 1, "kind": "port",
            "sample": f"{a.size / 2**20:.0f} MiB of the same workload, compress {a.size / (t1 - t0) / 1e6:.1f} MB/s"
                      f" + decompress {a.size / (t2 - t1) / 1e6:.1f} MB/s, oracle/snappy_oracle.c -O2, 1 thread,"
                      f" {cpu_model()}"}
    # every host core this process may use, over independent units
    threads, note = cpu_share()
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
            "cores_note": note,
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


def hbm_copy_gbps(dev, nbytes: int = GiB) -> float:
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


def checksum(t: torch.Tensor) -> int:
    """Position-sensitive checksum of a uint8 device tensor (C2/C3 verification)."""
    n = t.numel()
    k = 8192
    w = torch.arange(1, k + 1, device=t.device, dtype=torch.int64)
    m = n - n % k
    body = t[:m].view(-1, k).to(torch.int64)
    rows = (body * w).sum(dim=1)
    s = int((rows * torch.arange(1, rows.numel() + 1, device=t.device, dtype=torch.int64)).sum()) if m else 0
    tail = t[m:].to(torch.int64)
    s += int((tail * w[: tail.numel()]).sum()) * 7919 + n
    return s & ((1 << 62) - 1)


class Piece:
    """A unit-aligned part of the rank's range, compressed into its own slice
    of the rank's contiguous payload (pieces after the stream's first carry no
    varint preamble in the SINGLE layout)."""

    def __init__(self, off: int, n: int, flags: int):
        self.off, self.n, self.flags = off, n, flags
        self.clen = 0
        self.out_off = 0
        self.offs = None


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
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
    unit = chunk if layout == snappy_amd.STREAMS else 65536
    strong = args.total_bytes > 0
    if strong:
        total_in = args.total_bytes
        r_off, n = shard_range(total_in, world, rank, unit)
    else:
        n = args.bytes_per_gpu
        if decode_only and n == GiB and not args.keep_size:
            n = DECODE10G_BYTES
        total_in = n * world
        r_off = rank * n
    # the rank's range in HBM, generated on the host 1 GiB at a time
    x = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    host = np.empty(min(max(n, 1), GiB), dtype=np.uint8)
    for o in range(0, n, GiB):
        m = min(GiB, n - o)
        datagen.fill(host[:m], kind, seed, offset=r_off + o, threads=16)
        x[o:o + m].copy_(torch.from_numpy(host[:m]))
    del host
    codec = snappy_amd.Codec(dev.index)
    codec.enable_timing(True)
    stream = torch.cuda.current_stream(dev)
    codec.set_stream(stream.cuda_stream)
    units = codec.num_units(n, chunk, layout)
    # pieces (unit-aligned) bound the K1r token scratch of one call
    step_bytes = max(unit, (args.piece_bytes // unit) * unit)
    pieces = []
    for o in range(0, n, step_bytes):
        flags = snappy_amd.NO_PREAMBLE if (layout == snappy_amd.SINGLE and (r_off + o) > 0) else 0
        pieces.append(Piece(o, min(step_bytes, n - o), flags))
    out = torch.empty(max(sum(codec.max_output(p.n, chunk, layout) for p in pieces), 16), dtype=torch.uint8,
                      device=dev)
    for p in pieces:
        p.offs = torch.empty(codec.num_units(p.n, chunk, layout) + 1, dtype=torch.int64, device=dev)
    back = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    # SINGLE layout: the stream's first piece carries the global preamble
    header_value = total_in if layout == snappy_amd.SINGLE else n
    sizes_t = torch.zeros(world, dtype=torch.int64, device=cdev)

    def allgather(dst, src):
        if gloo:
            parts = list(dst.chunk(world))
            dist.all_gather(parts, src)
            if parts[0].data_ptr() != dst.data_ptr():
                dst.copy_(torch.cat(parts))
        else:
            dist.all_gather_into_tensor(dst, src)

    def compress_all():
        o = 0
        for p in pieces:
            p.out_off = o
            p.clen = codec.compress_ptr_ex(x.data_ptr() + p.off, p.n, chunk, layout, p.flags, header_value,
                                           out.data_ptr() + o, p.offs.data_ptr())
            o += p.clen
        return o

    def decompress_all():
        for p in pieces:
            codec.decompress_ptr_ex(out.data_ptr() + p.out_off, p.offs.data_ptr(), p.n, chunk, layout, p.flags,
                                    header_value, back.data_ptr() + p.off, check=False)

    pre_clen = None
    g_offs = None
    g_flags = pieces[0].flags
    if decode_only:  # the stream and its block index exist before the timed region
        pre_clen = compress_all()
        # one index over the whole rank stream (the pieces' indexes shifted to their payload offsets)
        g_offs = torch.cat([p.offs[:-1] + p.out_off for p in pieces] +
                           [torch.tensor([pre_clen], dtype=torch.int64, device=dev)])

    def step():
        if decode_only:
            codec.decompress_ptr_ex(out.data_ptr(), g_offs.data_ptr(), n, chunk, layout, g_flags, header_value,
                                    back.data_ptr(), check=False)
            return pre_clen
        clen = compress_all()
        if world > 1:  # C1: shard sizes -> global stream offsets
            mine = torch.tensor([clen], dtype=torch.int64, device=cdev)
            allgather(sizes_t, mine)
        decompress_all()
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
    ok = st == 0 and bool(torch.equal(back[:n], x[:n]))
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
    if world > 1 and not args.no_assemble:
        assemble = exchange(out, clen, back, n, world, dev, cdev, gloo, allgather)
        ok = ok and assemble["verified"]

    hbm_gbps = hbm_copy_gbps(dev) if rank == 0 else None
    ms_step = elapsed / args.steps * 1e3
    value = total_in / (elapsed / args.steps) / 1e6
    # kernel times are those of the step's last launch (the last piece, or the one decode)
    k1m, k3m, k4m = (float(np.mean(v)) for v in (k1, k3, k4))
    lastp = pieces[-1]
    comp_bytes = clen if decode_only else lastp.clen
    kern_n = n if decode_only else lastp.n
    # dominant kernel (longest average launch) and its algorithmic bytes per
    # launch: compress = N_in + N_out, decompress = N_comp + N_out
    k1_name = "k1r_match_units" if chunk <= 32768 else "k1r_match_units64"
    cands = [(k1m, k1_name, kern_n + comp_bytes), (k4m, "k4_decompress_units", comp_bytes + kern_n)]
    if decode_only:
        cands = cands[1:]
    dom_ms, dom_name, dom_bytes = max(cands)
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    traffic = None
    try:
        pm = json.load(open(args.pmc))
        if pm.get("workload") == args.workload and pm.get("bytes_per_gpu") == kern_n:
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
        size_txt = (f"{total_in / GiB:.4g} GiB in total over {world} GPU(s)" if strong else
                    f"{n / GiB:.4g} GiB/GPU")
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "MB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": f"{args.workload}: {size_txt}, {desc}; one step = "
                                   + ("one decode of the stream" if decode_only else "compress + decompress round trip"),
                       "bytes_per_gpu": n, "total_bytes": total_in, "chunk": chunk,
                       "layout": "STREAMS" if layout else "SINGLE", "units_per_gpu": units,
                       "pieces_per_gpu": len(pieces), "parallelism": f"dp{world} (block shards)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "kernel": dom_name, "kernel_ms": round(dom_ms, 3),
                         "algorithmic_bytes_per_launch": dom_bytes},
            "cpu_baseline": cpu,
            "cpu_baseline_all_cores": cpu_all,
            "cpu_reference": cpu_ref,
            "ratio": round(total_in / total_comp, 4),
            "compress_MBps": None if decode_only else round(kern_n / ((k1m + k3m) * 1e-3) / 1e6, 1),
            "decompress_MBps": round(kern_n / (k4m * 1e-3) / 1e6, 1),
            # src/result.c:40 defines decompress speed over the compressed bytes
            "decompress_MBps_ref_definition": round(comp_bytes / (k4m * 1e-3) / 1e6, 1),
            "hbm_copy_GBps_measured": hbm_gbps,
            "host_end_to_end": e2e,
            "kernel_ms": {"k1_match": None if decode_only else round(k1m, 3),
                          "k3_scan_k2_emit": None if decode_only else round(k3m, 3),
                          "k4_decode": round(k4m, 3)},
            "hbm_frac": {"compress_k1": None if decode_only else
                         round((kern_n + comp_bytes) / (k1m * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                         "decompress_k4": round((kern_n + comp_bytes) / (k4m * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)},
            "round_trip_ok": ok,
        }
        if assemble:
            line["exchange"] = assemble
        print(json.dumps(line), flush=True)
    codec.close()
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


def exchange(out, clen, back, n, world, dev, cdev, gloo, allgather) -> dict:
    """C2: every rank receives the whole compressed stream (padded all-gather:
    RCCL has no all-gatherv); C3: every rank receives the whole decoded output.
    Timed separately from the steps (max over ranks), verified with per-shard
    checksums."""
    res = {}
    sizes = torch.zeros(2 * world, dtype=torch.int64, device=cdev)
    allgather(sizes, torch.tensor([clen, n], dtype=torch.int64, device=cdev))
    sizes = sizes.view(world, 2).cpu()
    mx, mn = int(sizes[:, 0].max()), int(sizes[:, 1].max())  # shards differ (strong scaling): pad
    sums = torch.zeros(2 * world, dtype=torch.int64, device=cdev)
    allgather(sums, torch.tensor([checksum(out[:clen]), checksum(back[:n])], dtype=torch.int64, device=cdev))
    pad = torch.zeros(mx, dtype=torch.uint8, device=cdev)
    pad[:clen] = out[:clen].to(cdev)
    full_c = torch.empty(world * mx, dtype=torch.uint8, device=cdev)
    src_d = torch.zeros(mn, dtype=torch.uint8, device=cdev)
    src_d[:n] = back[:n].to(cdev)
    full_d = torch.empty(world * mn, dtype=torch.uint8, device=cdev)
    for name, dst, src in (("c2_stream_allgather", full_c, pad), ("c3_decoded_allgather", full_d, src_d)):
        allgather(dst, src)  # warm-up
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        allgather(dst, src)
        torch.cuda.synchronize(dev)
        dist.barrier()
        tt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt)
        res[name] = {"ms": round(t * 1e3, 3), "bytes_per_rank_out": int(dst.numel()),
                     "GBps_per_rank_in": round((world - 1) / world * dst.numel() / t / 1e9, 2)}
    full_c, full_d = full_c.to(dev), full_d.to(dev)
    good = True
    for r in range(world):
        good &= checksum(full_c[r * mx: r * mx + int(sizes[r, 0])]) == int(sums[2 * r])
        good &= checksum(full_d[r * mn: r * mn + int(sizes[r, 1])]) == int(sums[2 * r + 1])
    res["stream_bytes"] = int(sizes[:, 0].sum())
    res["verified"] = bool(good)
    return res


if __name__ == "__main__":
    main()
