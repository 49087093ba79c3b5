#!/usr/bin/env python3
"""bench.py -- MI355X Snappy codec benchmark (BASELINE.json metric).

One step = one compress (K1r match finder + K3 scan + K2 emit) and one
decompress (K4) of the rank's batch, inputs already resident in HBM.

Workloads (BASELINE.json configs):
  default, any N   configs[3], the metric's own curve ("at 1/2/4/8 MI355X"):
                   64 GiB of synthetic enwik8-like text as 2,097,152
                   independent 32 KiB streams (each == the reference's
                   snappy_compress() of its chunk), strong-scaled over the N
                   ranks (1 GiB global pieces, block-cyclic), so --gpus
                   1/2/4/8 is one job on one curve.  At N = 1 the same JSON line carries
                   compact sub-results for the other configs -- text32k
                   (configs[1]: 1 GiB of the same streams), text64k (one
                   snappy_compress() stream of 64 KiB blocks), random +
                   repeat (configs[2]), decode10g (configs[4]), config0 (the
                   1,000,000-byte text file through the FILE* API, the
                   compiled reference beside it) -- and host_file_api, the
                   FILE* entry points cmd.c calls, on a 4 GiB file in /dev/shm.
  --workload W     W alone: 1 GiB per rank at N = 1 (decode10g: its ~10 GB
                   stream), 64 GiB strong-scaled at N > 1.
  --weak / --bytes-per-gpu B   B bytes per rank (default 1 GiB).
  --total-bytes T  any fixed job size, strong-scaled.

Sharding is block-cyclic (dist.piece_plan): the job is cut into global pieces
(--e2e-piece-bytes, default a quarter of a share, <= 1 GiB) and piece g belongs
to rank g mod N.  Exchange steps: C1, the all-gather of the
shard sizes, is part of every step of the timed loop (`value`: the per-rank
compute curve).  With N > 1 a second timed loop runs the whole job end to end
as a pipeline -- per step: compress the rank's piece, C1, C2 (RCCL all-gather
of the step's payloads, padded: RCCL has no all-gatherv) copied into the
contiguous stream every rank then holds, decode of the rank's piece from that
stream; C2 and the decode overlap the next step's compress -- and reports it
as `value_end_to_end`.  C3 (all-gather of the decoded shards) is opt-in
(--c3).  Every phase is checked (round trip, per-piece checksums).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
                       [--workload text32k|text64k|random|repeat|decode10g]
                       [--total-bytes T | --weak [--bytes-per-gpu B]]
--gpus N without a torch.distributed launcher spawns the N ranks itself
(python -m torch.distributed.run, 127.0.0.1); this parent process never
touches the GPU.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "lightweight-snappy_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import datagen  # noqa: E402
import snappy_amd  # noqa: E402
from dist import (C2_MAX_BYTES, HBM_BYTES, c2_gather_step, default_e2e_piece, piece_plan, piece_step, pieces_of,  # noqa: E402
                  pipeline_steps, rank_plan)

METRIC = "compress + decompress MB/s at 1/2/4/8 MI355X; % HBM roofline; ratio vs ref"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
GiB = 1 << 30
CONFIG3_BYTES = 64 * GiB  # BASELINE configs[3]: 64 GB of 32 KB blocks over 1/2/4/8 GPUs

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
SUB_WORKLOADS = ("text32k", "text64k", "random", "repeat", "decode10g")
CONFIG0_BYTES = 1_000_000  # BASELINE configs[0]: one 1 MB text buffer (src/snappy_test.c:7)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="text32k", choices=sorted(WORKLOADS))
    ap.add_argument("--bytes-per-gpu", type=int, default=None,
                    help="weak scaling: input bytes per rank (default 1 GiB with --weak)")
    ap.add_argument("--total-bytes", type=int, default=0,
                    help="strong scaling: fixed job size sharded over the ranks (default: 68719476736 = "
                         "configs[3] for text32k at every N and for every workload at N > 1)")
    ap.add_argument("--weak", action="store_true", help="--bytes-per-gpu per rank instead of configs[3]")
    ap.add_argument("--piece-bytes", type=int, default=8 * GiB,
                    help="a rank compresses its range in pieces of at most this many bytes (bounds token scratch)")
    ap.add_argument("--no-assemble", action="store_true", help="N > 1: skip the end-to-end loop with C2")
    ap.add_argument("--e2e-piece-bytes", type=int, default=0,
                    help="the job's global piece (block-cyclic sharding, one pipeline step of the end-to-end loop "
                         "per piece per rank; default dist.default_e2e_piece: a quarter of a share, <= 1 GiB)")
    ap.add_argument("--c2-max-bytes", type=int, default=C2_MAX_BYTES,
                    help="one C2 all-gather sends at most this many bytes per rank (a step's larger payload is "
                         "gathered in several)")
    ap.add_argument("--e2e-dump", default=None,
                    help="rank 0 writes the reassembled stream of the end-to-end loop to this file (tests)")
    ap.add_argument("--no-e2e-overlap", action="store_true",
                    help="end-to-end loop: run each step's C2 and decode before the next step's compress (A/B)")
    ap.add_argument("--c3", action="store_true", help="N > 1: also time C3, the all-gather of the decoded shards")
    ap.add_argument("--e2e-steps", type=int, default=3, help="N > 1: steps of the end-to-end loop")
    ap.add_argument("--overlap", action="store_true",
                    help="decode piece k on a second stream while piece k + 1 compresses")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-e2e", action="store_true", help="skip the PCIe-inclusive host API samples")
    ap.add_argument("--no-sub", action="store_true", help="N = 1: skip the sub-results of the other configs")
    ap.add_argument("--file-api-bytes", type=int, default=4 * GiB, help="host_file_api: size of the /dev/shm file")
    ap.add_argument("--keep-size", action="store_true", help="decode10g: use --bytes-per-gpu as given")
    ap.add_argument("--dist-world1", action="store_true",
                    help="N = 1: still create the process group and run the end-to-end exchange loop (1 rank)")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="nccl (= RCCL, the real path) or gloo (CPU collectives; rehearsal with ranks sharing a GPU)")
    ap.add_argument("--cpu-sample-bytes", type=int, default=GiB)
    ap.add_argument("--pmc", default=None,
                    help="rocprofv3 PMC summary giving HBM traffic per launch (default: the profiles/pmc_*.json "
                         "written by tools/pmc_summary.py for this workload and launch size)")
    return ap.parse_args(argv)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int) -> int:
    """--gpus N outside a launcher: run N ranks under torch.distributed.run
    (a child process; nothing here has touched the GPU)."""
    port = _free_port()
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


def cpu_baseline(kind: str, seed: int, chunk: int, layout: int, sample: int, decode_only: bool = False,
                 all_cores: bool = True):
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
    if not all_cores:
        return base, None
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


def host_end_to_end(kind: str, seed: int, sample: int, runs: int = 5) -> dict:
    """PCIe-inclusive rate of the drop-in host API (snappy_compress_buffer /
    snappy_decompress_buffer: one SINGLE stream of 64 KiB blocks, pageable
    host buffers in and out).  Reported beside `value`, never as it."""
    lib = snappy_amd.lib()
    a = datagen.make(kind, sample, seed)
    cap = snappy_amd.max_compressed_length(a.size)
    comp = np.empty(cap, dtype=np.uint8)
    back = np.empty(a.size, dtype=np.uint8)
    got = ctypes.c_size_t(0)
    vp = ctypes.c_void_p
    tc, td = [], []
    for _ in range(1 + runs):  # the first call also allocates the pipeline's contexts: untimed
        t0 = time.perf_counter()
        rc = lib.snappy_compress_buffer(vp(a.ctypes.data), a.size, vp(comp.ctypes.data), ctypes.byref(got))
        t1 = time.perf_counter()
        assert rc == 0, rc
        clen = got.value
        rc = lib.snappy_decompress_buffer(vp(comp.ctypes.data), clen, vp(back.ctypes.data), a.size,
                                          ctypes.byref(got))
        t2 = time.perf_counter()
        assert rc == 0 and got.value == a.size, rc
        tc.append(t1 - t0)
        td.append(t2 - t1)
    assert np.array_equal(back, a)
    return dict({"bytes": int(a.size), "layout": "SINGLE 64 KiB blocks",
                 "note": f"pageable host buffers, H2D+D2H included; median of {runs} timed runs after one untimed"},
                **rate_stats(a.size, tc[1:], "compress"), **rate_stats(a.size, td[1:], "decompress"))


def rate_stats(nbytes: int, times, what: str) -> dict:
    """{what}_MBps (the median run) and its min / max over the runs."""
    r = sorted(nbytes / t / 1e6 for t in times)
    return {f"{what}_MBps": round(float(np.median(r)), 1), f"{what}_MBps_min": round(r[0], 1),
            f"{what}_MBps_max": round(r[-1], 1)}


def host_file_api(nbytes: int, runs: int = 3) -> dict:
    """The path src/cmd.c:90-98 actually calls: snappy_compress(FILE*, size,
    FILE*) and snappy_decompress(FILE*, FILE*) of libsnappy_amd.so, on an
    nbytes text file in /dev/shm (page cache, so the disk is not what is
    measured), in-process through libc stdio (no process start in the time).
    MB/s = uncompressed bytes / wall second, as src/result.c prints them.
    The output is checked byte for byte against the input."""
    lib = snappy_amd.lib()
    libc = ctypes.CDLL(None)
    libc.fopen.restype = ctypes.c_void_p
    libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    libc.fclose.argtypes = [ctypes.c_void_p]
    d = "/dev/shm" if os.path.isdir("/dev/shm") else None
    with tempfile.TemporaryDirectory(dir=d, prefix="snappy_bench_") as tmp:
        src, snp, dec = (os.path.join(tmp, x).encode() for x in ("in", "in.snp", "in.dec"))
        a = np.empty(nbytes, dtype=np.uint8)
        datagen.fill(a, "T", 1234, threads=16)
        a.tofile(src.decode())
        del a

        def run(fn, *files, size=None):
            fi = libc.fopen(files[0], b"rb")
            fo = libc.fopen(files[1], b"wb")
            assert fi and fo
            t0 = time.perf_counter()
            rc = fn(ctypes.c_void_p(fi), ctypes.c_ulonglong(size), ctypes.c_void_p(fo)) if size is not None else \
                fn(ctypes.c_void_p(fi), ctypes.c_void_p(fo))
            libc.fclose(ctypes.c_void_p(fo))
            t = time.perf_counter() - t0
            libc.fclose(ctypes.c_void_p(fi))
            return rc, t

        tcs, tds = [], []
        for _ in range(1 + runs):  # the first round also allocates the pipeline's pinned slots: untimed
            _, tc = run(lib.snappy_compress, src, snp, size=nbytes)
            assert lib.snappy_amd_last_status() == 0
            rc, td = run(lib.snappy_decompress, snp, dec)
            assert rc == 0 and lib.snappy_amd_last_status() == 0, rc
            tcs.append(tc)
            tds.append(td)
        clen = os.path.getsize(snp.decode())
        ok = os.path.getsize(dec.decode()) == nbytes and \
            np.array_equal(np.fromfile(dec.decode(), dtype=np.uint8), np.fromfile(src.decode(), dtype=np.uint8))
    return dict({"bytes": nbytes, "file": "/dev/shm" if d else "tmp", "compressed_bytes": clen,
                 "round_trip_ok": bool(ok),
                 "note": f"snappy_compress / snappy_decompress FILE* entry points (cmd.c's calls), text, median of "
                         f"{runs} timed runs after one untimed, file I/O + PCIe + kernels"},
                **rate_stats(nbytes, tcs[1:], "compress"), **rate_stats(nbytes, tds[1:], "decompress"))


def config0_file_api(reps: int = 20) -> dict:
    """BASELINE configs[0] as stated: snappy_compress + snappy_decompress
    (src/cmd.c:90-98's calls) on one 1,000,000-byte text buffer written to a
    file in /dev/shm -- the compiled reference (oracle/_ref/libsnappy_ref.so,
    1 core; CPU-baseline leg only) and libsnappy_amd.so's FILE* path side by
    side on the same file, in-process through libc stdio: the median of the
    reps - 1 calls after a first untimed one (min / max and the best beside it).
    Both outputs are checked: the two compressed files byte-identical, both
    decodes equal to the input.  MB/s = input bytes / wall second, as
    src/result.c:30-31 prints them."""
    lib = snappy_amd.lib()
    libc = ctypes.CDLL(None)
    libc.fopen.restype = ctypes.c_void_p
    libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    libc.fclose.argtypes = [ctypes.c_void_p]
    ref_path = os.path.join(ROOT, "oracle", "_ref", "libsnappy_ref.so")
    ref = ctypes.CDLL(ref_path) if os.path.exists(ref_path) else None  # RTLD_LOCAL: its own snappy_compress
    a = datagen.make("T", CONFIG0_BYTES, 1234)  # golden entry text_1000000
    d = "/dev/shm" if os.path.isdir("/dev/shm") else None
    res = {"workload": "config0: 1,000,000 B of synthetic text (golden text_1000000), one snappy_compress() stream, "
                       "FILE* API in and out of /dev/shm", "bytes": CONFIG0_BYTES}
    with tempfile.TemporaryDirectory(dir=d, prefix="snappy_c0_") as tmp:
        src = os.path.join(tmp, "in").encode()
        a.tofile(src.decode())

        def time_lib(l, tag):
            snp, dec = (os.path.join(tmp, f"{tag}.{x}").encode() for x in ("snp", "dec"))
            tcs, tds = [], []
            for _ in range(reps):
                for mode in (0, 1):
                    fi = libc.fopen(src if mode == 0 else snp, b"rb")
                    fo = libc.fopen(snp if mode == 0 else dec, b"wb")
                    assert fi and fo
                    t0 = time.perf_counter()
                    if mode == 0:
                        l.snappy_compress(ctypes.c_void_p(fi), ctypes.c_ulonglong(CONFIG0_BYTES), ctypes.c_void_p(fo))
                    else:
                        l.snappy_decompress(ctypes.c_void_p(fi), ctypes.c_void_p(fo))
                    libc.fclose(ctypes.c_void_p(fo))
                    t = time.perf_counter() - t0
                    libc.fclose(ctypes.c_void_p(fi))
                    (tcs if mode == 0 else tds).append(t)
            comp = open(snp.decode(), "rb").read()
            ok = open(dec.decode(), "rb").read() == a.tobytes()
            mc, md = float(np.median(tcs[1:])), float(np.median(tds[1:]))  # (the first call warms up)
            return dict({"round_trip_MBps": round(CONFIG0_BYTES / (mc + md) / 1e6, 1),
                         "compressed_bytes": len(comp), "round_trip_ok": ok,
                         "compress_MBps_best": round(CONFIG0_BYTES / min(tcs) / 1e6, 1),
                         "decompress_MBps_best": round(CONFIG0_BYTES / min(tds) / 1e6, 1)},
                        **rate_stats(CONFIG0_BYTES, tcs[1:], "compress"),
                        **rate_stats(CONFIG0_BYTES, tds[1:], "decompress")), comp

        gpu, comp_gpu = time_lib(lib, "gpu")
        assert lib.snappy_amd_last_status() == 0
        res["gpu_file_api"] = dict(gpu, note="libsnappy_amd.so snappy_compress/snappy_decompress, 1 MI355X: one "
                                             "65,536-byte-block stream, PCIe + launch latency dominate at 1 MB")
        ok = gpu["round_trip_ok"]
        if ref is not None:
            r, comp_ref = time_lib(ref, "ref")
            res["cpu_reference"] = dict(r, cores=1, kind="reference",
                                        note=f"reference src/*.c -O2 FILE* API, 1 thread, {cpu_model()}")
            res["identical_to_reference"] = comp_ref == comp_gpu
            ok = ok and r["round_trip_ok"] and comp_ref == comp_gpu
    res["round_trip_ok"] = bool(ok)
    return res


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
    s = 0
    # in 16 MiB slices, so the int64 temporaries stay small next to a 32 GiB shard
    for o in range(0, m, 1 << 24):
        e = min(m, o + (1 << 24))
        body = t[o:e].view(-1, k).to(torch.int64)
        rows = (body * w).sum(dim=1)
        r0 = o // k
        s += int((rows * torch.arange(r0 + 1, r0 + rows.numel() + 1, device=t.device, dtype=torch.int64)).sum())
    tail = t[m:].to(torch.int64)
    s += int((tail * w[: tail.numel()]).sum()) * 7919 + n
    return s & ((1 << 62) - 1)


def load_pmc(path, workload: str, n: int) -> dict:
    """{kernel: hbm_bytes per launch} from the tools/pmc_summary.py file
    measured on this workload with launches of n input bytes (the file at
    `path`, or the newest matching profiles/pmc_*.json)."""
    import glob
    cands = [path] if path else sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json")))
    best = None
    for p in cands:
        try:
            pm = json.load(open(p))
        except (OSError, ValueError):
            continue
        if pm.get("workload") == workload and pm.get("launch_bytes", pm.get("bytes_per_gpu")) == n and \
                "kernels" in pm and (best is None or str(pm.get("round", "")) > str(best[0].get("round", ""))):
            best = (pm, p)
    if best is None:
        return {}
    out = {k: v.get("hbm_bytes") for k, v in best[0]["kernels"].items()}
    out["_source"] = os.path.relpath(best[1], ROOT)
    return out


class Piece:
    """A unit-aligned launch over part of the rank's input x, compressed into
    its own slice of the rank's payload (only the stream's first launch
    carries the SINGLE varint preamble)."""

    def __init__(self, off: int, n: int, flags: int):
        self.off, self.n, self.flags = off, n, flags
        self.clen = 0
        self.out_off = 0
        self.offs = None


class GPiece:
    """One of the rank's global pieces (dist.piece_plan): global piece g at
    global offset goff, held at x[xoff:xoff+n]; in the end-to-end loop it is
    compressed into payload slot k (out[k*slot:]) and gathered in step k."""

    def __init__(self, k: int, g: int, goff: int, xoff: int, n: int, flags: int):
        self.k, self.g, self.goff, self.xoff, self.n, self.flags = k, g, goff, xoff, n, flags
        self.clen = 0
        self.offs = None


class Job:
    """One workload's buffers on this rank: the input (the rank's global
    pieces back to back) in HBM, the payload, the decoded output and the
    per-launch block indexes.  The timed loop compresses x in launches of
    <= piece_bytes (the compressed pieces packed); the end-to-end loop per
    global piece into fixed slots (dist.rank_plan sizes `out` for both)."""

    def __init__(self, name, codec, dev, gpieces, total_in, piece_bytes, e2e_piece, steps_e2e, keep_size=False):
        kind, seed, layout, chunk, desc = WORKLOADS[name]
        self.name, self.kind, self.seed, self.layout, self.chunk, self.desc = name, kind, seed, layout, chunk, desc
        self.codec, self.dev = codec, dev
        self.decode_only = name in DECODE_ONLY
        self.unit = chunk if layout == snappy_amd.STREAMS else 65536
        n = sum(m for _, _, m in gpieces)
        self.n, self.total_in = n, total_in
        self.gpieces = []
        xo = 0
        for k, (g, goff, m) in enumerate(gpieces):
            flags = snappy_amd.NO_PREAMBLE if (layout == snappy_amd.SINGLE and goff > 0) else 0
            self.gpieces.append(GPiece(k, g, goff, xo, m, flags))
            xo += m
        # the rank's pieces in HBM, generated on the host 1 GiB at a time
        self.x = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
        host = np.empty(min(max(n, 1), GiB), dtype=np.uint8)
        for gp in self.gpieces:
            for o in range(0, gp.n, GiB):
                m = min(GiB, gp.n - o)
                datagen.fill(host[:m], kind, seed, offset=gp.goff + o, threads=16)
                self.x[gp.xoff + o:gp.xoff + o + m].copy_(torch.from_numpy(host[:m]))
        del host
        self.units = codec.num_units(n, chunk, layout)
        # the timed loop's launches over x: x[0] is global offset 0 only on the rank owning piece 0
        first_global = bool(self.gpieces) and self.gpieces[0].goff == 0
        self.pieces = []
        o = 0
        for m in pieces_of(n, self.unit, piece_bytes):
            flags = snappy_amd.NO_PREAMBLE if (layout == snappy_amd.SINGLE and (o > 0 or not first_global)) else 0
            self.pieces.append(Piece(o, m, flags))
            o += m
        self.e2e_piece, self.steps_e2e = e2e_piece, steps_e2e
        self.slot = codec.max_output(e2e_piece, chunk, layout)
        cap = sum(codec.max_output(m, chunk, layout) for m in pieces_of(n, self.unit, piece_bytes))
        self.out_cap = max(cap, steps_e2e * self.slot, 16)
        self.out = torch.empty(self.out_cap, dtype=torch.uint8, device=dev)
        for p in self.pieces:
            p.offs = torch.empty(codec.num_units(p.n, chunk, layout) + 1, dtype=torch.int64, device=dev)
        self.back = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
        # SINGLE layout: the stream's first piece carries the global preamble
        self.header_value = total_in if layout == snappy_amd.SINGLE else n
        self.pre_clen = None
        self.g_offs = None
        self.dcodec = self.dstream = None  # --overlap: the decode codec and its stream
        self.last_dec = codec  # the codec of the last decode (its status is the one to read)
        if self.decode_only:  # the stream and its block index exist before the timed region
            self.pre_clen = self.compress_all()
            self.g_offs = torch.cat([p.offs[:-1] + p.out_off for p in self.pieces] +
                                    [torch.tensor([self.pre_clen], dtype=torch.int64, device=dev)])

    def compress_all(self) -> int:
        o = 0
        for p in self.pieces:
            p.out_off = o
            p.clen = self.codec.compress_ptr_ex(self.x.data_ptr() + p.off, p.n, self.chunk, self.layout, p.flags,
                                                self.header_value, self.out.data_ptr() + o, p.offs.data_ptr())
            o += p.clen
        return o

    def step_overlapped(self, c1=None) -> int:
        """One compress + decompress step with the decode of piece k (on the
        second codec's stream) running while piece k + 1 compresses: K4 is
        issue-bound and K1r latency-bound, so their waves share the CUs.  Piece
        k's compression waits for its previous decode (an event), so the next
        step never overwrites a payload still being read."""
        o = 0
        for k, p in enumerate(self.pieces):
            if self.dec_done[k] is not None:
                torch.cuda.current_stream(self.dev).wait_event(self.dec_done[k])
            p.out_off = o
            p.clen = self.codec.compress_ptr_ex(self.x.data_ptr() + p.off, p.n, self.chunk, self.layout, p.flags,
                                                self.header_value, self.out.data_ptr() + o, p.offs.data_ptr())
            o += p.clen
            # piece k is compressed (compress_ptr_ex synchronised its stream): decode it on stream B
            self.dstream.wait_stream(torch.cuda.current_stream(self.dev))
            self.dcodec.decompress_ptr_ex(self.out.data_ptr() + p.out_off, p.offs.data_ptr(), p.n, self.chunk,
                                          self.layout, p.flags, self.header_value, self.back.data_ptr() + p.off,
                                          check=False)
            self.last_dec = self.dcodec
            ev = torch.cuda.Event()
            ev.record(self.dstream)
            self.dec_done[k] = ev
        if c1 is not None:
            c1(o)
        return o

    def enable_overlap(self, dcodec, dstream) -> None:
        self.dcodec, self.dstream = dcodec, dstream
        self.dec_done = [None] * len(self.pieces)

    def decompress_all(self, base_ptr=None) -> None:
        """Decode every piece from the payload at base_ptr (default: this rank's own)."""
        base_ptr = self.out.data_ptr() if base_ptr is None else base_ptr
        self.last_dec = self.codec
        if self.decode_only:
            self.codec.decompress_ptr_ex(base_ptr, self.g_offs.data_ptr(), self.n, self.chunk, self.layout,
                                         self.pieces[0].flags, self.header_value, self.back.data_ptr(), check=False)
            return
        for p in self.pieces:
            self.codec.decompress_ptr_ex(base_ptr + p.out_off, p.offs.data_ptr(), p.n, self.chunk, self.layout,
                                         p.flags, self.header_value, self.back.data_ptr() + p.off, check=False)

    def verify(self) -> bool:
        st = self.last_dec.decompress_status()
        if st != 0:
            return False
        # in 1 GiB slices: torch.equal's temporaries stay small next to a 64 GiB shard
        return all(bool(torch.equal(self.back[o:min(o + GiB, self.n)], self.x[o:min(o + GiB, self.n)]))
                   for o in range(0, self.n, GiB))

    def free(self):
        for a in ("x", "out", "back", "g_offs"):
            setattr(self, a, None)
        for p in self.pieces + self.gpieces:
            p.offs = None
        torch.cuda.empty_cache()


def timed_steps(job: Job, steps: int, warmup: int, world: int, c1=None):
    """Warm up, then time exactly `steps` steps between barrier + synchronize;
    returns (elapsed seconds of this rank, clen, [k1 ms], [k3 ms], [k4 ms])."""
    dev = job.dev

    def step():
        if job.decode_only:
            job.decompress_all()
            return job.pre_clen
        if job.dcodec is not None:
            return job.step_overlapped(c1)
        clen = job.compress_all()
        if c1 is not None:
            c1(clen)
        job.decompress_all()
        return clen

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    k1, k3, k4 = [], [], []
    clen = 0
    t0 = time.perf_counter()
    for _ in range(steps):
        clen = step()
        a, b, c = job.codec.last_timings()
        if job.dcodec is not None:
            c = job.dcodec.last_timings()[2]
        k1.append(a), k3.append(b), k4.append(c)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    return time.perf_counter() - t0, clen, k1, k3, k4


def kernel_report(job: Job, clen: int, k1, k3, k4, pmc: dict) -> dict:
    """Kernel times of the step's last launch (the last piece, or the one
    decode), the dominant kernel's roofline and the per-path traffic."""
    k1m, k3m, k4m = (float(np.mean(v)) for v in (k1, k3, k4))
    lastp = job.pieces[-1]
    comp_bytes = clen if job.decode_only else lastp.clen
    kern_n = job.n if job.decode_only else lastp.n
    # dominant kernel (longest average launch) and its algorithmic bytes per
    # launch: compress = N_in + N_out, decompress = N_comp + N_out
    k1_name = "k1r_match_units" if job.chunk <= 32768 else "k1r_match_units64"
    alg = kern_n + comp_bytes
    cands = [(k1m, k1_name, alg), (k4m, "k4_decompress_units", alg)]
    if job.decode_only:
        cands = cands[1:]
    dom_ms, dom_name, dom_bytes = max(cands)
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    traffic = pmc.get(dom_name)
    roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            "kernel": dom_name, "kernel_ms": round(dom_ms, 3), "algorithmic_bytes_per_launch": dom_bytes,
            "launch_bytes": kern_n}
    if traffic is not None:
        roof["traffic_source"] = pmc.get("_source")
    # counter bytes of each whole path (K1r + K3 + K2 write the compressed
    # bytes; K4 alone decodes) beside the same path's algorithmic bytes
    paths = {}
    comp_k = [k1_name, "k3_scan", "k2_emit_units"]
    if not job.decode_only and all(pmc.get(k) is not None for k in comp_k):
        t = sum(pmc[k] for k in comp_k)
        paths["compress"] = {"counter_bytes": t, "algorithmic_bytes": alg, "ratio": round(t / alg, 3),
                             "kernels": comp_k}
    if pmc.get("k4_decompress_units") is not None:
        t = pmc["k4_decompress_units"] + (pmc.get("k4_decompress_back") or 0)
        paths["decompress"] = {"counter_bytes": t, "algorithmic_bytes": alg, "ratio": round(t / alg, 3),
                               "kernels": ["k4_decompress_units", "k4_decompress_back"]}
    if paths:
        roof["path_traffic"] = paths
    return {
        "roofline": roof,
        "compress_MBps": None if job.decode_only else round(kern_n / ((k1m + k3m) * 1e-3) / 1e6, 1),
        "decompress_MBps": round(kern_n / (k4m * 1e-3) / 1e6, 1),
        # src/result.c:40 defines decompress speed over the compressed bytes
        "decompress_MBps_ref_definition": round(comp_bytes / (k4m * 1e-3) / 1e6, 1),
        "kernel_ms": {"k1_match": None if job.decode_only else round(k1m, 3),
                      "k3_scan_k2_emit": None if job.decode_only else round(k3m, 3),
                      "k4_decode": round(k4m, 3)},
        "hbm_frac": {"compress_k1": None if job.decode_only else round(alg / (k1m * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                     "decompress_k4": round(alg / (k4m * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)},
    }


def sub_result(name: str, codec, dev, steps: int, warmup: int, piece_bytes: int, cpu: bool) -> dict:
    """A compact single-GPU line for another BASELINE config (1 GiB, or the
    ~10 GB stream of decode10g), with its own kernel times, roofline and a
    CPU baseline on a 64 MiB sample of the same workload."""
    n = DECODE10G_BYTES if name in DECODE_ONLY else GiB
    t_gen = time.perf_counter()
    job = Job(name, codec, dev, [(0, 0, n)], n, piece_bytes, n, 1)
    t_gen = time.perf_counter() - t_gen
    elapsed, clen, k1, k3, k4 = timed_steps(job, steps, warmup, 1)
    ok = job.verify()
    rep = kernel_report(job, clen, k1, k3, k4, load_pmc(None, name, job.n if job.decode_only
                                                        else job.pieces[-1].n))
    total_comp = clen
    job.free()
    res = {"workload": f"{name}: {n / GiB:.4g} GiB, {job.desc}", "value": round(n / (elapsed / steps) / 1e6, 1),
           "unit": "MB/s", "steps": steps, "ms_per_step": round(elapsed / steps * 1e3, 3),
           "ratio": round(n / total_comp, 4), "compress_MBps": rep["compress_MBps"],
           "decompress_MBps": rep["decompress_MBps"], "kernel_ms": rep["kernel_ms"],
           "roofline": {k: rep["roofline"][k] for k in ("kernel", "kernel_ms", "achieved", "frac", "traffic",
                                                        "traffic_source", "launch_bytes") if k in rep["roofline"]},
           "round_trip_ok": ok, "setup_s": round(t_gen, 1)}
    if "path_traffic" in rep["roofline"]:
        res["roofline"]["path_traffic"] = rep["roofline"]["path_traffic"]
    if cpu:
        kind, seed, layout, chunk, _ = WORKLOADS[name]
        base, _ = cpu_baseline(kind, seed, chunk, layout, 64 << 20, name in DECODE_ONLY, all_cores=False)
        res["cpu_baseline"] = base
    return res


def resolve_sizes(args, world: int, rank: int):
    """(strong, total input bytes, this rank's global pieces [(g, offset,
    bytes)], its bytes, the end-to-end piece, the pipeline's steps).
    Without size flags: configs[3] (64 GiB in total, strong scaling) for
    text32k at every N -- so --gpus 1/2/4/8 is one job on one curve -- and
    for every other compressing workload at N > 1; another workload alone at
    N = 1 is 1 GiB (decode10g: its ~10 GB stream).  Sharding is block-cyclic
    in pieces of --e2e-piece-bytes (dist.piece_plan; at N = 1 the whole
    range)."""
    kind, seed, layout, chunk, desc = WORKLOADS[args.workload]
    unit = chunk if layout == snappy_amd.STREAMS else 65536
    total = args.total_bytes
    weak = args.weak or args.bytes_per_gpu is not None
    if total == 0 and not weak and args.workload not in DECODE_ONLY and (world > 1 or args.workload == "text32k"):
        total = CONFIG3_BYTES
    strong = total > 0
    if not strong:
        n = args.bytes_per_gpu if args.bytes_per_gpu is not None else GiB
        if args.workload in DECODE_ONLY and args.bytes_per_gpu is None and not args.keep_size:
            n = DECODE10G_BYTES
        total = n * world
    e2e = piece_step(unit, args.e2e_piece_bytes) if args.e2e_piece_bytes else default_e2e_piece(total, world, unit)
    # a piece larger than the whole job is the job (dist.rank_plan sizes the
    # payload slot from the same bound, so the allocations match the plan)
    e2e = min(e2e, piece_step(unit, total + unit - 1))
    gp = piece_plan(total, world, rank, unit, e2e)
    return strong, total, gp, sum(m for _, _, m in gp), e2e, pipeline_steps(total, world, unit, e2e)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gloo = args.dist_backend == "gloo"
    # a process group also at N = 1 with --dist-world1 (the exchange code path
    # over a 1-rank RCCL communicator: what a 1-GPU box can run of it)
    use_dist = world > 1 or args.dist_world1
    if use_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        # gloo: rehearsal of the multi-rank path (ranks may share a GPU)
        local = local % torch.cuda.device_count() if gloo else local
        torch.cuda.set_device(local)
        if gloo:
            dist.init_process_group("gloo")
        else:
            # RCCL's collectives run on the process group's own stream: a high-priority
            # one takes a hardware queue of its own instead of sharing one of the
            # process's GPU_MAX_HW_QUEUES (4) with the compute streams, where a C2
            # collective would wait behind a K1r launch (DESIGN.md 6 lists a rank's streams)
            os.environ.setdefault("TORCH_NCCL_HIGH_PRIORITY", "1")
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if use_dist else 0)
    cdev = torch.device("cpu") if gloo else dev  # where collective tensors live

    decode_only = args.workload in DECODE_ONLY
    kind, seed, layout, chunk, desc = WORKLOADS[args.workload]
    unit = chunk if layout == snappy_amd.STREAMS else 65536
    strong, total_in, gpieces, n, e2e_piece, e2e_steps = resolve_sizes(args, world, rank)
    codec = snappy_amd.Codec(dev.index)
    codec.enable_timing(True)
    stream = torch.cuda.current_stream(dev)
    codec.set_stream(stream.cuda_stream)
    t_setup = time.perf_counter()
    job = Job(args.workload, codec, dev, gpieces, total_in, args.piece_bytes, e2e_piece, e2e_steps)
    dcodec = None
    if args.overlap and not decode_only:
        dcodec = snappy_amd.Codec(dev.index)
        dcodec.enable_timing(True)
        dstream = torch.cuda.Stream(dev)
        dcodec.set_stream(dstream.cuda_stream)
        job.enable_overlap(dcodec, dstream)
    t_setup = time.perf_counter() - t_setup
    sizes_t = torch.zeros(world, dtype=torch.int64, device=cdev)

    def allgather(dst, src):
        if gloo:
            parts = list(dst.chunk(world))
            dist.all_gather(parts, src)
            if parts[0].data_ptr() != dst.data_ptr():
                dst.copy_(torch.cat(parts))
        else:
            dist.all_gather_into_tensor(dst, src)

    def c1(clen):  # C1: shard sizes -> global stream offsets
        allgather(sizes_t, torch.tensor([clen], dtype=torch.int64, device=cdev))

    elapsed, clen, k1, k3, k4 = timed_steps(job, args.steps, args.warmup, world if use_dist else 1,
                                            c1 if use_dist else None)
    scratch_peak = codec.device_bytes() + (dcodec.device_bytes() if dcodec else 0)
    torch_peak = torch.cuda.max_memory_allocated(dev)  # the buffers of the steps, before any check runs
    ok = job.verify()
    if use_dist:
        t = torch.tensor([elapsed, 0.0 if ok else 1.0], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, bad = float(t[0]), float(t[1])
        ok = bad == 0.0
        tot = torch.tensor([clen], dtype=torch.int64, device=cdev)
        dist.all_reduce(tot)
        total_comp = int(tot)
    else:
        total_comp = clen
    mem_after_steps = torch.cuda.mem_get_info(dev)

    assemble = None
    if use_dist and not args.no_assemble and not decode_only:
        meta = dist.group.WORLD if gloo else dist.new_group(backend="gloo")  # C1: host-side sizes
        assemble = end_to_end(job, world, rank, args, cdev, gloo, allgather, total_in, meta)
        torch_peak = max(torch_peak, assemble.pop("torch_peak_bytes"))
        ok = ok and assemble["verified"]
        if args.c3:
            assemble["c3_decoded_allgather"] = gather_decoded(job, world, cdev, gloo, allgather)
            ok = ok and assemble["c3_decoded_allgather"]["verified"]

    ms_step = elapsed / args.steps * 1e3
    value = total_in / (elapsed / args.steps) / 1e6
    pmc = load_pmc(args.pmc, args.workload, job.n if decode_only else job.pieces[-1].n)
    config3 = strong and total_in == CONFIG3_BYTES and args.workload == "text32k"
    rep = kernel_report(job, clen, k1, k3, k4, pmc)
    plan = rank_plan(total_in, world, unit, args.piece_bytes, exchange=world > 1 and not args.no_assemble,
                     gather_decoded=args.c3, e2e_piece=e2e_piece, c2_max=args.c2_max_bytes)
    used = mem_after_steps[1] - mem_after_steps[0]
    rank_peak = torch_peak + scratch_peak
    n_units = job.units
    launch_bytes = job.n if decode_only else job.pieces[-1].n
    job.free()

    line = None
    if rank == 0:
        hbm_gbps = hbm_copy_gbps(dev)
        cpu = cpu_all = cpu_ref = e2e = None
        if world == 1 and not args.no_cpu_baseline:
            cpu, cpu_all = cpu_baseline(kind, seed, chunk, layout, min(args.cpu_sample_bytes, n), decode_only)
            cpu_ref = cpu_reference(kind, seed, chunk, layout, min(128 << 20, n), decode_only)
        if world == 1 and not args.no_host_e2e and not decode_only:
            e2e = host_end_to_end(kind, seed, min(n, 256 << 20))
        size_txt = (f"{total_in / GiB:.4g} GiB in total over {world} GPU(s)" if strong else
                    f"{n / GiB:.4g} GiB/GPU")
        cfg_name = "configs[3]" if config3 else \
            {"text32k": "configs[1]", "text64k": "configs[1] (64 KiB blocks)", "random": "configs[2]",
             "repeat": "configs[2]", "decode10g": "configs[4]"}[args.workload]
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "MB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": f"{args.workload} ({cfg_name}): {size_txt}, {desc}; one step = "
                                   + ("one decode of the stream" if decode_only else
                                      "compress + decompress round trip" + (" + C1 size all-gather" if world > 1
                                                                            else "")),
                       "bytes_per_gpu": n, "total_bytes": total_in, "chunk": chunk,
                       "layout": "STREAMS" if layout else "SINGLE", "units_per_gpu": n_units,
                       "pieces_per_gpu": len(job.pieces), "launch_bytes": launch_bytes,
                       "workload_name": args.workload, "parallelism": f"dp{world} (block shards)",
                       "overlap": bool(dcodec)},
            "roofline": rep["roofline"],
            "cpu_baseline": cpu,
            "cpu_baseline_all_cores": cpu_all,
            "cpu_reference": cpu_ref,
            "ratio": round(total_in / total_comp, 4),
            "compress_MBps": rep["compress_MBps"],
            "decompress_MBps": rep["decompress_MBps"],
            "decompress_MBps_ref_definition": rep["decompress_MBps_ref_definition"],
            "hbm_copy_GBps_measured": hbm_gbps,
            "host_end_to_end": e2e,
            "kernel_ms": rep["kernel_ms"],
            "hbm_frac": rep["hbm_frac"],
            "memory": {"rank_peak_bytes": int(rank_peak), "torch_peak_bytes": int(torch_peak),
                       "codec_scratch_bytes": int(scratch_peak), "device_bytes_in_use_after_steps": int(used),
                       "planned_peak_bytes_per_rank": plan["peak"], "hbm_bytes": HBM_BYTES,
                       "note": "rank_peak = torch allocator peak (shard, payload, decoded, indexes, C2 buffers) + "
                               "codec scratch (hipMalloc'd by the library); plan = dist.rank_plan, worst case"},
            "setup_s": round(t_setup, 1),
            "round_trip_ok": ok,
        }
        if assemble:
            line["value_end_to_end"] = assemble.pop("value_end_to_end")
            line["exchange"] = assemble
    if rank == 0 and world == 1 and not args.no_sub and config3:
        subs = {}
        sub_steps, sub_warm = max(1, min(args.steps, 10)), min(args.warmup, 2)
        for w in SUB_WORKLOADS:
            codec.trim()
            subs[w] = sub_result(w, codec, dev, sub_steps, sub_warm, args.piece_bytes, not args.no_cpu_baseline)
            ok = ok and subs[w]["round_trip_ok"]
        codec.trim()
        subs["config0"] = config0_file_api()
        ok = ok and subs["config0"]["round_trip_ok"]
        line["configs"] = subs
        if not args.no_host_e2e:
            codec.trim()
            fa = host_file_api(args.file_api_bytes)
            line["host_file_api"] = fa
            ok = ok and fa["round_trip_ok"]
        line["round_trip_ok"] = ok
    if line is not None:
        print(json.dumps(line), flush=True)
    codec.close()
    if dcodec:
        dcodec.close()
    if use_dist:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


def end_to_end(job: Job, world: int, rank: int, args, cdev, gloo, allgather, total_in: int, meta) -> dict:
    """The whole job as one pipeline, timed over --e2e-steps runs (max over
    ranks).  The job is sharded block-cyclically (dist.piece_plan): step k
    handles global pieces k*world .. k*world+world-1, one per rank.  Per step:
      compress the rank's piece k (compute stream; returns its size),
      C1  all-gather of the step's sizes over a host-side gloo group (so it
          never queues behind the RCCL stream's C2),
      C2  on the comm stream: RCCL all-gather of the step's payloads, padded
          to the step's largest (RCCL has no all-gatherv), at most
          --c2-max-bytes per rank per collective, into a gather buffer; then
          each rank's part is copied to its offset in the reassembled stream
          (known from the sizes: the step's pieces are a contiguous run of it),
      decode of the rank's piece out of the stream (decode stream).
    C2 and the decode of step k run while step k+1 compresses.  The stream
    every rank ends with is byte-identical to a 1-GPU stream (SINGLE: one
    snappy_compress() stream; STREAMS: the streams in order).  Verified
    afterwards: the round trip and every global piece's checksum (its owner's
    payload against its run of every rank's stream)."""
    dev = job.dev
    unit, chunk, layout = job.unit, job.chunk, job.layout
    steps_k = job.steps_e2e
    comp_stream = torch.cuda.current_stream(dev)
    # the C2 stream at high priority (a hardware queue of its own, as RCCL's own
    # stream): the exchange never queues behind the compress of the next step
    comm = torch.cuda.Stream(dev, priority=-1)
    dstream = torch.cuda.Stream(dev)
    dcodec = snappy_amd.Codec(dev.index)
    dcodec.set_stream(dstream.cuda_stream)
    overlap = not args.no_e2e_overlap
    for gp in job.gpieces:
        if gp.offs is None:
            gp.offs = torch.empty(job.codec.num_units(gp.n, chunk, layout) + 1, dtype=torch.int64, device=dev)
    # the reassembled stream: every global piece at its worst-case bound
    g_all = [m for r in range(world) for _, _, m in piece_plan(total_in, world, r, unit, job.e2e_piece)]
    stream_cap = sum(job.codec.max_output(m, chunk, layout) for m in g_all) + 16
    stream = torch.empty(stream_cap, dtype=torch.uint8, device=dev)
    cmax = max(1, min(job.slot, args.c2_max_bytes))
    gbuf = torch.empty(world * cmax, dtype=torch.uint8, device=cdev)
    sizes_log = []

    def c1(clen: int):
        t = torch.tensor([clen], dtype=torch.int64)
        parts = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(parts, t, group=meta)
        return [int(v) for v in parts]

    statuses = []  # (verification run) each step's decode status

    def run(verify=False):
        base = 0
        sizes_log.clear()
        statuses.clear()
        for k in range(steps_k):
            gp = job.gpieces[k] if k < len(job.gpieces) else None
            clen = 0
            if gp is not None:
                gp.clen = clen = job.codec.compress_ptr_ex(job.x.data_ptr() + gp.xoff, gp.n, chunk, layout,
                                                           gp.flags, job.header_value,
                                                           job.out.data_ptr() + k * job.slot, gp.offs.data_ptr())
            sz = c1(clen)  # C1
            sizes_log.append(sz)
            comm.wait_stream(comp_stream)
            with torch.cuda.stream(comm):  # C2 (a rank without a piece this step sends slot 0's bytes)
                so = (k if gp is not None else 0) * job.slot
                c2_gather_step(job.out[so:so + job.slot], sz, stream, base, gbuf)
            if gp is not None:
                dstream.wait_stream(comm)
                dcodec.decompress_ptr_ex(stream.data_ptr() + base + int(sum(sz[:rank])), gp.offs.data_ptr(), gp.n,
                                         chunk, layout, gp.flags, job.header_value, job.back.data_ptr() + gp.xoff,
                                         check=False)
                if verify:  # (waits for this step's decode: the verification run only)
                    statuses.append(dcodec.decompress_status())
            if not overlap:
                torch.cuda.synchronize(dev)
            base += sum(sz)
        comp_stream.wait_stream(comm)
        comp_stream.wait_stream(dstream)
        torch.cuda.synchronize(dev)
        return base

    run()  # untimed: warms the communicators and the gather buffer
    dist.barrier()
    torch.cuda.synchronize(dev)
    runs = max(1, args.e2e_steps)
    t0 = time.perf_counter()
    for _ in range(runs):
        total_stream = run()
    torch.cuda.synchronize(dev)
    dist.barrier()
    tt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=cdev)
    torch_peak = torch.cuda.max_memory_allocated(dev)  # before the checks' temporaries
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    t = float(tt) / runs
    # verification: one more (untimed) run into a poisoned output, every step's
    # decode status read -- the timed runs' output cannot vouch for itself
    job.back.fill_(0xA5)
    torch.cuda.synchronize(dev)
    total_stream = run(verify=True)
    st = next((v for v in statuses if v != 0), 0)
    ok = st == 0 and len(statuses) == len(job.gpieces) and all(bool(torch.equal(job.back[o:min(o + GiB, job.n)], job.x[o:min(o + GiB, job.n)]))
                         for o in range(0, job.n, GiB))
    # every global piece: its owner's payload checksum against its run of this rank's stream
    mine = [checksum(job.out[gp.k * job.slot:gp.k * job.slot + gp.clen]) for gp in job.gpieces]
    mine += [0] * (steps_k - len(mine))
    sums = [torch.zeros(steps_k, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sums, torch.tensor(mine, dtype=torch.int64), group=meta)
    base = 0
    for k, sz in enumerate(sizes_log):
        for r in range(world):
            if sz[r]:
                ok &= checksum(stream[base:base + sz[r]]) == int(sums[r][k])
            base += sz[r]
    ok &= base == total_stream
    if args.e2e_dump and rank == 0:
        stream[:total_stream].cpu().numpy().tofile(args.e2e_dump)
    flag = torch.tensor([0.0 if ok else 1.0], dtype=torch.float64, device=cdev)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX)
    max_step = max(max(sz) for sz in sizes_log)
    res = {"value_end_to_end": round(total_in / t / 1e6, 1),
           "end_to_end_ms_per_step": round(t * 1e3, 3), "end_to_end_steps": runs,
           "end_to_end_step": "per pipeline step: compress the rank's piece, C1 size all-gather, C2 all-gather of the "
                              "step's payloads + copy into the reassembled stream, decode of the piece from the stream;"
                              + (" C2 and decode overlap the next step's compress" if overlap else " serialised (A/B)"),
           "sharding": f"block-cyclic, global pieces of {job.e2e_piece} B, {steps_k} pipeline steps per rank",
           "stream_bytes": int(total_stream), "c2_padded_bytes_per_rank_in": int(sum(world * max(sz) for sz in sizes_log)),
           "c2_largest_collective_bytes_per_rank": int(min(max_step, cmax)),
           "backend": "gloo" if gloo else "nccl (RCCL)", "verified": float(flag) == 0.0,
           "torch_peak_bytes": torch_peak}
    dcodec.close()
    del stream, gbuf
    torch.cuda.empty_cache()
    return res


def gather_decoded(job: Job, world: int, cdev, gloo, allgather) -> dict:
    """C3 (opt-in): every rank receives every rank's decoded shard (padded to
    the largest).  The codec scratch and the input are released first, so
    this phase fits HBM at 64 GiB (dist.rank_plan)."""
    dev = job.dev
    job.codec.trim()
    n, m = job.n, job.back.numel()
    mine = torch.tensor([checksum(job.back[:n]), n], dtype=torch.int64, device=cdev)
    info = torch.zeros(2 * world, dtype=torch.int64, device=cdev)
    allgather(info, mine)
    info = info.view(world, 2).cpu()
    full = torch.empty(world * m, dtype=torch.uint8, device=cdev)
    src = job.back if not gloo else job.back.to(cdev)
    allgather(full, src)  # warm-up
    torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    allgather(full, src)
    torch.cuda.synchronize(dev)
    dist.barrier()
    tt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=cdev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    good = all(checksum(full[r * m:r * m + int(info[r, 1])]) == int(info[r, 0]) for r in range(world))
    t = float(tt)
    return {"ms": round(t * 1e3, 3), "bytes_per_rank_out": world * m,
            "GBps_per_rank_in": round((world - 1) / world * world * m / t / 1e9, 2), "verified": bool(good)}


if __name__ == "__main__":
    main()
