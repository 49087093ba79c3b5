"""World size 2-3 over gloo.  CPU: the sharded SINGLE-layout stream assembled
by dist.assemble is byte-identical to the whole-stream reference output with
the oracle as the per-shard codec.  GPU (ranks sharing cuda:0): the same
with the HIP shard path, and bench.py's own rank spawning, C2/C3 exchange
and strong-scaling pieces."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import datagen
import oracle

BLOCK = 65536


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def shard_compress(a: np.ndarray, header_value, first: bool) -> tuple:
    """Oracle stand-in for snappy_amd_compress_device_ex on one shard."""
    out = bytearray()
    offs = [0]
    if first:
        buf = ctypes.create_string_buffer(16)
        k = oracle.orc().oracle_varint_encode(header_value, buf)
        out += buf.raw[:k]
    tmp = np.empty(BLOCK + BLOCK // 32 + 64, dtype=np.uint8)
    for b in range(0, a.size, BLOCK):
        blk = np.ascontiguousarray(a[b:b + BLOCK])
        m = oracle.orc().oracle_compress_block(blk.ctypes.data_as(ctypes.c_void_p), blk.size,
                                               tmp.ctypes.data_as(ctypes.c_void_p))
        out += tmp[:m].tobytes()
        offs.append(len(out))
    return bytes(out), offs


def _worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import dist as sdist
        a = datagen.make("T", n, 77)
        off, ln = sdist.shard_range(n, world, rank, BLOCK)
        payload, offs = shard_compress(a[off:off + ln], n, rank == 0)
        pt = torch.frombuffer(bytearray(payload), dtype=torch.uint8) if payload else torch.zeros(0, dtype=torch.uint8)
        stream, index = sdist.assemble(pt, torch.tensor(offs, dtype=torch.int64))
        sizes = sdist.exchange_sizes(len(payload), torch.device("cpu"))
        want = oracle.compress(a.tobytes())
        ok = stream.numpy().tobytes() == want and sum(sizes) == len(want)
        # the global index splits the stream at every 65,536-byte block
        idx = index.numpy()
        ok = ok and idx[0] == 0 and idx[-1] == len(want) and np.all(np.diff(idx) > 0)
        q.put((rank, ok, len(idx)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 5 * BLOCK + 123), (2, 4 * BLOCK), (3, 7 * BLOCK + 1),
                                     (8, 21 * BLOCK + 77), (8, 5 * BLOCK)])
def test_sharded_stream_identical(world, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(60)
    assert all(ok for _, ok, _ in res), res
    units = (n + BLOCK - 1) // BLOCK
    assert all(k == units + 1 for _, _, k in res)


def _pipeline_worker(rank, world, port, n, piece, cmax, q):
    """One rank of bench.py's end-to-end pipeline on the CPU: block-cyclic
    pieces (dist.piece_plan) compressed by the oracle stand-in, per step C1
    (sizes) and C2 (dist.c2_gather_step over gloo, host buffers) into the
    stream every rank holds."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import dist as sdist
        a = datagen.make("T", n, 79)
        mine = sdist.piece_plan(n, world, rank, BLOCK, piece)
        steps = sdist.pipeline_steps(n, world, BLOCK, piece)
        slot = sdist.max_output(piece, BLOCK)
        stream = torch.zeros(sum(sdist.max_output(m, BLOCK) for r in range(world)
                                 for _, _, m in sdist.piece_plan(n, world, r, BLOCK, piece)) + 16, dtype=torch.uint8)
        gbuf = torch.empty(world * cmax, dtype=torch.uint8)
        base = 0
        for k in range(steps):
            src = torch.full((slot,), 0xAB, dtype=torch.uint8)  # padding a gather must never place
            clen = 0
            if k < len(mine):
                g, off, m = mine[k]
                payload, _ = shard_compress(a[off:off + m], n, off == 0)
                clen = len(payload)
                src[:clen] = torch.frombuffer(bytearray(payload), dtype=torch.uint8)
            sizes = sdist.exchange_sizes(clen, torch.device("cpu"))
            sdist.c2_gather_step(src, sizes, stream, base, gbuf)
            base += sum(sizes)
        q.put((rank, stream[:base].numpy().tobytes() == oracle.compress(a.tobytes())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,piece,cmax", [(2, 9 * BLOCK + 77, 2 * BLOCK, 1 << 20),
                                                (3, 20 * BLOCK, 2 * BLOCK, 5000),
                                                (8, 21 * BLOCK + 77, BLOCK, 30000),
                                                (4, 3 * BLOCK, 2 * BLOCK, 1 << 20)])
def test_pipelined_c2_stream_identical(world, n, piece, cmax):
    """bench.py's pipelined C2 (block-cyclic pieces, one all-gather per step,
    split into collectives of at most cmax bytes per rank, ranks without a
    piece in the last step) reassembles exactly the whole-input reference
    stream on every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipeline_worker, args=(r, world, port, n, piece, cmax, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(60)
    assert all(ok for _, ok in res), res


def test_shard_range_covers():
    import dist as sdist
    for n in (0, 1, BLOCK, 10 * BLOCK + 5, 123456789):
        for world in (1, 2, 3, 8):
            spans = [sdist.shard_range(n, world, r, BLOCK) for r in range(world)]
            pos = 0
            for off, ln in spans:
                assert off == pos or ln == 0
                assert off % BLOCK == 0
                pos = off + ln if ln else pos
            assert sum(ln for _, ln in spans) == n


def _gpu_worker(rank, world, port, n, layout, chunk, q):
    """One rank of the HIP shard path: ranks share cuda:0, collectives over gloo."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import dist as sdist
        import snappy_amd
        torch.cuda.set_device(0)
        codec = snappy_amd.Codec(0)
        a = datagen.make("T", n, 78)
        unit = BLOCK if layout == snappy_amd.SINGLE else chunk
        off, ln = sdist.shard_range(n, world, rank, unit)
        x = torch.from_numpy(a[off:off + ln].copy()).cuda()
        flags = snappy_amd.NO_PREAMBLE if (layout == snappy_amd.SINGLE and off > 0) else 0
        hv = n if layout == snappy_amd.SINGLE else ln
        units = codec.num_units(ln, chunk, layout)
        out = torch.empty(max(codec.max_output(ln, chunk, layout), 16), dtype=torch.uint8, device="cuda")
        offs = torch.empty(units + 1, dtype=torch.int64, device="cuda")
        clen = codec.compress_ptr_ex(x.data_ptr(), ln, chunk, layout, flags, hv, out.data_ptr(), offs.data_ptr())
        # C2 over gloo: the whole stream and its global index on every rank
        stream, index = sdist.assemble(out[:clen].cpu(), offs.cpu())
        # each rank decodes its own blocks from the assembled stream (shard of the global index)
        u0 = off // unit
        mine = index[u0:u0 + units + 1].cuda() - int(index[u0])
        sub = stream[int(index[u0]):int(index[u0 + units])].cuda()
        back = torch.empty(max(ln, 1), dtype=torch.uint8, device="cuda")
        codec.decompress_ptr_ex(sub.data_ptr(), mine.data_ptr(), ln, chunk, layout, flags, hv, back.data_ptr())
        ok_dec = bool(torch.equal(back[:ln], x))
        if layout == snappy_amd.SINGLE:
            want = oracle.compress(a.tobytes())
        else:
            want = oracle.compress_streams(a, chunk)[0].tobytes()
        q.put((rank, stream.numpy().tobytes() == want, ok_dec, len(index)))
        codec.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world,n,layout,chunk", [(2, 300 * BLOCK + 4567, 0, BLOCK), (2, 9 << 20, 1, 32768),
                                                  (3, 50 * BLOCK, 0, BLOCK)])
def test_gpu_sharded_stream_identical(world, n, layout, chunk):
    """The HIP shard path (snappy_amd_compress_device_ex with NO_PREAMBLE on
    ranks > 0), world 2-3 on one GPU: the assembled stream is byte-identical
    to the 1-rank stream (== the reference's), and every rank decodes its
    blocks from it."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, n, layout, chunk, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(60)
    assert all(same and dec for _, same, dec, _ in res), res


def _bench(*args):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), *args], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, "\n".join(l for l in r.stderr.splitlines() if l.startswith("[rank"))[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.gpu
def test_bench_spawns_ranks_weak():
    """bench.py --gpus 2 --weak (no launcher): spawns two ranks (gloo rehearsal
    on one GPU), prints one line with n_gpus 2; the end-to-end loop (compress,
    C1, C2, compaction, decode from the stream) and C3 are timed and verified."""
    d = _bench("--gpus", "2", "--weak", "--dist-backend", "gloo", "--bytes-per-gpu", str(64 << 20), "--steps", "2",
               "--warmup", "1", "--no-host-e2e", "--c3")
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["round_trip_ok"]
    assert d["exchange"]["verified"] and d["value_end_to_end"] > 0
    assert d["exchange"]["c3_decoded_allgather"]["verified"]
    assert d["config"]["total_bytes"] == 2 * (64 << 20)


@pytest.mark.gpu
def test_bench_strong_pieces(tmp_path):
    """--total-bytes fixes the job (strong scaling); --piece-bytes splits a
    rank's pieces into several compress calls, SINGLE layout (one stream).
    The end-to-end pipeline (block-cyclic pieces of 25 blocks, 5 steps, the
    last with one rank idle) reassembles exactly the reference's stream of
    the whole input on rank 0."""
    total = 100 * BLOCK * 2 + 12345
    dump = str(tmp_path / "stream.snp")
    d = _bench("--gpus", "2", "--dist-backend", "gloo", "--workload", "text64k", "--total-bytes",
               str(total), "--piece-bytes", str(40 * BLOCK), "--steps", "2", "--warmup", "1",
               "--no-host-e2e", "--e2e-dump", dump)
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["round_trip_ok"]
    assert d["config"]["pieces_per_gpu"] == 3 and d["exchange"]["verified"]
    got = open(dump, "rb").read()
    assert d["exchange"]["stream_bytes"] == len(got)
    assert got == oracle.compress(datagen.make("T", total, 1234).tobytes())


@pytest.mark.gpu
def test_bench_rccl_world1_large_collective(tmp_path):
    """RCCL at configs[3]'s real counts: a 1-rank communicator whose C2 sends
    one all-gather of more than 2^32 bytes (5 GiB of random bytes in one
    piece, payload ~5.4 GB, --c2-max-bytes above it).  The reassembled
    stream's checksums and the round trip are verified by bench.py."""
    n = 5 << 30
    d = _bench("--dist-world1", "--dist-backend", "nccl", "--workload", "random", "--bytes-per-gpu", str(n),
               "--e2e-piece-bytes", str(n), "--c2-max-bytes", str(8 << 30), "--steps", "1", "--warmup", "0",
               "--e2e-steps", "1", "--no-host-e2e", "--no-cpu-baseline", "--no-sub")
    ex = d["exchange"]
    assert d["round_trip_ok"] and ex["verified"] and ex["backend"].startswith("nccl")
    assert ex["c2_largest_collective_bytes_per_rank"] > 1 << 32
    assert ex["stream_bytes"] > n  # random bytes: every block stored as literals


@pytest.mark.gpu
def test_bench_gloo_world2_large_payload():
    """gloo world 2 (ranks sharing the GPU) with a per-rank payload above
    2^32 bytes sent as one collective: 9 GiB of random bytes, one 4.5 GiB
    piece per rank (payload ~4.8 GB each).  Shard checksums and the round
    trip are verified on both ranks."""
    d = _bench("--gpus", "2", "--dist-backend", "gloo", "--workload", "random", "--total-bytes", str(9 << 30),
               "--e2e-piece-bytes", str(9 << 29), "--c2-max-bytes", str(8 << 30), "--steps", "1", "--warmup", "0",
               "--e2e-steps", "1", "--no-host-e2e")
    ex = d["exchange"]
    assert d["round_trip_ok"] and ex["verified"]
    assert ex["c2_largest_collective_bytes_per_rank"] > 1 << 32


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_bench_memory_within_plan(world):
    """Per-rank device memory of a scaled strong-scaling run (gloo ranks on one
    GPU, text32k, pieces of 64 MiB) stays within dist.rank_plan for that size
    -- the plan that DESIGN.md 6 extrapolates to 64 GiB at N = 1/2/4/8 (the
    CPU test test_rank_plan_fits_hbm checks those fit 288 GB).  The measured
    peak is the torch allocator's peak (shard, payload, decoded output, block
    indexes, the C2 gather buffer and stream) plus the library's scratch."""
    total = 384 << 20
    d = _bench("--gpus", str(world), "--dist-backend", "gloo", "--total-bytes", str(total), "--piece-bytes",
               str(64 << 20), "--steps", "1", "--warmup", "1", "--no-host-e2e")
    m = d["memory"]
    assert d["round_trip_ok"] and d["exchange"]["verified"]
    assert 0 < m["rank_peak_bytes"] <= m["planned_peak_bytes_per_rank"], m
    # the plan is a worst-case bound, not a vacuous one: text uses a good part of it
    assert m["rank_peak_bytes"] >= 0.3 * m["planned_peak_bytes_per_rank"], m


@pytest.mark.gpu
def test_bench_world8_rehearsal():
    """configs[3]'s 8-rank path on the one GPU of a box: bench.py --gpus 8
    spawns 8 ranks (torch.distributed.run, gloo collectives, all ranks on
    cuda:0) of a 256 MiB strong-scaled job (block-cyclic 8 MiB pieces, four
    pipeline steps per rank, compress launches of 16 MiB) -- C1 in every
    step, the overlapped end-to-end pipeline (C2 per step into the stream,
    decode from it), per-piece checksums and the round trip verified on
    every rank, and every rank's measured peak within dist.rank_plan."""
    total = 256 << 20
    d = _bench("--gpus", "8", "--dist-backend", "gloo", "--total-bytes", str(total), "--piece-bytes", str(16 << 20),
               "--steps", "1", "--warmup", "1", "--no-host-e2e")
    assert d["n_gpus"] == 8 and d["scaling"] == "strong" and d["round_trip_ok"]
    assert d["config"]["total_bytes"] == total and d["config"]["bytes_per_gpu"] == total // 8
    assert d["config"]["pieces_per_gpu"] == 2
    assert d["exchange"]["verified"] and d["value_end_to_end"] > 0
    assert "4 pipeline steps" in d["exchange"]["sharding"]
    m = d["memory"]
    assert 0 < m["rank_peak_bytes"] <= m["planned_peak_bytes_per_rank"], m


@pytest.mark.gpu
def test_bench_rccl_world1():
    """The RCCL (nccl backend) exchange code path on the one GPU a box has:
    a 1-rank communicator runs C1 in every step and the end-to-end loop's C2
    all-gather + compaction + decode from the reassembled stream."""
    d = _bench("--dist-world1", "--dist-backend", "nccl", "--bytes-per-gpu", str(256 << 20), "--steps", "2",
               "--warmup", "1", "--no-host-e2e", "--no-cpu-baseline", "--no-sub")
    assert d["round_trip_ok"] and d["exchange"]["verified"] and d["exchange"]["backend"].startswith("nccl")
    assert d["value_end_to_end"] > 0
