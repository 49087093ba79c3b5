"""CPU, world_size 2 over gloo: the sharded SINGLE-layout stream assembled
by dist.assemble is byte-identical to the whole-stream reference output (the
per-shard codec here is the oracle: the GPU path is exercised by bench.py's
multi-GPU run and by the gpu tests of the same shard flags)."""
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


@pytest.mark.parametrize("world,n", [(2, 5 * BLOCK + 123), (2, 4 * BLOCK), (3, 7 * BLOCK + 1)])
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
