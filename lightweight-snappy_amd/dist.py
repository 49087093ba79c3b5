"""Multi-GPU sharding of the codec.

Units (65,536-byte blocks of one stream, or independent 32 KiB streams) are
independent, so ranks own contiguous unit ranges and compress/decompress
them with no data-path collective.  The exchange steps that exist are:
  C1  all-gather of the per-shard compressed sizes -> each shard's offset in
      the global stream / global block index (8 bytes per rank);
  C2  (optional) all-gather of the shards to reassemble the whole stream on
      every rank (RCCL over xGMI on GPUs; gloo in the CPU tests).
A SINGLE-layout stream sharded this way is byte-identical to the 1-GPU
stream: rank 0 writes the varint preamble of the global length, the other
ranks compress with SNAPPY_AMD_NO_PREAMBLE, and every shard boundary is a
multiple of 65,536 input bytes (src/snappy_compression.c:419-425 blocks).
"""
from __future__ import annotations

from typing import List, Tuple

import torch
import torch.distributed as dist


def shard_range(n_total: int, world: int, rank: int, unit: int) -> Tuple[int, int]:
    """Byte range [off, off+len) of rank's shard: contiguous, unit-aligned.
    Rounded up, so rank 0 (which writes a SINGLE stream's preamble) always
    owns the first unit when there is one; with fewer units than ranks the
    empty shards are later ranks'."""
    units = (n_total + unit - 1) // unit
    u0 = -(-units * rank // world)
    u1 = -(-units * (rank + 1) // world)
    off = u0 * unit
    return off, max(0, min(n_total, u1 * unit) - off)


BLOCK = 65536
GiB = 1 << 30
HBM_BYTES = 288 * 10**9  # MI355X HBM3E, 288 GB (MI355X_MICROARCH.md; the spec figure, the smaller reading)
K2_SEG = 256              # csrc/snappy_kernels.h SNAPPY_K2_SEG
COMPACT_BOUNCE = 256 << 20  # bench.py's in-place compaction of the C2 gather stages pieces of this size


def max_output(n: int, unit: int) -> int:
    """snappy_amd_max_output (csrc/snappy_device.hip): worst-case payload bytes."""
    units = (n + unit - 1) // unit
    return n + units * (unit // 32 + 32) + 16


def _grown(need: int) -> int:
    """Bytes grow() in csrc/snappy_device.hip allocates for `need`."""
    return need + min(need // 8, 64 << 20) + 4096


def pieces_of(n: int, unit: int, piece_bytes: int) -> List[int]:
    """Sizes of the unit-aligned pieces bench.py compresses a rank's range in."""
    step = max(unit, (piece_bytes // unit) * unit)
    return [min(step, n - o) for o in range(0, n, step)]


def rank_plan(total: int, world: int, unit: int, piece_bytes: int, exchange: bool = True,
              gather_decoded: bool = False) -> dict:
    """Peak device bytes of one bench.py rank (the largest shard) for a job of
    `total` input bytes sharded over `world` ranks, worst case (incompressible
    data: every payload at its snappy_amd_max_output bound).

    Resident through the run: the shard (x), its payload (out, sized for the
    largest shard so the C2 all-gather can send equal counts), the decoded
    shard (back), the per-piece block indexes and the codec's scratch for the
    largest piece (K1r token lists + escapes, token counts, unit sizes, K2
    segment records, K4 status words).  With `exchange` (world > 1): C2's
    padded all-gather buffer (world x payload), compacted in place into the
    reassembled stream through a 256 MiB staging buffer.
    `gather_decoded` (C3, opt-in) runs after the codec scratch and C2 buffers
    are released: every rank then also holds world x the largest shard."""
    shard = max(shard_range(total, world, r, unit)[1] for r in range(world))
    ps = pieces_of(shard, unit, piece_bytes)
    big = max(ps) if ps else 0
    units_big = (big + unit - 1) // unit
    tok_cap = unit // 4 + 2
    segs = (tok_cap + K2_SEG - 1) // K2_SEG
    out_cap = sum(max_output(p, unit) for p in ps)
    plan = {
        "shard_x": shard,
        "payload_out": out_cap,
        "decoded_back": shard,
        "block_indexes": sum(((p + unit - 1) // unit + 1) * 8 for p in ps),
        "scratch_tokens": _grown(units_big * tok_cap * 8 + units_big * 32),
        "scratch_counts_sizes": 2 * _grown(units_big * 4),
        "scratch_segments": _grown(units_big * segs * 8),
        "scratch_status": _grown((units_big + 2) * 4),
    }
    if exchange and world > 1:
        plan["c2_gather_buffer"] = world * out_cap
        plan["c2_compaction_bounce"] = COMPACT_BOUNCE
    plan["peak"] = sum(plan.values())
    if gather_decoded and world > 1:
        c3 = plan["shard_x"] + plan["payload_out"] + plan["decoded_back"] + plan["block_indexes"] + world * shard
        plan["c3_phase_peak"] = c3
        plan["peak"] = max(plan["peak"], c3)
    return plan


def exchange_sizes(local_size: int, device, group=None) -> List[int]:
    """C1: every rank learns every shard's compressed size."""
    world = dist.get_world_size(group)
    mine = torch.tensor([local_size], dtype=torch.int64, device=device)
    allv = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(allv, mine, group=group)
    return [int(v.item()) for v in allv]


def assemble(payload: torch.Tensor, offsets: torch.Tensor, group=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """C2: gather every shard's compressed bytes and unit index.

    payload: this rank's compressed bytes (uint8); offsets: its unit index
    (int64, units+1 entries, starting at 0).  Returns (stream, index) for the
    whole job, identical on every rank; index entries are global byte offsets.
    """
    dev = payload.device
    world = dist.get_world_size(group)
    sizes = exchange_sizes(payload.numel(), dev, group)
    nunits = exchange_sizes(offsets.numel() - 1, dev, group)
    mx = max(max(sizes), 1)
    mu = max(nunits) + 1
    pad = torch.zeros(mx, dtype=torch.uint8, device=dev)
    pad[: payload.numel()] = payload
    pado = torch.zeros(mu, dtype=torch.int64, device=dev)
    pado[: offsets.numel()] = offsets
    bufs = [torch.empty(mx, dtype=torch.uint8, device=dev) for _ in range(world)]
    obufs = [torch.empty(mu, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    dist.all_gather(obufs, pado, group=group)
    parts, idx, base = [], [], 0
    for r in range(world):
        parts.append(bufs[r][: sizes[r]])
        idx.append(obufs[r][: nunits[r]] + base)
        base += sizes[r]
    idx.append(torch.tensor([base], dtype=torch.int64, device=dev))
    return torch.cat(parts), torch.cat(idx)
