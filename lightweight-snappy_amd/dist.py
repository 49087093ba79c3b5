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
    """Byte range [off, off+len) of rank's shard: contiguous, unit-aligned."""
    units = (n_total + unit - 1) // unit
    u0 = units * rank // world
    u1 = units * (rank + 1) // world
    off = u0 * unit
    return off, max(0, min(n_total, u1 * unit) - off)


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
