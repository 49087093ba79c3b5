"""Multi-GPU sharding of the codec.

Units (65,536-byte blocks of one stream, or independent 32 KiB streams) are
independent, so ranks own contiguous unit ranges and compress/decompress
them with no data-path collective.  The exchange steps that exist are:
  C1  all-gather of the per-shard compressed sizes -> each shard's offset in
      the global stream / global block index (8 bytes per rank);
  C2  (optional) all-gather of the shards to reassemble the whole stream on
      every rank (RCCL over xGMI on GPUs; gloo in the CPU tests).  bench.py
      shards block-cyclically (piece_plan) and runs C2 per pipeline step,
      overlapped with the next step's compression.
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
    """Byte range [off, off+len) of rank's shard: contiguous, unit-aligned
    (the split snappy_*_buffer_multi and the oracle shard tests use).
    Rounded up, so rank 0 (which writes a SINGLE stream's preamble) always
    owns the first unit when there is one.  With fewer units than ranks the
    empty shards can fall at any rank except 0 (units=5, world=8: ranks 2, 5
    and 7 are empty)."""
    units = (n_total + unit - 1) // unit
    u0 = -(-units * rank // world)
    u1 = -(-units * (rank + 1) // world)
    off = u0 * unit
    return off, max(0, min(n_total, u1 * unit) - off)


def piece_step(unit: int, piece_bytes: int) -> int:
    """Bytes of one global piece: piece_bytes rounded down to whole units."""
    return max(unit, (piece_bytes // unit) * unit)


def global_pieces(n_total: int, unit: int, piece_bytes: int) -> int:
    """Number of global pieces the job is cut into."""
    step = piece_step(unit, piece_bytes)
    return (n_total + step - 1) // step


def piece_plan(n_total: int, world: int, rank: int, unit: int, piece_bytes: int) -> List[Tuple[int, int, int]]:
    """Block-cyclic sharding of bench.py's job: the input is cut into global
    pieces of piece_step() bytes (the last one shorter) and global piece g
    belongs to rank g mod world.  Returns this rank's pieces as (g, global
    offset, bytes), ascending.  Pipeline step k of the end-to-end loop handles
    global pieces k*world .. k*world+world-1, one per rank, so after step k's
    all-gather every rank holds a contiguous run of the stream and its offset
    is known from the sizes alone (no compaction of the whole stream at the
    end).  Rank 0 owns piece 0 (the SINGLE preamble); with world = 1 this is
    the contiguous range."""
    step = piece_step(unit, piece_bytes)
    g_n = global_pieces(n_total, unit, piece_bytes)
    return [(g, g * step, min(step, n_total - g * step)) for g in range(rank, g_n, world)]


def pipeline_steps(n_total: int, world: int, unit: int, piece_bytes: int) -> int:
    """Steps of the end-to-end pipeline: ceil(global pieces / world)."""
    return (global_pieces(n_total, unit, piece_bytes) + world - 1) // world


def default_e2e_piece(n_total: int, world: int, unit: int, cap: int = 1 << 30) -> int:
    """The end-to-end pipeline's piece: a quarter of a rank's share (at least
    four steps to overlap), at most `cap` (1 GiB: 8 steps per rank for
    configs[3] at N = 8), whole units.  When the share is whole units, the
    piece divides it where a divisor lies within 2x of the target (the
    smallest such piece count), so every rank gets exactly its share (weak
    scaling) and the pieces are equal."""
    share = -(-n_total // max(world, 1))
    target = piece_step(unit, min(cap, max(unit, share // 4)))
    if share % unit == 0 and share > 0:
        units = share // unit
        k0 = -(-units // (target // unit))
        for k in range(k0, 2 * k0 + 1):  # (no divisor near the target: the target, last piece short)
            if units % k == 0:
                return (units // k) * unit
    return target


BLOCK = 65536
GiB = 1 << 30
HBM_BYTES = 288 * 10**9  # MI355X HBM3E, 288 GB (MI355X_MICROARCH.md; the spec figure, the smaller reading)
K2_SEG = 256              # csrc/snappy_kernels.h SNAPPY_K2_SEG


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


C2_MAX_BYTES = 1 << 30   # bench.py: one C2 all-gather sends at most this many bytes per rank


def rank_plan(total: int, world: int, unit: int, piece_bytes: int, exchange: bool = True,
              gather_decoded: bool = False, e2e_piece: int = 0, c2_max: int = C2_MAX_BYTES) -> dict:
    """Peak device bytes of one bench.py rank (the largest shard) for a job of
    `total` input bytes sharded block-cyclically (piece_plan, pieces of
    `e2e_piece`, default default_e2e_piece) over `world` ranks, worst case
    (incompressible data: every payload at its snappy_amd_max_output bound).

    Resident through the run: the shard (x, the rank's pieces back to back),
    its payload (out: the timed loop's launches of <= piece_bytes packed, or
    the end-to-end loop's one slot per pipeline step, whichever is larger),
    the decoded shard (back), the block indexes and the codec's scratch for
    the largest launch (K1r token lists + escapes, token counts, unit sizes,
    K2 segment records, K4 status words).  With `exchange` (world > 1): the
    reassembled stream (every global piece at its bound) and the C2 gather
    buffer (world x one all-gather's count, at most c2_max per rank).
    `gather_decoded` (C3, opt-in) runs after the codec scratch and C2 buffers
    are released: every rank then also holds world x the largest shard."""
    e2e = piece_step(unit, e2e_piece or default_e2e_piece(total, world, unit))
    e2e = min(e2e, piece_step(unit, total + unit - 1))  # (as bench.resolve_sizes: at most the job)
    shard = max(sum(n for _, _, n in piece_plan(total, world, r, unit, e2e)) for r in range(world))
    ps = pieces_of(shard, unit, piece_bytes)
    big = max(ps + [min(e2e, total)]) if ps else 0
    units_big = (big + unit - 1) // unit
    tok_cap = unit // 4 + 2
    segs = (tok_cap + K2_SEG - 1) // K2_SEG
    steps = pipeline_steps(total, world, unit, e2e)
    slot = max_output(min(e2e, max(total, 1)), unit)
    out_cap = max(sum(max_output(p, unit) for p in ps), steps * slot)
    own = piece_plan(total, world, 0, unit, e2e)
    plan = {
        "shard_x": shard,
        "payload_out": out_cap,
        "decoded_back": shard,
        "block_indexes": sum(((p + unit - 1) // unit + 1) * 8 for p in ps) +
                         sum(((n + unit - 1) // unit + 1) * 8 for _, _, n in own),
        "scratch_tokens": _grown(units_big * tok_cap * 8 + units_big * 32),
        "scratch_counts_sizes": 2 * _grown(units_big * 4),
        "scratch_segments": _grown(units_big * segs * 8),
        "scratch_status": 2 * _grown((units_big + 2) * 4),
    }
    if exchange and world > 1:
        plan["c2_stream"] = sum(max_output(n, unit) for _, _, n in
                                (x for r in range(world) for x in piece_plan(total, world, r, unit, e2e)))
        plan["c2_gather_buffer"] = world * min(slot, c2_max)
    plan["peak"] = sum(plan.values())
    if gather_decoded and world > 1:
        c3 = plan["shard_x"] + plan["payload_out"] + plan["decoded_back"] + plan["block_indexes"] + world * shard
        plan["c3_phase_peak"] = c3
        plan["peak"] = max(plan["peak"], c3)
    return plan


def c2_gather_step(src: torch.Tensor, sizes: List[int], stream: torch.Tensor, base: int, gbuf: torch.Tensor,
                   group=None) -> None:
    """C2 of one pipeline step (bench.py's end-to-end loop).  Every rank
    contributes the first max(sizes) bytes of `src` (its piece's payload slot,
    at least that long; a rank without a piece this step sends any bytes,
    sizes[rank] = 0); rank r's sizes[r] bytes land at stream[base +
    sum(sizes[:r]):] on every rank -- the step's pieces are consecutive
    global pieces, so they form one contiguous run of the stream.  The gather
    goes through `gbuf` (world x at most gbuf.numel() // world bytes per rank
    per collective, so no single collective's count exceeds that), on the
    caller's current stream: RCCL all_gather_into_tensor when gbuf is on the
    GPU, a gloo all_gather when it is in host memory (then the copies into
    the stream are blocking, since the next chunk reuses gbuf)."""
    world = dist.get_world_size(group)
    cmax = gbuf.numel() // world
    assert cmax > 0 and src.numel() >= max(sizes)
    host = gbuf.device.type == "cpu"
    mx = max(sizes)
    pre = [0]
    for v in sizes:
        pre.append(pre[-1] + v)
    for c0 in range(0, mx, cmax):
        m = min(cmax, mx - c0)
        piece = src[c0:c0 + m]
        if host:
            dist.all_gather(list(gbuf[:world * m].chunk(world)), piece.cpu(), group=group)
        else:
            dist.all_gather_into_tensor(gbuf[:world * m], piece, group=group)
        for r in range(world):
            a = min(m, sizes[r] - c0)
            if a > 0:
                d = base + pre[r] + c0
                stream[d:d + a].copy_(gbuf[r * m:r * m + a], non_blocking=not host)


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
