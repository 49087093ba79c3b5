"""CPU: bench.py's job sizing and the per-rank device-memory plan of
configs[3] (64 GiB of 32 KiB text streams over 1/2/4/8 MI355X).
No GPU call: bench is imported for its pure functions only."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import dist as sdist  # noqa: E402
import snappy_amd  # noqa: E402

GiB = 1 << 30


def _sizes(a, world, rank):
    strong, total, gp, n, e2e, steps = bench.resolve_sizes(a, world, rank)
    return strong, total, n, e2e, steps, gp


def test_default_sizes():
    a = bench.parse([])
    # configs[3] at every N: the N = 1 point is the same 64 GiB job (one curve), in 1 GiB pieces
    assert _sizes(a, 1, 0)[:5] == (True, 64 * GiB, 64 * GiB, GiB, 64)
    a1 = bench.parse(["--bytes-per-gpu", str(GiB)])  # configs[1] alone
    assert _sizes(a1, 1, 0)[:3] == (False, GiB, GiB)
    a2 = bench.parse(["--workload", "text64k"])  # another workload alone at N = 1: 1 GiB
    assert _sizes(a2, 1, 0)[:3] == (False, GiB, GiB)
    assert _sizes(a2, 2, 1)[:2] == (True, 64 * GiB)
    for world in (2, 4, 8):  # configs[3]: 64 GiB strong-scaled, block-cyclic 1 GiB pieces
        strong, total, n, e2e, steps, gp = _sizes(a, world, world - 1)
        assert strong and total == 64 * GiB and n == 64 * GiB // world and e2e == GiB
        assert steps == 64 // world and [g for g, _, _ in gp] == list(range(world - 1, 64, world))
    a = bench.parse(["--weak"])
    strong, total, n, e2e, steps, gp = _sizes(a, 2, 1)
    assert (strong, total, n) == (False, 2 * GiB, GiB) and e2e * 2 * steps == total
    a = bench.parse(["--total-bytes", str(64 * GiB)])  # the N = 1 point of configs[3]
    assert _sizes(a, 1, 0)[:3] == (True, 64 * GiB, 64 * GiB)
    a = bench.parse(["--workload", "decode10g"])
    assert _sizes(a, 1, 0)[2] == bench.DECODE10G_BYTES


@pytest.mark.parametrize("total,world,unit", [(64 * GiB, 8, 32768), (200 * 65536 + 12345, 2, 65536),
                                              (5 * 65536, 8, 65536), (1, 3, 65536), (0, 2, 32768),
                                              (256 << 20, 8, 32768), (18_499_960_832, 1, 65536)])
def test_piece_plan_covers(total, world, unit):
    """Block-cyclic pieces: every byte once, unit-aligned, piece g on rank g
    mod world (rank 0 holds global offset 0), each pipeline step one piece
    per rank at most."""
    e2e = sdist.default_e2e_piece(total, world, unit)
    assert e2e % unit == 0 and e2e <= GiB
    plans = [sdist.piece_plan(total, world, r, unit, e2e) for r in range(world)]
    allp = sorted(x for p in plans for x in p)
    pos = 0
    for g, off, n in allp:
        assert off == pos and off % unit == 0 and n > 0
        pos += n
    assert pos == total
    for r, p in enumerate(plans):
        assert all(g % world == r for g, _, _ in p)
        assert len(p) <= sdist.pipeline_steps(total, world, unit, e2e)
    if total:
        assert plans[0][0][1] == 0
    # a share of whole units is split into equal pieces (weak scaling: equal shares)
    if total % (world * unit) == 0 and total:
        assert len({n for _, _, n in allp}) == 1 or e2e == sdist.piece_step(unit, min(GiB, total // world // 4))


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_rank_plan_fits_hbm(world):
    """Worst-case (incompressible) peak of one rank at 64 GiB, default pieces:
    under 288 GB at every N, C3 included when asked for."""
    a = bench.parse([])
    p = sdist.rank_plan(64 * GiB, world, 32768, a.piece_bytes, exchange=True, gather_decoded=True)
    assert p["peak"] < sdist.HBM_BYTES, p
    if world > 1:
        assert "c2_stream" in p and "c2_gather_buffer" in p and "c3_phase_peak" in p
        # the reassembled stream holds the whole job (worst case), the gather buffer one collective per rank
        assert p["c2_stream"] >= sdist.max_output(64 * GiB, 32768) and p["c2_gather_buffer"] <= world * (1 << 30)


def test_plan_matches_library_bounds():
    """The plan's payload bound is the library's own snappy_amd_max_output."""
    for n, unit in ((GiB, 32768), (8 * GiB + 12345, 65536), (1, 65536)):
        layout = snappy_amd.STREAMS if unit == 32768 else snappy_amd.SINGLE
        assert sdist.max_output(n, unit) == snappy_amd.Codec.max_output(n, unit, layout)
    assert sdist.pieces_of(20 * GiB + 5, 32768, 8 * GiB) == [8 * GiB, 8 * GiB, 4 * GiB + 5]


def test_e2e_piece_larger_than_job_is_the_job():
    # --e2e-piece-bytes above the job size: the piece (and so the payload slot
    # and the gather buffer) is the job rounded up to whole units, in both the
    # sizing bench.py allocates from and the plan it is checked against
    total = (256 << 20) + 12345
    a = bench.parse(["--total-bytes", str(total), "--e2e-piece-bytes", str(4 * GiB)])
    strong, tot, n, e2e, steps, gp = _sizes(a, 1, 0)
    assert e2e == ((total + 32767) // 32768) * 32768 and steps == 1
    big = sdist.rank_plan(total, 1, 32768, 8 * GiB, e2e_piece=4 * GiB)
    same = sdist.rank_plan(total, 1, 32768, 8 * GiB, e2e_piece=e2e)
    assert big == same
