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


def test_default_sizes():
    a = bench.parse([])
    # configs[3] at every N: the N = 1 point is the same 64 GiB job (one curve)
    assert bench.resolve_sizes(a, 1, 0) == (True, 64 * GiB, 0, 64 * GiB, 64 * GiB)
    a1 = bench.parse(["--bytes-per-gpu", str(GiB)])  # configs[1] alone
    assert bench.resolve_sizes(a1, 1, 0) == (False, GiB, 0, GiB, GiB)
    a2 = bench.parse(["--workload", "text64k"])  # another workload alone at N = 1: 1 GiB
    assert bench.resolve_sizes(a2, 1, 0) == (False, GiB, 0, GiB, GiB)
    assert bench.resolve_sizes(a2, 2, 1)[:2] == (True, 64 * GiB)
    for world in (2, 4, 8):  # configs[3]: 64 GiB strong-scaled
        strong, total, off, n, n_max = bench.resolve_sizes(a, world, world - 1)
        assert strong and total == 64 * GiB and n == n_max == 64 * GiB // world
        assert off == (world - 1) * n
    a = bench.parse(["--weak"])
    assert bench.resolve_sizes(a, 2, 1) == (False, 2 * GiB, GiB, GiB, GiB)
    a = bench.parse(["--total-bytes", str(64 * GiB)])  # the N = 1 point of configs[3]
    assert bench.resolve_sizes(a, 1, 0) == (True, 64 * GiB, 0, 64 * GiB, 64 * GiB)
    a = bench.parse(["--workload", "decode10g"])
    assert bench.resolve_sizes(a, 1, 0)[3] == bench.DECODE10G_BYTES


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_rank_plan_fits_hbm(world):
    """Worst-case (incompressible) peak of one rank at 64 GiB, default pieces:
    under 288 GB at every N, C3 included when asked for."""
    a = bench.parse([])
    p = sdist.rank_plan(64 * GiB, world, 32768, a.piece_bytes, exchange=True, gather_decoded=True)
    assert p["peak"] < sdist.HBM_BYTES, p
    if world > 1:
        assert "c2_gather_buffer" in p and "c3_phase_peak" in p


def test_plan_matches_library_bounds():
    """The plan's payload bound is the library's own snappy_amd_max_output."""
    for n, unit in ((GiB, 32768), (8 * GiB + 12345, 65536), (1, 65536)):
        layout = snappy_amd.STREAMS if unit == 32768 else snappy_amd.SINGLE
        assert sdist.max_output(n, unit) == snappy_amd.Codec.max_output(n, unit, layout)
    assert sdist.pieces_of(20 * GiB + 5, 32768, 8 * GiB) == [8 * GiB, 8 * GiB, 4 * GiB + 5]
