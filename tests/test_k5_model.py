"""K5c's batch-parsed chain walk (k5_chain<MARK> in snappy_kernels.hip), as the
lane-level model in tools/k5_model.py, against the serial walk of the block
index on seeded foreign streams, a truncation and byte flips (CPU only)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import k5_model  # noqa: E402
from golden_inputs import build_stream, random_ops  # noqa: E402


def test_batch_walk_matches_serial_walk():
    rng = np.random.default_rng(3)
    outcomes = []
    for seed, n in ((101, 150_000), (102, 900_000)):
        s = build_stream(random_ops(seed, n, 131072))
        variants = [s, s[: len(s) - 777]]
        b = bytearray(s)
        for p in rng.integers(8, len(b), 2):
            b[p] ^= int(rng.integers(1, 255))
        variants.append(bytes(b))
        outcomes += [k5_model.check(v) for v in variants]
    assert outcomes[0] == k5_model.OK and outcomes[3] == k5_model.OK
