"""Rebuild the inputs of tests/golden/golden.json from their closed-form
specs (no reference needed: datagen.c + tests/golden/license.bin)."""
import os

import datagen

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def make_input(spec: dict) -> bytes:
    kind = spec["kind"]
    n = spec["size"]
    if kind == "bytes":
        return bytes.fromhex(spec["hex"])
    if kind == "license":
        lic = open(os.path.join(GOLD, "license.bin"), "rb").read()
        return (lic * (n // len(lic) + 1))[:n]
    if kind == "iota64":
        return (bytes(range(64)) * (n // 64 + 1))[:n]
    if kind == "K":
        return datagen.make("K", n, spec["seed"], spec["period"]).tobytes()
    return datagen.make(kind, n, spec.get("seed", 0)).tobytes()
