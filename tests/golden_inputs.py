"""Rebuild the inputs of tests/golden/golden.json from their closed-form
specs (no reference needed: datagen.c + tests/golden/license.bin), and build
raw Snappy streams element by element (decoder vectors the reference
compressor never writes: copies into earlier 65,536-byte blocks, elements
straddling block boundaries, copy-4, wide literal headers)."""
import os

import datagen

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BLOCK = 65536


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


# ---- raw element encoders (format of src/snappy_decompression.c:290-333) ----
def varint(n: int) -> bytes:
    out = bytearray()
    while n >= 128:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def enc_literal(data: bytes, width: int = -1) -> bytes:
    """Literal element; width = extra length bytes (0 = length in the tag),
    -1 = the smallest that fits."""
    m = len(data) - 1
    assert m >= 0
    if width < 0:
        width = 0 if m < 60 else (1 if m < 1 << 8 else 2 if m < 1 << 16 else 3 if m < 1 << 24 else 4)
    if width == 0:
        assert m < 60
        return bytes([m << 2]) + data
    assert m < 1 << (8 * width)
    return bytes([(59 + width) << 2]) + m.to_bytes(width, "little") + data


def enc_copy(length: int, off: int, kind: int) -> bytes:
    """kind 1: copy-1 (len 4..11, off < 2048); 2: copy-2 (len 1..64, off < 65536);
    4: copy-4 (len 1..64, off < 2^32)."""
    if kind == 1:
        assert 4 <= length <= 11 and 0 <= off < 2048
        return bytes([((off >> 8) << 5) | ((length - 4) << 2) | 1, off & 0xFF])
    assert 1 <= length <= 64
    if kind == 2:
        assert 0 <= off < 1 << 16
        return bytes([((length - 1) << 2) | 2]) + off.to_bytes(2, "little")
    assert 0 <= off < 1 << 32
    return bytes([((length - 1) << 2) | 3]) + off.to_bytes(4, "little")


def uncompressed_length(stream: bytes) -> int:
    v, sh = 0, 0
    for b in stream[:10]:
        v |= (b & 0x7F) << sh
        sh += 7
        if not b & 0x80:
            return v
    raise ValueError("bad varint")


def build_stream(ops) -> bytes:
    """ops: ["lit", n, seed(, width)] (n random bytes of datagen R/seed) or
    ["copy", length, offset, kind]; the preamble is varint(total output)."""
    body, total = bytearray(), 0
    for op in ops:
        if op[0] == "lit":
            width = op[3] if len(op) > 3 else -1
            body += enc_literal(datagen.make("R", op[1], op[2]).tobytes(), width)
            total += op[1]
        else:
            body += enc_copy(op[1], op[2], op[3])
            total += op[1]
    return varint(total) + bytes(body)


class SplitMix64:
    def __init__(self, seed: int):
        self.s = seed & (2**64 - 1)

    def next(self) -> int:
        self.s = (self.s + 0x9E3779B97F4A7C15) & (2**64 - 1)
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
        return z ^ (z >> 31)

    def below(self, n: int) -> int:
        return self.next() % n


def random_ops(seed: int, n_out: int, max_off: int = 2 * BLOCK, max_lit: int = 70000) -> list:
    """A valid stream of n_out output bytes as a foreign encoder might write
    it: literals of all header widths (some spanning blocks), copies of every
    kind reaching up to max_off back (across block boundaries), overlapping
    copies, all lengths 1..64."""
    r = SplitMix64(seed)
    ops, op = [], 0
    while op < n_out:
        left = n_out - op
        if op == 0 or r.below(10) < 3:
            c = r.below(100)
            n = 1 + (r.below(16) if c < 50 else r.below(64) if c < 85 else r.below(4096) if c < 97 else r.below(max_lit))
            n = min(n, left)
            m = n - 1
            minw = 0 if m < 60 else (1 if m < 256 else 2 if m < 65536 else 3)
            width = minw if r.below(4) else min(4, minw + r.below(3))
            if width == 0 and m >= 60:
                width = 1
            ops.append(["lit", n, int(r.next() & 0xFFFFFFFF), width])
            op += n
            continue
        c = r.below(100)
        lim = min(op, max_off)
        off = 1 + (r.below(min(lim, 64)) if c < 30 else r.below(min(lim, 2047)) if c < 60 else
                   r.below(min(lim, 65535)) if c < 85 else r.below(lim))
        length = min(1 + r.below(64), left)
        kinds = [4]
        if off < 65536:
            kinds.append(2)
        if 4 <= length <= 11 and off < 2048:
            kinds += [1, 1]
        ops.append(["copy", length, off, kinds[r.below(len(kinds))]])
        op += length
    return ops


def decoder_vector_ops() -> dict:
    """Hand-built streams whose elements cross 65,536-byte output boundaries
    or copy from earlier blocks (the reference decodes one whole output
    buffer, src/snappy_decompression.c:345-363; copies check only
    offset <= 131,072, :262)."""
    B = BLOCK
    v = {
        # a copy at output 65,536 reaching back into block 0, each copy kind
        "xblock_copy1": [["lit", B, 11], ["copy", 8, 100, 1], ["lit", 20, 12]],
        "xblock_copy2": [["lit", B + 4, 13], ["copy", 64, 60000, 2], ["copy", 33, 65535, 2]],
        "xblock_copy4_64k": [["lit", B + 1000, 14], ["copy", 40, B, 4], ["copy", 7, B + 999, 4]],
        "xblock_copy4_128k": [["lit", 70000, 15], ["lit", 70000, 16], ["copy", 20, 2 * B, 4], ["lit", 5, 17]],
        # elements straddling the 65,536 boundary
        "straddle_literal": [["lit", B + 4, 18]],
        "straddle_literal_tail": [["lit", 100, 19], ["lit", B, 20], ["copy", 30, 5, 2]],
        "straddle_copy": [["lit", B - 10, 21], ["copy", 40, 1000, 2], ["lit", 50, 22]],
        "straddle_copy_overlap": [["lit", B - 3, 23], ["copy", 64, 3, 2], ["copy", 11, 2, 1]],
        "straddle_copy4": [["lit", B - 1, 24], ["copy", 2, 1, 4], ["lit", 9, 25]],
        # overlapping copies (offset < length) just after the boundary: the
        # repeated bytes lie in the earlier block
        "xblock_copy_overlap": [["lit", B + 2, 29], ["copy", 60, 5, 2], ["copy", 9, 7, 1], ["lit", 3, 30]],
        "xblock_copy1_overlap": [["lit", B, 31], ["copy", 11, 4, 1], ["copy", 64, 1, 2]],
        # a literal covering a whole block (block 1 starts and ends inside it)
        "literal_spans_3_blocks": [["lit", 1000, 26], ["lit", 131000, 27, 3], ["copy", 64, 131072, 4]],
        # every block copies from the previous one: a pass-2 dependency chain
        "chain_5_blocks": [["lit", 70000, 28]] + [["copy", 64, 65536 + 17 * (i % 50), 4] for i in range(4700)],
    }
    return v
