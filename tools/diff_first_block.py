#!/usr/bin/env python3
"""Debug aid: compress a seeded input with the library (GPU) and with the
oracle (CPU), report the first 64 KiB block whose compressed bytes differ and
the first differing element of that block (both streams parsed).
Usage: tools/diff_first_block.py [T|R|P] [bytes]   (GPU box; test infrastructure)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "lightweight-snappy_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import datagen  # noqa: E402
import oracle  # noqa: E402
import snappy_amd  # noqa: E402


def elements(comp, start):
    """[(stream offset, kind, length, offset)] of one block's elements from start."""
    out, p = [], start
    while p < len(comp):
        tag = comp[p]; t = tag & 3; m = tag >> 2
        if t == 0:
            k = max(m - 59, 0)
            ln = (int.from_bytes(comp[p + 1:p + 1 + k], "little") if k else m) + 1
            out.append((p, "lit", ln, 0)); p += 1 + k + ln
        elif t == 1:
            out.append((p, "c1", (m & 7) + 4, ((tag >> 5) << 8) | comp[p + 1])); p += 2
        elif t == 2:
            out.append((p, "c2", m + 1, int.from_bytes(comp[p + 1:p + 3], "little"))); p += 3
        else:
            out.append((p, "c4", m + 1, int.from_bytes(comp[p + 1:p + 5], "little"))); p += 5
    return out


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "T"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4 << 20
    data = bytes(datagen.make(kind, n, 1234 if kind == "T" else 1))
    g = snappy_amd.compress(data)
    o = oracle.compress(data)
    print("lengths gpu", len(g), "oracle", len(o), "identical", g == o)
    if g == o:
        return
    i = next(k for k in range(min(len(g), len(o))) if g[k] != o[k])
    # walk both streams' elements to the first difference, tracking the output position
    hdr = 0
    while o[hdr] & 0x80:
        hdr += 1
    hdr += 1
    eg, eo = elements(g, hdr), elements(o, hdr)
    pos = 0
    for a, b in zip(eg, eo):
        if a[1:] != b[1:]:
            print(f"first differing element at output position {pos} (block {pos >> 16}, in-block {pos & 65535}):")
            print("  gpu   ", a, "\n  oracle", b)
            break
        pos += a[2]
    print("first differing byte", i)


if __name__ == "__main__":
    main()
