#!/usr/bin/env python3
"""Lane-level model of K5c's batch-parse chain walk (k5_chain<MARK> in
snappy_kernels.hip): 64 lanes parse candidate elements at x + lane, pointer
doubling finds the chain, prefix sums place the elements, the first bad /
at-or-past-N / past-N element ends the batch.  Checked here against the serial
walk of the original K5c (element by element, the same checks and entries) on
seeded foreign streams, truncations and byte flips, one chunk at a time from
every chunk's true entry.  Usage: python3 tools/k5_model.py [cases]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "lightweight-snappy_amd")]
from golden_inputs import build_stream, random_ops  # noqa: E402

B = 65536
S = 16384  # K5_S
OK, TRUNC, OVERRUN, UNSUP = 0, -3, -5, -8


def parse(s, x):
    """k5_parse: (ok, size, len) of the element at x (bytes past the stream read 0)."""
    clen = len(s)
    if x >= clen:
        return False, 2, 1
    b = [s[x + k] if x + k < clen else 0 for k in range(5)]
    tag, t, m = b[0], b[0] & 3, b[0] >> 2
    if t == 0:
        k = m - 59 if m >= 60 else 0
        lv = m if k == 0 else int.from_bytes(bytes(b[1:1 + k]), "little")
        ln, hb = lv + 1, 1 + k
        size = hb + ln
    else:
        ln = (m & 7) + 4 if t == 1 else m + 1
        hb = {1: 2, 2: 3, 3: 5}[t]
        size = hb
    return x + hb <= clen, size, ln


def serial(s, x, end, op, N, offs):
    """The original K5c loop over [x, end) from output op."""
    clen = len(s)
    while x < end and op < N:
        ok, size, ln = parse(s, x)
        if not ok or x + size > clen:
            return TRUNC, x, op
        nb = (op // B + 1) * B
        while nb < op + ln and nb < N:
            skip = nb - op
            if skip >> 24 or x >> 40:
                return UNSUP, x, op
            offs[nb // B] = x | (skip << 40)
            nb += B
        op += ln
        x += size
        if op > N:
            return OVERRUN, x, op
        if op % B == 0 and op < N:
            offs[op // B] = x
    return OK, x, op


def batched(s, c0, x, end, op, N, offs):
    """k5_chain<true> with x relative to c0, lanes as lists."""
    clen, st = len(s), OK
    while x < end - c0 and op < N and st == OK:
        par = [parse(s, c0 + x + l) for l in range(64)]
        size = [p[1] for p in par]
        nxt = [l + min(size[l], 64) for l in range(64)]
        pos, l0 = [], 0
        while l0 < 64 and len(pos) < 32:  # = the pointer-doubling result
            pos.append(l0)
            l0 = nxt[l0]
        pos = [p for p in pos if x + p < end - c0]
        E = len(pos)
        assert E >= 1
        e_ok = [par[p][0] for p in pos]
        e_size = [par[p][1] for p in pos]
        e_len = [par[p][2] for p in pos]
        e_x = [x + sum(e_size[:k]) for k in range(E)]
        e_op = [op + sum(e_len[:k]) for k in range(E)]
        nexec, er = E, OK
        for k in range(E):
            bad = not e_ok[k] or c0 + e_x[k] + e_size[k] > clen
            if bad:
                nexec, er = k, TRUNC
                break
            if e_op[k] >= N:
                nexec = k
                break
            if e_op[k] + e_len[k] > N:
                nexec, er = k + 1, OVERRUN
                break
        for k in range(nexec):  # end entries (lane-parallel in the kernel)
            e_end = e_op[k] + e_len[k]
            if e_end % B == 0 and e_end < N:
                offs[e_end // B] = c0 + e_x[k] + e_size[k]
        for k in range(nexec):  # straddles, lane order
            nb, e_end, kx = (e_op[k] // B + 1) * B, e_op[k] + e_len[k], c0 + e_x[k]
            while nb < e_end and nb < N:
                skip = nb - e_op[k]
                if skip >> 24 or kx >> 40:
                    er = UNSUP
                    break
                offs[nb // B] = kx | (skip << 40)
                nb += B
        if nexec:
            x = e_x[nexec - 1] + e_size[nexec - 1]
            op = e_op[nexec - 1] + e_len[nexec - 1]
        if er != OK:
            st = er
    return st, c0 + x, op


def check(s):
    h, N, k = 0, 0, 0
    while True:
        b = s[k]
        N |= (b & 0x7F) << (7 * k)
        k += 1
        if not b & 0x80:
            break
    h = k
    # true entries by the serial walk, chunk by chunk (K5b), then both walks per chunk
    x, op, c = h, 0, 0
    while h + c * S < len(s) and op < N:
        c0 = h + c * S
        end = min(c0 + S, len(s))
        if x < end:
            o1, o2 = {}, {}
            r1 = serial(s, x, end, op, N, o1)
            r2 = batched(s, c0, x - c0, end, op, N, o2)
            if r1[0] == OK:
                assert r2 == r1 and o1 == o2, (c, r1, r2)
            else:  # an error: the same error (the entries are discarded)
                assert r2[0] == r1[0], (c, r1, r2)
                return r1[0]
            x, op = r1[1], r1[2]
        c += 1
    return OK


def main():
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    rng = np.random.default_rng(11)
    n_err = 0
    for seed in range(cases):
        s = bytearray(build_stream(random_ops(seed, 200_000 + 50_000 * (seed % 4), 131072)))
        variants = [bytes(s), bytes(s[: len(s) - 1 - seed * 37]), bytes(s[: len(s) // 2])]
        for _ in range(3):
            b = bytearray(s)
            for p in rng.integers(8, len(b), 3):
                b[p] ^= int(rng.integers(1, 255))
            variants.append(bytes(b))
        for v in variants:
            n_err += check(v) != OK
    print(f"k5 model: {cases * 6} streams, batch walk == serial walk ({n_err} ending in an error)")


if __name__ == "__main__":
    main()
