#!/usr/bin/env python3
"""Python model of K1r's lane-space rounds (one 64-lane window, per-lane
lists) checked against a serial restatement of compress_next_block
(src/snappy_compression.c:384-403).  A logic check for the round structure,
not a product path: it compares (position, length, offset) token lists.

Usage: python tools/k1r_model.py [n_blocks]
"""
import random
import sys

MUL = 0x1E35A7BD
TAGMUL = 0x9E3779B1


def be32(b, q):
    return (b[q] << 24) | (b[q + 1] << 16) | (b[q + 2] << 8) | b[q + 3]


def table_shift(L):
    T, lg = 256, 8
    while T < 4096 and T < L:
        T <<= 1
        lg += 1
    return 32 - lg


def serial_tokens(b):
    L = len(b)
    sh = table_shift(L)
    tab = {}
    h = lambda q: ((be32(b, q) * MUL) & 0xFFFFFFFF) >> sh
    p, skip, toks = 1, 33, []
    while not (L - p < (skip >> 5) + 15):
        c = tab.get(h(p), 0)
        if be32(b, c) == be32(b, p):
            n = 4
            while p + n < L and b[p + n] == b[c + n]:
                n += 1
            toks.append((p, n, p - c))
            tab[h(p)] = p
            p += n
            skip = 32
        else:
            tab[h(p - 1)] = p - 1
            tab[h(p)] = p
            p += skip >> 5
            skip += 1
    return toks


def lanespace_tokens(b, DMAX=16, LSMIN=4, RMIN=8):
    L = len(b)
    bp = bytes(b) + bytes(300)
    sh = table_shift(L)
    hsh = lambda q: ((be32(bp, q) * MUL) & 0xFFFFFFFF) >> sh
    tag = lambda q: ((be32(bp, q) * TAGMUL) & 0xFFFFFFFF) >> 24
    tab = {}  # slot -> (pos, tag)
    tab_get = lambda s: tab.get(s, (0, tag(0)))
    p, skip, toks = 1, 33, []
    q0, d0, lsw, lmax = None, -10**9, False, 0
    hv = pd = ent = None
    while not (L - p < (skip >> 5) + 15):
        if skip <= 64 - LSMIN:
            lane0 = p - q0 if q0 is not None else -1
            if not lsw or p - 1 < q0 or lane0 + RMIN > lmax:
                q0 = p - 1
                if (q0 >> 2) - d0 > 34:
                    d0 = q0 >> 2
                hv = [(hsh(q0 + l), tag(q0 + l)) for l in range(64)]
                pd = []
                for l in range(64):
                    d = next((d for d in range(1, DMAX + 1) if l - d >= 0 and hv[l - d][0] == hv[l][0]), None)
                    pd.append(d)
                lmax = min(62, 4 * d0 + 191 - q0)
                ent = [tab_get(hv[l][0]) for l in range(64)]
                lsw = True
                lane0 = 1
            kmax = min(64 - skip, DMAX - 1, lmax - lane0, L - p - 16)
            if skip + kmax == 64 and L - p - kmax < 17:
                kmax -= 1
            f = None
            for l in range(lane0, lane0 + kmax + 1):
                k = l - lane0
                inr = k >= 1 and pd[l] is not None and pd[l] <= k + 1
                if inr:
                    cand, hit = q0 + l - pd[l], hv[l - pd[l]] == hv[l]
                else:
                    cand, hit = ent[l][0], ent[l][1] == hv[l][1]
                if hit:
                    f, c = l, cand
                    break
            lo = lane0 - 1
            if f is not None:
                pf = q0 + f
                n = 0
                while pf + n < L and bp[pf + n] == bp[c + n]:
                    n += 1
                hi = f
                if n >= 4:
                    toks.append((pf, n, pf - c))
                    if f == lane0:
                        lo = lane0
                    np_, skip = pf + n, 32
                else:
                    np_, skip = pf + ((skip + f - lane0) >> 5), skip + f - lane0 + 1
            else:
                f = lane0 + kmax + 1
                hi, np_ = f - 1, q0 + f - 1 + ((skip + kmax) >> 5)
                skip += kmax + 1
            for l in range(lo, hi + 1):  # lane order: the highest lane wins a slot
                tab[hv[l][0]] = (q0 + l, hv[l][1])
            ent = [tab_get(hv[l][0]) for l in range(64)]
            p = np_
            continue
        lsw = False
        # general (serial) probe, as the legacy W-lane path computes it
        c, ctag = tab_get(hsh(p))
        if be32(bp, c) == be32(bp, p):
            n = 4
            while p + n < L and bp[p + n] == bp[c + n]:
                n += 1
            toks.append((p, n, p - c))
            tab[hsh(p)] = (p, tag(p))
            p += n
            skip = 32
        else:
            tab[hsh(p - 1)] = (p - 1, tag(p - 1))
            tab[hsh(p)] = (p, tag(p))
            p += skip >> 5
            skip += 1
    return toks


def text(n, rng):
    words = ["".join(rng.choice("etaoinshrdlucmfw") for _ in range(rng.randint(2, 9))) for _ in range(300)]
    out = []
    while sum(len(w) + 1 for w in out) < n:
        out.append(words[min(int(rng.paretovariate(1.1)) - 1, 299)])
    return " ".join(out).encode()[:n]


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    rng = random.Random(7)
    cases = [bytes(range(64)) * 64, bytes(4096), bytes(i & 0xFF for i in range(8192))]
    for i in range(nb):
        n = rng.choice([100, 2049, 4096, 9000, 32768])
        kind = rng.choice("tmrp")
        if kind == "t":
            cases.append(text(n, rng))
        elif kind == "r":
            cases.append(bytes(rng.getrandbits(8) for _ in range(n)))
        elif kind == "p":
            per = rng.randint(1, 80)
            pat = bytes(rng.getrandbits(8) for _ in range(per))
            cases.append((pat * (n // per + 1))[:n])
        else:
            t = text(n, rng)
            cases.append(bytes(x if rng.random() < 0.97 else rng.getrandbits(8) for x in t))
    bad = 0
    for i, b in enumerate(cases):
        a, m = serial_tokens(b), lanespace_tokens(b)
        if a != m:
            bad += 1
            j = next((j for j in range(min(len(a), len(m))) if a[j] != m[j]), min(len(a), len(m)))
            print(f"case {i} len {len(b)}: first difference at token {j}: serial {a[j:j+2]} lanes {m[j:j+2]}")
    print(f"{len(cases) - bad}/{len(cases)} cases identical")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
