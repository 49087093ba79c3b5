// tools/k1r_chain_sim.c -- would a K1r round that resolves two matches pay?
// Replays the reference match loop (src/snappy_compression.c:384-403, as
// oracle/snappy_oracle.c restates it) over 32 KiB units of a text file and
// counts, per match: whether the next match starts at the first probe after
// the copy (a "chain"), how often a same-offset run of table candidates
// predicts the copy length exactly, and how often the next probe is a match
// with the length among the three most frequent (4, 5, 6) -- the best a
// one-gather round with 16-lane compare groups could speculate on.
//   gcc -O2 -o /tmp/k1r_chain_sim tools/k1r_chain_sim.c && /tmp/k1r_chain_sim FILE [UNIT]
// (FILE: e.g. datagen.make("T", 64 << 20, 1234) written out)
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
static inline uint32_t be32(const uint8_t *p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }
int main(int argc, char **argv) {
    if (argc < 2) { fprintf(stderr, "usage: %s FILE [UNIT]\n", argv[0]); return 2; }
    FILE *f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 1; }
    fseek(f, 0, SEEK_END);
    size_t N = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *in0 = malloc(N);
    if (!in0 || fread(in0, 1, N, f) != N) { fprintf(stderr, "read failed\n"); return 1; }
    fclose(f);
    uint32_t U = argc > 2 ? (uint32_t)atoi(argv[2]) : 32768;
    long matches = 0, chain = 0, lenhist[80] = {0}, runok = 0, runok_chain = 0, spec3 = 0, spec3r = 0;
    for (size_t b = 0; b + U <= N; b += U) {
        const uint8_t *in = in0 + b; uint32_t L = U;
        uint16_t table[4096]; memset(table, 0, sizeof table);
        uint32_t T = 256, lg = 8; while (T < 4096 && T < L) { T <<= 1; lg++; }
        uint32_t shift = 32 - lg;
        uint32_t skip = 33, p = 1;
        int prev_match_end = -1;
        while (!(L - p < (skip >> 5) + 15)) {
            uint32_t cur = be32(in + p), h = (cur * 0x1e35a7bdu) >> shift, cand = table[h];
            if (be32(in + cand) == cur) {
                uint32_t n = 4; while (p + n < L && in[p + n] == in[cand + n]) n++;
                matches++;
                if ((int)p == prev_match_end) chain++;
                lenhist[n < 79 ? n : 79]++;
                table[h] = (uint16_t)p;
                // run predictor on the table after this match's insert
                uint32_t r = 1;
                while (p + r + 3 < L) {
                    uint32_t x = be32(in + p + r), hx = (x * 0x1e35a7bdu) >> shift;
                    if (table[hx] != cand + r || be32(in + cand + r) != x) break;
                    r++;
                }
                uint32_t s = p + r + 3;
                int ok = (s == p + n);
                runok += ok;
                // next probe s = p + n: is it a match? (sequential truth: table unchanged in between)
                uint32_t q = p + n;
                int nexthit = 0;
                if (!(L - q < 1 + 15)) {
                    uint32_t c2 = be32(in + q), h2 = (c2 * 0x1e35a7bdu) >> shift;
                    nexthit = be32(in + table[h2]) == c2;
                }
                if (ok && nexthit) runok_chain++;
                if (nexthit && (n == 4 || n == 5 || n == 6)) spec3++;
                if (nexthit && (ok || n == 4 || n == 5)) spec3r++;
                skip = 32;
                p += n;
                prev_match_end = p;
            } else {
                table[(be32(in + p - 1) * 0x1e35a7bdu) >> shift] = (uint16_t)(p - 1);
                table[h] = (uint16_t)p;
                p += skip >> 5; skip++;
            }
        }
    }
    printf("unit %u: matches %ld chain(next match at first probe) %.3f\n", U, matches, (double)chain / matches);
    printf("run predictor exact %.3f ; run-exact AND next probe hits %.3f\n", (double)runok / matches, (double)runok_chain / matches);
    printf("next hits with len in {4,5,6} %.3f ; run-or-{4,5} %.3f\n", (double)spec3 / matches, (double)spec3r / matches);
    double cum = 0; for (int i = 4; i < 20; i++) { cum += (double)lenhist[i] / matches; printf("len %d: %.3f (cum %.3f)\n", i, (double)lenhist[i] / matches, cum); }
    return 0;
}
