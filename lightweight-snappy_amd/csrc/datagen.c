/*
 * datagen.c -- seeded synthetic inputs for tests and bench.py (SURVEY.md
 * §8(d), Appendix D).  Every generator is counter-based per 1 MiB chunk so
 * the GPU box regenerates bit-identical inputs from (kind, seed, size) and
 * large buffers are filled by several threads.
 *
 *   T  text   : Zipf(1.2) draws over a 50,000-word seeded vocabulary with
 *               letter frequencies ~ 1/rank^0.9 ("enwik8-like" stand-in;
 *               there is no enwik8 in the image and no network).
 *   R  random : splitmix64 bytes.
 *   P  repeat : 64 splitmix64 bytes tiled (the all-copy best case).
 *   L  lcg    : x=(x*1103515245+12345)&0x7fffffff, byte=(x>>16)&0xff
 *               (SURVEY.md Appendix B known-answer input; serial).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>
#include <math.h>
#include <pthread.h>

#define GEN_CHUNK (1u << 20)
#define VOCAB 50000
#define MAXW 12
#define GUIDE_BITS 16

static inline uint64_t splitmix64(uint64_t *s)
{
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

typedef struct {
    char words[VOCAB][MAXW];
    uint8_t len[VOCAB];
    double cdf[VOCAB];
    /* guide[b] = first word whose cdf >= b / 2^GUIDE_BITS: a draw u in bucket b
     * is found by bisecting [guide[b], guide[b + 1]] only (same word as a
     * bisection of the whole table, ~4x faster on the Zipf head) */
    uint16_t guide[(1u << GUIDE_BITS) + 1];
} vocab_t;

static vocab_t *g_vocab;
static uint64_t g_vocab_seed = ~0ull;
static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER;

static const char *k_common[] = {"the", "of", "and", "in", "to", "a", "is", "was", "for", "as"};

static void build_vocab(uint64_t seed)
{
    vocab_t *v = (vocab_t *)calloc(1, sizeof(vocab_t));
    static const char alpha[] = "etaoinshrdlcumwfgypbvkjxqz";
    double lw[26], tot = 0;
    for (int i = 0; i < 26; i++) { lw[i] = 1.0 / pow(i + 1, 0.9); tot += lw[i]; }
    double lc[26], acc = 0;
    for (int i = 0; i < 26; i++) { acc += lw[i] / tot; lc[i] = acc; }
    uint64_t s = seed * 0x2545F4914F6CDD1Dull + 12345;
    for (int w = 0; w < VOCAB; w++) {
        if (w < (int)(sizeof(k_common) / sizeof(k_common[0]))) {
            v->len[w] = (uint8_t)strlen(k_common[w]);
            memcpy(v->words[w], k_common[w], v->len[w]);
            continue;
        }
        int L = 2 + (int)(splitmix64(&s) % 9);
        v->len[w] = (uint8_t)L;
        for (int i = 0; i < L; i++) {
            double u = (splitmix64(&s) >> 11) * (1.0 / 9007199254740992.0);
            int k = 0;
            while (k < 25 && u > lc[k]) k++;
            v->words[w][i] = alpha[k];
        }
    }
    double z = 0;
    for (int r = 0; r < VOCAB; r++) z += 1.0 / pow(r + 1, 1.2);
    double c = 0;
    for (int r = 0; r < VOCAB; r++) { c += 1.0 / pow(r + 1, 1.2) / z; v->cdf[r] = c; }
    v->cdf[VOCAB - 1] = 1.0;
    int w = 0;
    for (uint32_t b = 0; b <= (1u << GUIDE_BITS); b++) {
        const double x = (double)b / (double)(1u << GUIDE_BITS);
        while (w < VOCAB - 1 && v->cdf[w] < x) w++;
        v->guide[b] = (uint16_t)w;
    }
    g_vocab = v;
}

static void ensure_vocab(uint64_t seed)
{
    pthread_mutex_lock(&g_lock);
    if (!g_vocab || g_vocab_seed != seed) {
        free(g_vocab);
        build_vocab(seed);
        g_vocab_seed = seed;
    }
    pthread_mutex_unlock(&g_lock);
}

static void text_chunk(uint8_t *out, size_t n, uint64_t seed, uint64_t chunk)
{
    const vocab_t *v = g_vocab;
    uint64_t s = seed ^ (chunk * 0xD1B54A32D192ED03ull) ^ 0x5851F42D4C957F2Dull;
    size_t o = 0;
    int since_period = 0;
    while (o < n) {
        double u = (splitmix64(&s) >> 11) * (1.0 / 9007199254740992.0);
        const uint32_t b = (uint32_t)(u * (double)(1u << GUIDE_BITS));
        int lo = v->guide[b], hi = v->guide[b + 1];
        while (lo < hi) { int mid = (lo + hi) >> 1; if (v->cdf[mid] < u) lo = mid + 1; else hi = mid; }
        char buf[32];
        int k = 0;
        if (lo == 0) { memcpy(buf, "[[the", 5); k = 5; }
        else if (lo == 1) { memcpy(buf, "of]],\n", 6); k = 6; }
        else { memcpy(buf, v->words[lo], v->len[lo]); k = v->len[lo]; }
        if (++since_period > 14 && (splitmix64(&s) & 7) == 0) { buf[k++] = '.'; since_period = 0; }
        buf[k++] = ' ';
        for (int i = 0; i < k && o < n; i++) out[o++] = (uint8_t)buf[i];
    }
}

static void random_chunk(uint8_t *out, size_t n, uint64_t seed, uint64_t byte_off)
{
    /* counter-based: 8 bytes per counter value, so any chunk is addressable */
    for (size_t i = 0; i < n; i += 8) {
        uint64_t s = seed * 0x9E3779B97F4A7C15ull + (byte_off + i) / 8;
        uint64_t r = splitmix64(&s);
        size_t k = n - i < 8 ? n - i : 8;
        memcpy(out + i, &r, k);
    }
}

typedef struct { uint8_t *out; size_t n; size_t off; int kind; uint64_t seed; size_t c0, c1; uint8_t pat[64]; } gen_job;

static void *gen_worker(void *arg)
{
    gen_job *j = (gen_job *)arg;
    for (size_t c = j->c0; c < j->c1; c++) {
        size_t b = c * GEN_CHUNK;
        size_t L = j->n - b < GEN_CHUNK ? j->n - b : GEN_CHUNK;
        if (j->kind == 'T') text_chunk(j->out + b, L, j->seed, (j->off + b) / GEN_CHUNK);
        else if (j->kind == 'R') random_chunk(j->out + b, L, j->seed, j->off + b);
        else if (j->kind == 'P') for (size_t i = 0; i < L; i++) j->out[b + i] = j->pat[(j->off + b + i) & 63];
        else if (j->kind == 'Z') memset(j->out + b, 0, L);
    }
    return NULL;
}

/* Fill out[0..n) with bytes [off, off+n) of generator `kind` ('T','R','P',
 * 'Z'; 'L' only at off 0).  `off` must be a multiple of 1 MiB so each rank
 * of a sharded bench can build only its own shard.  Returns 0 on success,
 * -1 on an unknown kind, -2 on a misaligned offset. */
int snappy_gen_fill_at(uint8_t *out, size_t n, size_t off, int kind, uint64_t seed, int nthreads)
{
    if (off % GEN_CHUNK) return -2;
    if (kind == 'L') {
        if (off) return -2;
        uint32_t x = (uint32_t)seed;
        for (size_t i = 0; i < n; i++) { x = (x * 1103515245u + 12345u) & 0x7fffffffu; out[i] = (uint8_t)((x >> 16) & 0xff); }
        return 0;
    }
    if (kind != 'T' && kind != 'R' && kind != 'P' && kind != 'Z') return -1;
    if (kind == 'T') ensure_vocab(seed);
    gen_job proto;
    memset(&proto, 0, sizeof(proto));
    proto.out = out; proto.n = n; proto.off = off; proto.kind = kind; proto.seed = seed;
    if (kind == 'P') random_chunk(proto.pat, 64, seed, 0);
    size_t nc = (n + GEN_CHUNK - 1) / GEN_CHUNK;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    if ((size_t)nthreads > nc) nthreads = nc ? (int)nc : 1;
    pthread_t th[64];
    gen_job jobs[64];
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = proto;
        jobs[t].c0 = nc * t / nthreads;
        jobs[t].c1 = nc * (t + 1) / nthreads;
        if (nthreads == 1) gen_worker(&jobs[t]);
        else pthread_create(&th[t], NULL, gen_worker, &jobs[t]);
    }
    if (nthreads > 1) for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    return 0;
}

int snappy_gen_fill(uint8_t *out, size_t n, int kind, uint64_t seed, int nthreads)
{
    return snappy_gen_fill_at(out, n, 0, kind, seed, nthreads);
}
