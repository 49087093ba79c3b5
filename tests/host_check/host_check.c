/*
 * host_check.c -- TEST INFRASTRUCTURE: the host side of libsnappy_amd under
 * AddressSanitizer + UndefinedBehaviorSanitizer (tests/host_check/Makefile
 * instruments the host code of snappy_device.hip and snappy_host.c; the gfx950
 * kernels are the product objects, unchanged).  Checks against the oracle
 * (oracle/snappy_oracle.c, linked in as the checker), never the thing tested.
 *
 *   host_check_asan nodev   no GPU: varint round trips and truncated varints,
 *                           every host entry point's error path, the -b
 *                           compressor's host threads (the build container;
 *                           tests/test_host_check.py)
 *   host_check_asan gpu     the buffer and FILE* pipelines (ragged sizes, a
 *                           three-chunk input), the sidecar index and a
 *                           corrupted one, malformed streams, pooled host
 *                           contexts from four threads (tests -m gpu)
 *
 * Reference behaviour followed: snappy_compress / snappy_decompress
 * (src/snappy_compression.c:414-428, src/snappy_decompression.c:290-363) as
 * restated by the oracle; varint (src/varint.c:12-42).
 */
#include <pthread.h>
#include <sanitizer/lsan_interface.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "snappy_amd.h"

size_t oracle_compress(const uint8_t *in, size_t n, uint8_t *out);
size_t oracle_max_compressed_length(size_t n);
int oracle_decompress(const uint8_t *in, size_t n, uint8_t *out, size_t cap, size_t *out_len);
int snappy_gen_fill(uint8_t *out, size_t n, int kind, uint64_t seed, int nthreads);

static int g_fail = 0;
#define CHECK(cond, ...)                                                                           \
    do {                                                                                           \
        if (!(cond)) {                                                                             \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);                                   \
            fprintf(stderr, __VA_ARGS__);                                                          \
            fputc('\n', stderr);                                                                   \
            g_fail++;                                                                              \
        }                                                                                          \
    } while (0)

static uint8_t *make_input(size_t n, int kind, uint64_t seed)
{
    uint8_t *a = malloc(n ? n : 1);
    if (n && snappy_gen_fill(a, n, kind, seed, 8) != 0) {
        fprintf(stderr, "datagen failed\n");
        exit(2);
    }
    return a;
}

static void check_varints(void)
{
    const uint64_t vals[] = {0, 1, 127, 128, 16383, 16384, 1000000, 0xFFFFFFFFull, 1ull << 35, UINT64_MAX};
    for (size_t i = 0; i < sizeof vals / sizeof *vals; i++) {
        uint8_t b[16];
        const uint32_t k = snappy_varint_encode(vals[i], b);
        uint64_t v = 0;
        CHECK(k >= 1 && k <= 10, "varint length %u", k);
        CHECK(snappy_varint_decode(b, k, &v) == k && v == vals[i], "varint round trip of %llu",
              (unsigned long long)vals[i]);
        for (uint32_t t = 0; t < k; t++) {  // every truncation: 0 (no complete varint)
            uint8_t *c = malloc(t ? t : 1);  // exact-size copy: a read past it is an ASan report
            memcpy(c, b, t);
            CHECK(snappy_varint_decode(c, t, &v) == 0, "truncated varint (%u of %u bytes) accepted", t, k);
            free(c);
        }
    }
    uint8_t over[11];
    memset(over, 0x80, sizeof over);
    uint64_t v;
    CHECK(snappy_varint_decode(over, sizeof over, &v) == 0, "11-byte varint accepted");
    CHECK(snappy_max_compressed_length(0) >= 1, "max length of 0");
}

/* no device: each host entry reports an error and leaves no pending state */
static void check_nodev(void)
{
    uint8_t in[300], out[600], back[300];
    size_t len = 0;
    memset(in, 'a', sizeof in);
    CHECK(snappy_compress_buffer(in, sizeof in, out, &len) < 0, "compress without a device succeeded");
    const uint8_t stream[] = {10, 0x24, 'a', 'b', 'c', 'd', 'e', 'f', 'g', 'h', 'i', 'j'};
    int st = snappy_decompress_buffer(stream, sizeof stream, back, sizeof back, &len);
    CHECK(st < 0, "decompress without a device: %d", st);
    len = 99;  // the empty stream (what an empty input compresses to) decodes to nothing
    st = snappy_decompress_buffer(stream, 0, back, sizeof back, &len);
    CHECK(st == 0 && len == 0, "empty stream: %d, %zu bytes", st, len);
    uint64_t n = 0;
    CHECK(snappy_uncompressed_length(stream, sizeof stream, &n) == 0 && n == 10, "uncompressed length");
    CHECK(snappy_uncompressed_length(stream, 0, &n) < 0, "uncompressed length of nothing");
    FILE *fi = tmpfile(), *fo = tmpfile();
    fwrite(in, 1, sizeof in, fi);
    rewind(fi);
    snappy_compress(fi, sizeof in, fo);
    CHECK(snappy_amd_last_status() < 0, "FILE* compress without a device: %d", snappy_amd_last_status());
    rewind(fi);
    CHECK(snappy_decompress(fi, fo) < 0, "FILE* decompress of raw text succeeded");
    fclose(fi);
    fclose(fo);
    snappy_amd_host_release();
}

/* the -b compressor (host threads, no device): every output decodes (oracle)
 * to its input, the FILE* form writes the buffer form's bytes, a short
 * output buffer is refused */
static void check_bst(void)
{
    const size_t sizes[] = {1, 4, 15, 16, 17, 100, 65535, 65536, 65537, 200000, (33u << 20) + 777};
    for (size_t i = 0; i < sizeof sizes / sizeof *sizes; i++) {
        for (int k = 0; k < 3; k++) {
            const int kind = "TRP"[k];
            const size_t n = sizes[i];
            uint8_t *a = make_input(n, kind, 5 + i);
            const size_t cap = snappy_max_compressed_length(n);
            uint8_t *c = malloc(cap), *back = malloc(n);
            size_t len = 0, dl = 0;
            CHECK(snappy_compress_bst_buffer(a, n, c, cap, &len) == 0, "bst compress %zu", n);
            CHECK(oracle_decompress(c, len, back, n, &dl) == 0 && dl == n && !memcmp(back, a, n),
                  "bst round trip %zu kind %c", n, kind);
            FILE *fi = tmpfile(), *fo = tmpfile();
            fwrite(a, 1, n, fi);
            rewind(fi);
            CHECK(snappy_compress_bst(fi, n, fo) == 0, "bst FILE* %zu", n);
            CHECK((size_t)ftell(fo) == len, "bst FILE* length %zu", n);
            rewind(fo);
            uint8_t *f = malloc(len ? len : 1);
            CHECK(fread(f, 1, len, fo) == len && !memcmp(f, c, len), "bst FILE* bytes %zu", n);
            size_t l2 = 0;
            CHECK(snappy_compress_bst_buffer(a, n, c, len - 1, &l2) == SNAPPY_AMD_ERR_CAPACITY, "bst short buffer");
            fclose(fi);
            fclose(fo);
            free(a);
            free(c);
            free(back);
            free(f);
        }
    }
    size_t len = 7;
    CHECK(snappy_compress_bst_buffer(NULL, 0, NULL, 0, &len) == 0 && len == 0, "bst of nothing");
}

static void round_trip_buffer(size_t n, int kind, uint64_t seed)
{
    uint8_t *a = make_input(n, kind, seed);
    const size_t cap = snappy_max_compressed_length(n);
    uint8_t *c = malloc(cap), *r = malloc(oracle_max_compressed_length(n));
    uint8_t *b = malloc(n ? n : 1);
    size_t len = 0, got = 0;
    int st = snappy_compress_buffer(a, n, c, &len);
    const size_t rl = oracle_compress(a, n, r);
    CHECK(st == 0 && len == rl && memcmp(c, r, rl) == 0, "buffer compress n=%zu kind=%d: st %d len %zu oracle %zu",
          n, kind, st, len, rl);
    if (n) {
        st = snappy_decompress_buffer(c, len, b, n, &got);
        CHECK(st == 0 && got == n && memcmp(a, b, n) == 0, "buffer decompress n=%zu: st %d got %zu", n, st, got);
        if (n > 1) {  // one byte too little room
            st = snappy_decompress_buffer(c, len, b, n - 1, &got);
            CHECK(st == SNAPPY_AMD_ERR_CAPACITY, "capacity n=%zu: st %d", n, st);
        }
    }
    free(a);
    free(c);
    free(r);
    free(b);
}

static uint8_t *read_all(FILE *f, size_t *n)
{
    fseeko(f, 0, SEEK_END);
    *n = (size_t)ftello(f);
    rewind(f);
    uint8_t *p = malloc(*n ? *n : 1);
    CHECK(fread(p, 1, *n, f) == *n, "read back");
    return p;
}

static void round_trip_file(size_t n, int kind, uint64_t seed, int indexed)
{
    uint8_t *a = make_input(n, kind, seed), *r = malloc(oracle_max_compressed_length(n));
    const size_t rl = oracle_compress(a, n, r);
    FILE *fi = tmpfile(), *fc = tmpfile(), *fo = tmpfile(), *fx = indexed ? tmpfile() : NULL;
    CHECK(fwrite(a, 1, n, fi) == n, "write input");
    rewind(fi);
    int st;
    if (indexed) st = snappy_compress_file_indexed(fi, n, fc, fx);
    else {
        snappy_compress(fi, n, fc);
        st = snappy_amd_last_status();
    }
    size_t cl;
    uint8_t *c = read_all(fc, &cl);
    CHECK(st == 0 && cl == rl && memcmp(c, r, rl) == 0, "FILE* compress n=%zu indexed=%d: st %d len %zu oracle %zu",
          n, indexed, st, cl, rl);
    rewind(fc);
    st = indexed ? (rewind(fx), snappy_decompress_file_indexed(fc, fx, fo)) : snappy_decompress(fc, fo);
    size_t ol;
    uint8_t *o = read_all(fo, &ol);
    CHECK(st == 0 && ol == n && memcmp(o, a, n) == 0, "FILE* decompress n=%zu indexed=%d: st %d got %zu", n, indexed,
          st, ol);
    if (indexed && n > 65536) {
        size_t xl;
        uint8_t *x = read_all(fx, &xl);
        CHECK(xl >= 40, "index length %zu", xl);
        uint64_t e, e0;
        memcpy(&e0, x + 32, 8);  // entry 1 (after magic, N, count, entry 0)
        for (int k = 0; k < 2; k++) {
            // k 0: entry 1 one byte off an element start -- the index still looks
            // well-formed; block 0's chain ends before it, so K4 refuses it (ERR_INDEX);
            // k 1: entry 1 past the stream's end -- refused before any decoding
            e = k == 0 ? e0 + 1 : (uint64_t)cl + 100;
            memcpy(x + 32, &e, 8);
            FILE *fb = tmpfile(), *fo2 = tmpfile();
            fwrite(x, 1, xl, fb);
            rewind(fb);
            rewind(fc);
            st = snappy_decompress_file_indexed(fc, fb, fo2);
            CHECK(st == SNAPPY_AMD_ERR_INDEX, "index entry %s: st %d", k ? "past the stream" : "off by one byte", st);
            fclose(fb);
            fclose(fo2);
        }
        free(x);
    }
    fclose(fi);
    fclose(fc);
    fclose(fo);
    if (fx) fclose(fx);
    free(a);
    free(r);
    free(c);
    free(o);
}

/* malformed streams: every status is an error code, never a crash or an
 * out-of-bounds host access */
static void malformed(void)
{
    const size_t n = 200000;
    uint8_t *a = make_input(n, 'T', 5);
    uint8_t *c = malloc(snappy_max_compressed_length(n)), *b = malloc(n);
    size_t len = 0, got;
    CHECK(snappy_compress_buffer(a, n, c, &len) == 0, "compress");
    const size_t cuts[] = {1, 2, 3, 100, len / 2, len - 1};
    for (size_t i = 0; i < sizeof cuts / sizeof *cuts; i++) {
        uint8_t *t = malloc(cuts[i]);  // exact size
        memcpy(t, c, cuts[i]);
        int st = snappy_decompress_buffer(t, cuts[i], b, n, &got);
        CHECK(st < 0, "stream cut at %zu of %zu accepted", cuts[i], len);
        free(t);
    }
    uint64_t s = 99;
    for (int k = 0; k < 16; k++) {  // random bytes after a valid preamble
        size_t m = 1000 + 997 * (size_t)k;
        uint8_t *t = malloc(m);
        for (size_t i = 0; i < m; i++) {
            s = s * 6364136223846793005ull + 1442695040888963407ull;
            t[i] = (uint8_t)(s >> 56);
        }
        const uint32_t h = snappy_varint_encode(m * 3, t);
        (void)h;
        int st = snappy_decompress_buffer(t, m, b, m * 3 < n ? m * 3 : n, &got);
        CHECK(st <= 0, "garbage stream %d: status %d", k, st);
        free(t);
    }
    free(a);
    free(c);
    free(b);
}

static void *thread_main(void *arg)
{
    const int t = (int)(intptr_t)arg;
    // 'R' / 'P' keep no shared generator state ('T' builds a global vocabulary)
    round_trip_buffer((size_t)(3 << 20) + 4097 * (size_t)t, t & 1 ? 'R' : 'P', 40 + t);
    return NULL;
}

int main(int argc, char **argv)
{
    const char *mode = argc > 1 ? argv[1] : "nodev";
    check_varints();
    if (!strcmp(mode, "nodev")) {
        check_nodev();
        check_bst();
    } else {
        const size_t sizes[] = {0, 1, 17, 65535, 65536, 65537, 1000000, (size_t)(150 << 20) + 12345};
        for (size_t i = 0; i < sizeof sizes / sizeof *sizes; i++) round_trip_buffer(sizes[i], 'T', 7 + i);
        round_trip_buffer(5 << 20, 'R', 3);
        round_trip_buffer(5 << 20, 'Z', 3);
        round_trip_file(0, 'T', 1, 0);
        round_trip_file(1000000, 'T', 2, 0);
        round_trip_file((size_t)(150 << 20) + 777, 'T', 3, 0);
        round_trip_file((size_t)(70 << 20) + 5, 'T', 4, 1);
        malformed();
        pthread_t th[4];
        for (int t = 0; t < 4; t++) pthread_create(&th[t], NULL, thread_main, (void *)(intptr_t)t);
        for (int t = 0; t < 4; t++) pthread_join(th[t], NULL);
        CHECK(snappy_amd_host_pool_size() >= 1, "pool size");
        CHECK(snappy_amd_host_release() == 0, "release");
    }
    printf("host_check %s: %s (%d failures)\n", mode, g_fail ? "FAIL" : "ok", g_fail);
    if (strcmp(mode, "nodev")) {
        // With a device, run the leak check the exit handlers would run (it exits
        // with LSan's code on a leak), then leave without the HIP runtime's static
        // destructors: under ASan its teardown has died inside libhsa-runtime64
        // (a sanitizer device-allocator CHECK after the runtime unloaded, once in
        // eight runs; profiles/r06ae_gpu_tests.log), after every check here passed
        fflush(stdout);
        fflush(stderr);
        __lsan_do_leak_check();
        _exit(g_fail ? 1 : 0);
    }
    return g_fail ? 1 : 0;
}
