/*
 * bst_host.c -- the reference's `-b` compressor, snappy_compress_bst
 * (src/snappy_compression_tree.c:291-306, its matcher src/BST.c:30-82),
 * restated for the host: the blocks are independent, so a pool of host threads
 * compresses them side by side and the bytes are written in block order.
 *
 * What the reference computes (the output is its, byte for byte):
 *   - the stream is varint(input_size) + the compressed 65,536-byte blocks
 *     (:293-303); the preamble sits in the first block's output buffer, so an
 *     empty input writes nothing (as snappy_compress does);
 *   - a block keeps 4,096 binary search trees indexed by the multiplicative
 *     hash of the 4 bytes at a position (:68-71, :137-143) and keyed by those 4
 *     bytes (BST.c:30-43); a probe looks its 4 bytes up in their tree (:174-180).
 *     A tree holds only values of its own hash, so the trees together are one
 *     dictionary from a 4-byte value to a position -- the bucket never changes a
 *     result, and a hash map keyed by the value reproduces every lookup:
 *       * a miss at p inserts p - 1 and p (:204-208), each only if its value is
 *         not present yet (BST.c:37-41: an equal key leaves the node alone);
 *       * a hit at p copies from the stored position, emits the pending
 *         literal, the copy (length 4 + the common prefix up to the block end,
 *         :55-66, :216-223, written as 64/60-byte pieces :113-125), and then
 *         stores p as the value's position (:221) -- no other inserts;
 *       * the skip / end test / literal bookkeeping are snappy_compress's
 *         (:154-157, :182-199, :269-288): first probe at 1, step skip >> 5;
 *   - the trees are emptied after every block (:234-239; the table size only
 *     shrinks at the last block, so every tree a block used is emptied).
 * No GPU is involved: this mode is not the north-star path.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "snappy_amd.h"
#include "snappy_amd_internal.h"

#define BST_BLOCK 65536u
#define BST_SLOTS_LOG 17                        /* >= 2 x the 65,536 values a block can insert */
#define BST_SLOTS (1u << BST_SLOTS_LOG)
#define BST_BLOCK_OUT (BST_BLOCK + BST_BLOCK / 32 + 64)  /* literal-only worst case + tags */
#define BST_CHUNK_BLOCKS 512u                   /* 32 MiB of input per read */

/* value -> position map of one block: open addressing, the block's
 * generation stamp marks live slots (no clearing between blocks) */
typedef struct {
    uint32_t *key, *pos, *gen;
    uint32_t cur;
} bst_map;

static int map_init(bst_map *m)
{
    m->key = (uint32_t *)malloc(BST_SLOTS * sizeof(uint32_t));
    m->pos = (uint32_t *)malloc(BST_SLOTS * sizeof(uint32_t));
    m->gen = (uint32_t *)calloc(BST_SLOTS, sizeof(uint32_t));
    m->cur = 0;
    return m->key && m->pos && m->gen ? 0 : -1;
}

static void map_free(bst_map *m)
{
    free(m->key);
    free(m->pos);
    free(m->gen);
}

static void map_new_block(bst_map *m)
{
    if (++m->cur == 0) { /* stamp wrapped: clear once every 2^32 blocks */
        memset(m->gen, 0, BST_SLOTS * sizeof(uint32_t));
        m->cur = 1;
    }
}

/* slot of value v: its own if present, else the empty slot it would take */
static inline uint32_t map_slot(const bst_map *m, uint32_t v, int *found)
{
    uint32_t s = (v * 0x9E3779B1u) >> (32 - BST_SLOTS_LOG);
    for (;;) {
        if (m->gen[s] != m->cur) { *found = 0; return s; }
        if (m->key[s] == v) { *found = 1; return s; }
        s = (s + 1) & (BST_SLOTS - 1);
    }
}

static inline void map_insert_absent(bst_map *m, uint32_t v, uint32_t p)
{
    int found;
    const uint32_t s = map_slot(m, v, &found);
    if (found) return;
    m->gen[s] = m->cur;
    m->key[s] = v;
    m->pos[s] = p;
}

static inline uint32_t be32(const uint8_t *p)
{
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

static inline uint8_t *put_literal(uint8_t *o, const uint8_t *src, uint32_t len)
{
    uint32_t m = len - 1;
    if (m < 60) {
        *o++ = (uint8_t)(m << 2);
    } else {
        uint8_t *tag = o++;
        uint32_t code = 59;
        while (m > 0) {
            *o++ = (uint8_t)m;
            m >>= 8;
            code++;
        }
        *tag = (uint8_t)(code << 2);
    }
    memcpy(o, src, len);
    return o + len;
}

static inline uint8_t *put_one_copy(uint8_t *o, uint32_t len, uint32_t off)
{
    if (len < 12 && off < 2048) {
        *o++ = (uint8_t)(((off >> 8) << 5) + ((len - 4) << 2) + 1);
        *o++ = (uint8_t)off;
    } else {
        *o++ = (uint8_t)(((len - 1) << 2) | 2);
        *o++ = (uint8_t)off;
        *o++ = (uint8_t)(off >> 8);
    }
    return o;
}

static inline uint8_t *put_copy(uint8_t *o, uint32_t len, uint32_t off)
{
    while (len > 68) {
        o = put_one_copy(o, 64, off);
        len -= 64;
    }
    if (len > 64) {
        o = put_one_copy(o, 60, off);
        len -= 60;
    }
    return put_one_copy(o, len, off);
}

/* one block of L (1..65,536) bytes -> its elements at o; returns the end */
static uint8_t *bst_block(bst_map *m, const uint8_t *in, uint32_t L, uint8_t *o)
{
    map_new_block(m);
    uint32_t skip = 32, p, lit;
    /* the block starts with a literal: one append (:271-272) */
    p = skip++ >> 5;
    lit = p;
    for (;;) {
        /* is_block_end (:154-157): the end test consumes one skip increment */
        if (L - p < (skip++ >> 5) + 15) break;
        const uint32_t v = be32(in + p);
        int found;
        const uint32_t s = map_slot(m, v, &found);
        if (found) {
            const uint32_t c = m->pos[s];
            if (lit) o = put_literal(o, in + p - lit, lit);
            lit = 0;
            skip = 32;
            uint32_t len = 4;
            while (p + len < L && in[p + len] == in[c + len]) len++;
            o = put_copy(o, len, p - c);
            m->pos[s] = p;
            p += len;
        } else {
            map_insert_absent(m, be32(in + p - 1), p - 1);
            /* v is absent (the lookup missed); p - 1's insert may have added it */
            map_insert_absent(m, v, p);
            const uint32_t step = skip++ >> 5;
            lit += step;
            p += step;
        }
    }
    lit += L - p;
    if (lit) o = put_literal(o, in + L - lit, lit);
    return o;
}

/* ---- the block pool ---------------------------------------------------- */
typedef struct {
    const uint8_t *in;
    size_t n;             /* bytes of this chunk */
    uint8_t *out;         /* BST_BLOCK_OUT per block */
    uint32_t *len;        /* output bytes per block */
    uint32_t nblk;
    uint32_t next;        /* next block to take (under mu) */
    pthread_mutex_t mu;
} bst_job;

typedef struct {
    bst_job *job;
    bst_map map;
} bst_worker;

static void *bst_run(void *arg)
{
    bst_worker *w = (bst_worker *)arg;
    bst_job *j = w->job;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        const uint32_t b = j->next < j->nblk ? j->next++ : j->nblk;
        pthread_mutex_unlock(&j->mu);
        if (b >= j->nblk) break;
        const size_t at = (size_t)b * BST_BLOCK;
        const uint32_t L = (uint32_t)(j->n - at < BST_BLOCK ? j->n - at : BST_BLOCK);
        uint8_t *o = j->out + (size_t)b * BST_BLOCK_OUT;
        j->len[b] = (uint32_t)(bst_block(&w->map, j->in + at, L, o) - o);
    }
    return NULL;
}

static int bst_threads(void)
{
    const char *e = getenv("SNAPPY_AMD_BST_THREADS");
    long t = e ? strtol(e, NULL, 10) : sysconf(_SC_NPROCESSORS_ONLN);
    if (t < 1) t = 1;
    if (t > 16) t = 16; /* the GPU box's CPU share */
    return (int)t;
}

/* compress n bytes (whole blocks except possibly the last) with `nt` workers */
static int bst_chunk(bst_worker *w, int nt, const uint8_t *in, size_t n, uint8_t *out, uint32_t *len)
{
    bst_job job;
    memset(&job, 0, sizeof(job));
    job.in = in;
    job.n = n;
    job.out = out;
    job.len = len;
    job.nblk = (uint32_t)((n + BST_BLOCK - 1) / BST_BLOCK);
    pthread_mutex_init(&job.mu, NULL);
    const int use = (uint32_t)nt < job.nblk ? nt : (int)job.nblk;
    pthread_t tid[16];
    int started = 0;
    for (int t = 1; t < use; t++) {
        w[t].job = &job;
        if (pthread_create(&tid[t], NULL, bst_run, &w[t]) != 0) break;
        started = t;
    }
    w[0].job = &job;
    bst_run(&w[0]);
    for (int t = 1; t <= started; t++) pthread_join(tid[t], NULL);
    pthread_mutex_destroy(&job.mu);
    return SNAPPY_AMD_OK;
}

int snappy_compress_bst_buffer(const uint8_t *in, size_t n, uint8_t *out, size_t cap, size_t *out_len)
{
    if (!out_len || (n && (!in || !out))) return SNAPPY_AMD_ERR_ARG;
    *out_len = 0;
    if (n == 0) return SNAPPY_AMD_OK; /* no block: not even the preamble is written */
    const int nt = bst_threads();
    bst_worker w[16];
    int rc = SNAPPY_AMD_OK, made = 0;
    for (; made < nt; made++)
        if (map_init(&w[made].map)) { map_free(&w[made].map); rc = SNAPPY_AMD_ERR_IO; break; }
    const size_t per = (size_t)BST_CHUNK_BLOCKS * BST_BLOCK;
    uint8_t *stage = rc ? NULL : (uint8_t *)malloc((size_t)BST_CHUNK_BLOCKS * BST_BLOCK_OUT);
    uint32_t *len = rc ? NULL : (uint32_t *)malloc(BST_CHUNK_BLOCKS * sizeof(uint32_t));
    if (!rc && (!stage || !len)) rc = SNAPPY_AMD_ERR_IO;
    size_t o = 0;
    if (!rc) {
        uint8_t hdr[10];
        const uint32_t h = snappy_varint_encode((uint64_t)n, hdr);
        if (h > cap) rc = SNAPPY_AMD_ERR_CAPACITY;
        else { memcpy(out, hdr, h); o = h; }
    }
    for (size_t at = 0; !rc && at < n; at += per) {
        const size_t m = n - at < per ? n - at : per;
        bst_chunk(w, made, in + at, m, stage, len);
        const uint32_t nblk = (uint32_t)((m + BST_BLOCK - 1) / BST_BLOCK);
        for (uint32_t b = 0; b < nblk && !rc; b++) {
            if (o + len[b] > cap) { rc = SNAPPY_AMD_ERR_CAPACITY; break; }
            memcpy(out + o, stage + (size_t)b * BST_BLOCK_OUT, len[b]);
            o += len[b];
        }
    }
    for (int t = 0; t < made; t++) map_free(&w[t].map);
    free(stage);
    free(len);
    if (!rc) *out_len = o;
    return rc;
}

int snappy_amd_bst_compress_file(FILE *fin, uint64_t header_value, FILE *fout)
{
    const int nt = bst_threads();
    bst_worker w[16];
    int rc = SNAPPY_AMD_OK, made = 0;
    for (; made < nt; made++)
        if (map_init(&w[made].map)) { map_free(&w[made].map); rc = SNAPPY_AMD_ERR_IO; break; }
    const size_t per = (size_t)BST_CHUNK_BLOCKS * BST_BLOCK;
    uint8_t *in = rc ? NULL : (uint8_t *)malloc(per);
    uint8_t *stage = rc ? NULL : (uint8_t *)malloc((size_t)BST_CHUNK_BLOCKS * BST_BLOCK_OUT);
    uint32_t *len = rc ? NULL : (uint32_t *)malloc(BST_CHUNK_BLOCKS * sizeof(uint32_t));
    if (!rc && (!in || !stage || !len)) rc = SNAPPY_AMD_ERR_IO;
    int first = 1;
    while (!rc) {
        /* the reference reads 65,536-byte blocks until fread returns 0 (:145-148, :297) */
        size_t m = 0;
        while (m < per) {
            const size_t got = fread(in + m, 1, per - m, fin);
            if (got == 0) break;
            m += got;
        }
        if (ferror(fin)) { rc = SNAPPY_AMD_ERR_IO; break; }
        if (m == 0) break;
        if (first) {
            uint8_t hdr[10];
            const uint32_t h = snappy_varint_encode(header_value, hdr);
            if (fwrite(hdr, 1, h, fout) != h) { rc = SNAPPY_AMD_ERR_IO; break; }
            first = 0;
        }
        bst_chunk(w, made, in, m, stage, len);
        const uint32_t nblk = (uint32_t)((m + BST_BLOCK - 1) / BST_BLOCK);
        for (uint32_t b = 0; b < nblk; b++)
            if (fwrite(stage + (size_t)b * BST_BLOCK_OUT, 1, len[b], fout) != len[b]) { rc = SNAPPY_AMD_ERR_IO; break; }
        if (m < per) break;
    }
    for (int t = 0; t < made; t++) map_free(&w[t].map);
    free(in);
    free(stage);
    free(len);
    return rc;
}
