/*
 * snappy_oracle.c -- CPU restatement of the reference Snappy block codec.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * product path.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product library never links it.
 *
 * It restates (clean-room, from SURVEY.md Appendix A and the reference
 * behaviour) the algorithm of tturturiello/lightweight-snappy:
 *   - stream driver       src/snappy_compression.c:414-428
 *   - block match finder  src/snappy_compression.c:384-403 (+ helpers)
 *   - element encoders    src/snappy_compression.c:95-165
 *   - varint              src/varint.c:12-20 (encode), :28-42 (decode)
 *   - decoder             src/snappy_decompression.c:290-363
 * Parity is pinned against the compiled reference itself (oracle/_ref, see
 * oracle/Makefile) through the fixtures in tests/golden/ (gen_golden.py).
 *
 * Differences from the reference that are deliberate and documented:
 *   - the decoder accumulates the stream length in 64 bits (the reference
 *     uses `int`, varint.c:28-42, and mis-decodes streams >= 2^31 bytes);
 *   - the decoder bounds-checks every element and returns an error code
 *     instead of reading/writing outside its buffers
 *     (snappy_decompression.c:262 is a no-op check).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>
#include <pthread.h>

#define ORC_MAX_BLOCK 65536u
#define ORC_MAX_TABLE 4096u

/* LEB128 encode; src/varint.c:12-20 (MSB_mask is a signed char, so the
 * loop condition `n & MSB_mask` is n >= 128). */
uint32_t oracle_varint_encode(uint64_t n, uint8_t *out)
{
    uint32_t k = 0;
    while (n >= 128) {
        out[k++] = (uint8_t)((n & 0x7F) | 0x80);
        n >>= 7;
    }
    out[k++] = (uint8_t)n;
    return k;
}

/* LEB128 decode, 64-bit (hardened form of src/varint.c:28-42).
 * Returns bytes consumed, 0 on truncated / over-long input. */
uint32_t oracle_varint_decode(const uint8_t *in, size_t n, uint64_t *value)
{
    uint64_t v = 0;
    for (uint32_t k = 0; k < 10 && k < n; k++) {
        v |= (uint64_t)(in[k] & 0x7F) << (7 * k);
        if (!(in[k] & 0x80)) { *value = v; return k + 1; }
    }
    return 0;
}

/* Worst-case encoded size of one block of L bytes: every 61+ byte literal
 * followed by a minimal copy gains at most 2 bytes per 65 input bytes. */
size_t oracle_max_block_bytes(uint32_t L)
{
    return (size_t)L + L / 32 + 16;
}

size_t oracle_max_compressed_length(size_t n)
{
    size_t blocks = (n + ORC_MAX_BLOCK - 1) / ORC_MAX_BLOCK;
    return 10 + n + blocks * (ORC_MAX_BLOCK / 32 + 16);
}

/* big-endian 4-byte load; src/snappy_compression.c:239-241 */
static inline uint32_t be32(const uint8_t *p)
{
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

/* literal element; src/snappy_compression.c:95-120 */
static inline uint8_t *emit_literal(uint8_t *o, const uint8_t *src, uint32_t len)
{
    uint32_t m = len - 1;
    if (m < 60) {
        *o++ = (uint8_t)(m << 2);
    } else {
        uint8_t *tag = o++;
        uint32_t code = 59;
        while (m > 0) { *o++ = (uint8_t)(m & 0xFF); m >>= 8; code++; }
        *tag = (uint8_t)(code << 2);
    }
    memcpy(o, src, len);
    return o + len;
}

/* one copy piece (len <= 64); src/snappy_compression.c:131-145 */
static inline uint8_t *emit_piece(uint8_t *o, uint32_t len, uint32_t off)
{
    if (len < 12 && off < 2048) {
        *o++ = (uint8_t)(((off >> 8) << 5) + ((len - 4) << 2) + 1);
        *o++ = (uint8_t)(off & 0xFF);
    } else {
        *o++ = (uint8_t)(((len - 1) << 2) | 2);
        *o++ = (uint8_t)(off & 0xFF);
        *o++ = (uint8_t)((off >> 8) & 0xFF);
    }
    return o;
}

/* copy split 64/60; src/snappy_compression.c:153-165 */
static inline uint8_t *emit_copy(uint8_t *o, uint32_t len, uint32_t off)
{
    while (len > 68) { o = emit_piece(o, 64, off); len -= 64; }
    if (len > 64) { o = emit_piece(o, 60, off); len -= 60; }
    return emit_piece(o, len, off);
}

/* One block (L <= 65536) -> raw Snappy elements.  Restates
 * compress_next_block (src/snappy_compression.c:384-403) with
 * set_htable_size :198-204, is_block_end :229-232, found_match :259-265,
 * update_hash_table :303-307, append_literal :283-287, emit_copy :323-329,
 * find_copy_length :61-72.  Returns bytes written. */
size_t oracle_compress_block(const uint8_t *in, uint32_t L, uint8_t *out)
{
    uint16_t table[ORC_MAX_TABLE];
    uint32_t T = 256, lg = 8;
    while (T < ORC_MAX_TABLE && T < L) { T <<= 1; lg++; }
    const uint32_t shift = 32 - lg;
    memset(table, 0, sizeof(table));

    uint8_t *o = out;
    uint32_t skip = 33;          /* start_new_literal + append_literal */
    uint32_t p = 1;              /* position 0 is never probed */
    uint32_t lit = 0;            /* start of pending literal */
    while (!(L - p < (skip >> 5) + 15)) {
        uint32_t cur = be32(in + p);
        uint32_t h = (cur * 0x1e35a7bdu) >> shift;
        uint32_t cand = table[h];
        if (be32(in + cand) == cur) {
            if (p > lit) o = emit_literal(o, in + lit, p - lit);
            skip = 32;
            uint32_t n = 4;
            while (p + n < L && in[p + n] == in[cand + n]) n++;
            o = emit_copy(o, n, p - cand);
            table[h] = (uint16_t)p;
            p += n;
            lit = p;
        } else {
            table[(be32(in + p - 1) * 0x1e35a7bdu) >> shift] = (uint16_t)(p - 1);
            table[h] = (uint16_t)p;
            p += skip >> 5;
            skip++;
        }
    }
    if (L > lit) o = emit_literal(o, in + lit, L - lit);
    return (size_t)(o - out);
}

/* Whole stream: varint(n) ++ blocks of 65536 bytes; empty input -> empty
 * output (snappy_compression.c:414-428; the header is only flushed with the
 * first block, :417-421). */
size_t oracle_compress(const uint8_t *in, size_t n, uint8_t *out)
{
    if (n == 0) return 0;
    uint8_t *o = out + oracle_varint_encode(n, out);
    for (size_t b = 0; b < n; b += ORC_MAX_BLOCK) {
        uint32_t L = (uint32_t)((n - b) < ORC_MAX_BLOCK ? (n - b) : ORC_MAX_BLOCK);
        o += oracle_compress_block(in + b, L, o);
    }
    return (size_t)(o - out);
}

/* Decoder status codes (match include/snappy_amd.h). */
#define ORC_OK 0
#define ORC_ERR_HEADER (-2)
#define ORC_ERR_TRUNCATED (-3)
#define ORC_ERR_OFFSET (-4)
#define ORC_ERR_OVERRUN (-5)
#define ORC_ERR_CAPACITY (-6)

/* Element loop of src/snappy_decompression.c:290-333 (tag dispatch, copy-1
 * hi bits from (tag>>5), LE 1/2/4-byte offsets, byte-serial overlapping
 * copies :273-280), over an in-memory buffer, decoding exactly `want` bytes
 * into out[0..want).  `base` bytes before `out` may be referenced by copies
 * (0 for a whole stream).  Returns bytes of `in` consumed or <0. */
long long oracle_decode_elements(const uint8_t *in, size_t n, uint8_t *out, size_t want, size_t base)
{
    size_t ip = 0, op = 0;
    while (op < want) {
        if (ip >= n) return ORC_ERR_TRUNCATED;
        uint8_t tag = in[ip++];
        size_t len, off;
        switch (tag & 3) {
        case 0: {
            len = (tag >> 2) + 1;
            if (len > 60) {
                uint32_t k = (uint32_t)len - 60;
                if (ip + k > n) return ORC_ERR_TRUNCATED;
                len = 0;
                for (uint32_t i = 0; i < k; i++) len |= (size_t)in[ip + i] << (8 * i);
                len += 1;
                ip += k;
            }
            if (ip + len > n) return ORC_ERR_TRUNCATED;
            if (op + len > want) return ORC_ERR_OVERRUN;
            memcpy(out + op, in + ip, len);
            ip += len; op += len;
            continue;
        }
        case 1:
            if (ip + 1 > n) return ORC_ERR_TRUNCATED;
            len = ((tag >> 2) & 7) + 4;
            off = ((size_t)(tag >> 5) << 8) | in[ip];
            ip += 1;
            break;
        case 2:
            if (ip + 2 > n) return ORC_ERR_TRUNCATED;
            len = (tag >> 2) + 1;
            off = (size_t)in[ip] | ((size_t)in[ip + 1] << 8);
            ip += 2;
            break;
        default:
            if (ip + 4 > n) return ORC_ERR_TRUNCATED;
            len = (tag >> 2) + 1;
            off = (size_t)in[ip] | ((size_t)in[ip + 1] << 8) | ((size_t)in[ip + 2] << 16) | ((size_t)in[ip + 3] << 24);
            ip += 4;
            break;
        }
        if (off == 0 || off > op + base) return ORC_ERR_OFFSET;
        if (op + len > want) return ORC_ERR_OVERRUN;
        for (size_t i = 0; i < len; i++) out[op + i] = out[op + i - off];
        op += len;
    }
    return (long long)ip;
}

/* snappy_decompress (src/snappy_decompression.c:345-363) over memory.
 * Empty input decodes to empty output. */
int oracle_decompress(const uint8_t *in, size_t n, uint8_t *out, size_t cap, size_t *out_len)
{
    *out_len = 0;
    if (n == 0) return ORC_OK;
    uint64_t N;
    uint32_t h = oracle_varint_decode(in, n, &N);
    if (h == 0) return ORC_ERR_HEADER;
    if (N > cap) return ORC_ERR_CAPACITY;
    long long r = oracle_decode_elements(in + h, n - h, out, (size_t)N, 0);
    if (r < 0) return (int)r;
    *out_len = (size_t)N;
    return ORC_OK;
}

/* ---- "streams" layout: the input cut into `chunk`-byte pieces, each an
 * independent snappy_compress() stream; offsets[i]..offsets[i+1] delimit
 * stream i in the concatenation.  Used for the 1 GiB-of-32 KiB-blocks
 * config (BASELINE.json configs[1]).  Multi-threaded over streams for the
 * all-cores CPU baseline. */
typedef struct {
    const uint8_t *in; size_t n; uint32_t chunk;
    uint8_t *scratch; size_t stride; size_t *sizes;
    const uint8_t *cin; const uint64_t *offs; uint8_t *dout; int *status;
    size_t first, last;
} orc_job;

static void *orc_compress_worker(void *arg)
{
    orc_job *j = (orc_job *)arg;
    for (size_t s = j->first; s < j->last; s++) {
        size_t b = s * j->chunk;
        size_t L = (j->n - b) < j->chunk ? (j->n - b) : j->chunk;
        j->sizes[s] = oracle_compress(j->in + b, L, j->scratch + s * j->stride);
    }
    return NULL;
}

static void *orc_decompress_worker(void *arg)
{
    orc_job *j = (orc_job *)arg;
    for (size_t s = j->first; s < j->last; s++) {
        size_t b = s * j->chunk;
        size_t L = (j->n - b) < j->chunk ? (j->n - b) : j->chunk;
        size_t got = 0;
        int st = oracle_decompress(j->cin + j->offs[s], j->offs[s + 1] - j->offs[s], j->dout + b, L, &got);
        if (st == ORC_OK && got != L) st = ORC_ERR_OVERRUN;
        if (st != ORC_OK) *j->status = st;
    }
    return NULL;
}

static void orc_run(orc_job *proto, size_t nstreams, int nthreads, void *(*fn)(void *))
{
    if (nthreads < 1) nthreads = 1;
    if ((size_t)nthreads > nstreams) nthreads = (int)(nstreams ? nstreams : 1);
    pthread_t th[256];
    orc_job jobs[256];
    if (nthreads > 256) nthreads = 256;
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = *proto;
        jobs[t].first = nstreams * t / nthreads;
        jobs[t].last = nstreams * (t + 1) / nthreads;
        if (nthreads == 1) fn(&jobs[t]);
        else pthread_create(&th[t], NULL, fn, &jobs[t]);
    }
    if (nthreads > 1)
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

/* Returns total bytes written to `out`; offsets has nstreams+1 entries. */
size_t oracle_compress_streams(const uint8_t *in, size_t n, uint32_t chunk, uint8_t *out,
                               uint64_t *offsets, int nthreads)
{
    size_t ns = (n + chunk - 1) / chunk;
    size_t stride = oracle_max_block_bytes(chunk) + 16;
    uint8_t *scratch = (uint8_t *)malloc(ns * stride + 1);
    size_t *sizes = (size_t *)malloc((ns + 1) * sizeof(size_t));
    orc_job job = {0};
    job.in = in; job.n = n; job.chunk = chunk; job.scratch = scratch; job.stride = stride; job.sizes = sizes;
    orc_run(&job, ns, nthreads, orc_compress_worker);
    size_t o = 0;
    for (size_t s = 0; s < ns; s++) {
        offsets[s] = o;
        memcpy(out + o, scratch + s * stride, sizes[s]);
        o += sizes[s];
    }
    offsets[ns] = o;
    free(scratch); free(sizes);
    return o;
}

/* One whole stream (oracle_compress) with its blocks compressed by `nthreads`
 * threads: snappy_compress() resets the table for every block
 * (src/snappy_compression.c:419-425), so block b's output depends on block b's
 * bytes alone and the stream is varint(n) ++ the blocks in order.  Used to
 * check multi-GiB GPU streams bit for bit. */
static void *orc_block_worker(void *arg)
{
    orc_job *j = (orc_job *)arg;
    for (size_t s = j->first; s < j->last; s++) {
        size_t b = s * ORC_MAX_BLOCK;
        uint32_t L = (uint32_t)((j->n - b) < ORC_MAX_BLOCK ? (j->n - b) : ORC_MAX_BLOCK);
        j->sizes[s] = oracle_compress_block(j->in + b, L, j->scratch + s * j->stride);
    }
    return NULL;
}

size_t oracle_compress_threaded(const uint8_t *in, size_t n, uint8_t *out, int nthreads)
{
    if (n == 0) return 0;
    size_t nb = (n + ORC_MAX_BLOCK - 1) / ORC_MAX_BLOCK;
    size_t stride = oracle_max_block_bytes(ORC_MAX_BLOCK) + 16;
    uint8_t *scratch = (uint8_t *)malloc(nb * stride + 1);
    size_t *sizes = (size_t *)malloc(nb * sizeof(size_t));
    orc_job job = {0};
    job.in = in; job.n = n; job.scratch = scratch; job.stride = stride; job.sizes = sizes;
    orc_run(&job, nb, nthreads, orc_block_worker);
    size_t o = oracle_varint_encode(n, out);
    for (size_t s = 0; s < nb; s++) {
        memcpy(out + o, scratch + s * stride, sizes[s]);
        o += sizes[s];
    }
    free(scratch); free(sizes);
    return o;
}

/* Variant that leaves streams in place at a fixed stride (no compaction);
 * used by the timed CPU baseline so the measurement is the codec only. */
void oracle_compress_streams_strided(const uint8_t *in, size_t n, uint32_t chunk, uint8_t *scratch,
                                     size_t stride, size_t *sizes, int nthreads)
{
    size_t ns = (n + chunk - 1) / chunk;
    orc_job job = {0};
    job.in = in; job.n = n; job.chunk = chunk; job.scratch = scratch; job.stride = stride; job.sizes = sizes;
    orc_run(&job, ns, nthreads, orc_compress_worker);
}

int oracle_decompress_streams(const uint8_t *cin, const uint64_t *offsets, size_t n, uint32_t chunk,
                              uint8_t *out, int nthreads)
{
    size_t ns = (n + chunk - 1) / chunk;
    int status = ORC_OK;
    orc_job job = {0};
    job.cin = cin; job.offs = offsets; job.n = n; job.chunk = chunk; job.dout = out; job.status = &status;
    orc_run(&job, ns, nthreads, orc_decompress_worker);
    return status;
}
