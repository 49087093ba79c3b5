/*
 * snappy_host.c -- C host layer of the MI355X Snappy codec: the reference's
 * FILE* entry points, the varint preamble and the host-buffer API, built on
 * the HIP shim (snappy_device.hip).  No compression or decompression of the
 * GPU path runs on the CPU here: every byte goes through the gfx950 kernels
 * (the -b BST mode, a different algorithm, is bst_host.c's host threads).
 *
 * Reference interfaces replaced (tturturiello/lightweight-snappy):
 *   snappy_compress      src/snappy_compression.h:8, .c:414-428
 *   snappy_decompress    src/snappy_decompression.h:15, .c:345-363
 *   snappy_compress_bst  src/snappy_compression_tree.h:10, .c:291-306
 *   parse_to_varint / varint_to_dim   src/varint.c:12-20 / :28-42
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "snappy_amd.h"
#include "snappy_amd_internal.h"

static __thread int g_last_status = SNAPPY_AMD_OK;

int snappy_amd_last_status(void) { return g_last_status; }

uint32_t snappy_varint_encode(uint64_t n, uint8_t *out)
{
    uint32_t k = 0;
    while (n >= 128) {
        out[k++] = (uint8_t)((n & 0x7F) | 0x80);
        n >>= 7;
    }
    out[k++] = (uint8_t)n;
    return k;
}

uint32_t snappy_varint_decode(const uint8_t *in, size_t n, uint64_t *value)
{
    uint64_t v = 0;
    for (uint32_t k = 0; k < 10 && k < n; k++) {
        v |= (uint64_t)(in[k] & 0x7F) << (7 * k);
        if (!(in[k] & 0x80)) {
            *value = v;
            return k + 1;
        }
    }
    return 0;
}

size_t snappy_max_compressed_length(size_t n)
{
    return snappy_amd_max_output(n, SNAPPY_AMD_BLOCK, SNAPPY_AMD_SINGLE) + 16;
}

int snappy_compress_buffer(const uint8_t *in, size_t n, uint8_t *out, size_t *out_len)
{
    if (!out_len || (n && (!in || !out))) return SNAPPY_AMD_ERR_ARG;
    return snappy_amd_host_compress(in, n, (uint64_t)n, out, snappy_max_compressed_length(n), out_len);
}

int snappy_uncompressed_length(const uint8_t *in, size_t n, uint64_t *len)
{
    if (!in || !len) return SNAPPY_AMD_ERR_ARG;
    return snappy_varint_decode(in, n, len) ? SNAPPY_AMD_OK : SNAPPY_AMD_ERR_HEADER;
}

int snappy_decompress_buffer(const uint8_t *in, size_t n, uint8_t *out, size_t cap, size_t *out_len)
{
    if (!out_len || (n && !in)) return SNAPPY_AMD_ERR_ARG;
    return snappy_amd_host_decompress(in, n, out, cap, out_len);
}

/* Read from the current position of f to EOF (the reference reads 65,536-B
 * chunks until fread returns 0: snappy_compression.c:210-213, :419-425). */
static int slurp(FILE *f, uint8_t **buf, size_t *len)
{
    size_t cap = 1 << 20, n = 0;
    uint8_t *b = (uint8_t *)malloc(cap);
    if (!b) return SNAPPY_AMD_ERR_IO;
    for (;;) {
        if (n == cap) {
            cap *= 2;
            uint8_t *nb = (uint8_t *)realloc(b, cap);
            if (!nb) { free(b); return SNAPPY_AMD_ERR_IO; }
            b = nb;
        }
        size_t got = fread(b + n, 1, cap - n, f);
        n += got;
        if (got == 0) break;
    }
    if (ferror(f)) { free(b); return SNAPPY_AMD_ERR_IO; }
    *buf = b;
    *len = n;
    return SNAPPY_AMD_OK;
}

void snappy_compress(FILE *file_input, unsigned long long input_size, FILE *file_compressed)
{
    /* header = the caller's input_size, as the reference writes it; an empty
     * read writes nothing (snappy_compression.c:417-421) */
    int rc = (file_input && file_compressed)
                 ? snappy_amd_host_compress_file(file_input, (uint64_t)input_size, file_compressed, NULL, NULL)
                 : SNAPPY_AMD_ERR_ARG;
    g_last_status = rc;
    if (rc != SNAPPY_AMD_OK) fprintf(stderr, "snappy_compress: error %d\n", rc);
}

/* sidecar index file -> its entries (malloc'd) */
static int read_index(FILE *f, uint64_t **entries, size_t *count)
{
    uint64_t h[3];
    if (fread(h, sizeof(uint64_t), 3, f) != 3 || h[0] != SNAPPY_AMD_IDX_MAGIC) return SNAPPY_AMD_ERR_INDEX;
    if (h[2] > (h[1] >> 16) + 2) return SNAPPY_AMD_ERR_INDEX;
    uint64_t *e = (uint64_t *)malloc((h[2] ? h[2] : 1) * sizeof(uint64_t));
    if (!e) return SNAPPY_AMD_ERR_IO;
    /* exactly count entries: a short file or trailing bytes are refused (as by
     * snappy_amd.read_index) */
    if (fread(e, sizeof(uint64_t), h[2], f) != h[2] || fgetc(f) != EOF) { free(e); return SNAPPY_AMD_ERR_INDEX; }
    *entries = e;
    *count = (size_t)h[2];
    return SNAPPY_AMD_OK;
}

static int decompress_file(FILE *file_input, FILE *idx, FILE *file_decompressed, const char *what)
{
    uint8_t *in = NULL, *out = NULL;
    uint64_t *ent = NULL;
    size_t n = 0, len = 0, count = 0;
    int rc = (file_input && file_decompressed) ? SNAPPY_AMD_OK : SNAPPY_AMD_ERR_ARG;
    if (rc == SNAPPY_AMD_OK && idx) rc = read_index(idx, &ent, &count);
    /* a regular file: the pipelined decoder (chunked reads overlapped with the
     * copies to HBM, chunked copies back overlapped with the writes) */
    if (rc == SNAPPY_AMD_OK) {
        rc = snappy_amd_host_decompress_file(file_input, ent, count, file_decompressed);
        if (rc != SNAPPY_AMD_ERR_UNSUPPORTED) {
            free(ent);
            g_last_status = rc;
            if (rc != SNAPPY_AMD_OK) fprintf(stderr, "%s: error %d\n", what, rc);
            return rc;
        }
        rc = slurp(file_input, &in, &n); /* a pipe: read it whole (the reference's decoder needs fseek anyway) */
    }
    if (rc == SNAPPY_AMD_OK && n > 0) {
        uint64_t N = 0;
        rc = snappy_uncompressed_length(in, n, &N);
        if (rc == SNAPPY_AMD_OK) {
            out = (uint8_t *)malloc(N ? N : 1);
            rc = !out ? SNAPPY_AMD_ERR_IO
                      : idx ? snappy_amd_host_decompress_idx(in, n, ent, count, out, N, &len)
                            : snappy_amd_host_decompress(in, n, out, N, &len);
        }
        if (rc == SNAPPY_AMD_OK && len && fwrite(out, 1, len, file_decompressed) != len) rc = SNAPPY_AMD_ERR_IO;
    }
    free(in);
    free(out);
    free(ent);
    g_last_status = rc;
    if (rc != SNAPPY_AMD_OK) fprintf(stderr, "%s: error %d\n", what, rc);
    return rc;
}

int snappy_decompress(FILE *file_input, FILE *file_decompressed)
{
    return decompress_file(file_input, NULL, file_decompressed, "snappy_decompress");
}

int snappy_decompress_file_indexed(FILE *file_input, FILE *idx, FILE *file_decompressed)
{
    if (!idx) return g_last_status = SNAPPY_AMD_ERR_ARG;
    return decompress_file(file_input, idx, file_decompressed, "snappy_decompress_file_indexed");
}

int snappy_compress_file_indexed(FILE *file_input, unsigned long long input_size, FILE *file_compressed, FILE *idx)
{
    int rc = (file_input && file_compressed && idx)
                 ? snappy_amd_host_compress_file(file_input, (uint64_t)input_size, file_compressed, idx, NULL)
                 : SNAPPY_AMD_ERR_ARG;
    g_last_status = rc;
    if (rc != SNAPPY_AMD_OK) fprintf(stderr, "snappy_compress_file_indexed: error %d\n", rc);
    return rc;
}

int snappy_compress_bst(FILE *file_input, unsigned long long input_size, FILE *file_compressed)
{
    /* the reference's -b stream (snappy_compression_tree.c:291-306), host threads
     * (bst_host.c); header = the caller's input_size, an empty read writes nothing */
    int rc = (file_input && file_compressed)
                 ? snappy_amd_bst_compress_file(file_input, (uint64_t)input_size, file_compressed)
                 : SNAPPY_AMD_ERR_ARG;
    g_last_status = rc;
    if (rc != SNAPPY_AMD_OK) fprintf(stderr, "snappy_compress_bst: error %d\n", rc);
    return rc;
}
