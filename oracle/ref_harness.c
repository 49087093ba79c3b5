/*
 * ref_harness.c -- TEST INFRASTRUCTURE ONLY (never shipped, never measured
 * as the product).  Wraps the compiled reference's FILE* API
 * (snappy_compress, src/snappy_compression.c:414; snappy_decompress,
 * src/snappy_decompression.c:345; snappy_compress_bst,
 * src/snappy_compression_tree.c:291) in memory-to-memory calls so that
 * oracle/gen_golden.py can produce golden vectors from the reference itself.
 * Built by oracle/Makefile into oracle/_ref/ from the sources where they lie
 * under /root/reference/src (nothing is copied into this repository).
 */
#include <stdio.h>
#include <string.h>

void snappy_compress(FILE *file_input, unsigned long long input_size, FILE *file_compressed);
int snappy_decompress(FILE *file_input, FILE *file_decompressed);
int snappy_compress_bst(FILE *file_input, unsigned long long input_size, FILE *file_compressed);

static long long run(int mode, const unsigned char *in, size_t n, unsigned char *out, size_t cap)
{
    FILE *fi = tmpfile(), *fo = tmpfile();
    if (!fi || !fo) return -1;
    if (n && fwrite(in, 1, n, fi) != n) return -1;
    fflush(fi);
    rewind(fi);
    if (mode == 0) snappy_compress(fi, n, fo);
    else if (mode == 1) snappy_decompress(fi, fo);
    else snappy_compress_bst(fi, n, fo);
    fflush(fo);
    long long sz = ftell(fo);
    rewind(fo);
    if (sz < 0 || (size_t)sz > cap) { fclose(fi); fclose(fo); return -2; }
    size_t got = fread(out, 1, (size_t)sz, fo);
    fclose(fi);
    fclose(fo);
    return (long long)got;
}

long long ref_compress_mem(const unsigned char *in, size_t n, unsigned char *out, size_t cap) { return run(0, in, n, out, cap); }
long long ref_decompress_mem(const unsigned char *in, size_t n, unsigned char *out, size_t cap) { return run(1, in, n, out, cap); }
long long ref_compress_bst_mem(const unsigned char *in, size_t n, unsigned char *out, size_t cap) { return run(2, in, n, out, cap); }
