/*
 * cmd.c -- `snappy [-c|-b|-d] [-r] infile outfile`, the CLI of the reference
 * (src/cmd.c:19-105: same flags, same last-two-argv file names, usage +
 * exit(1) on argc < 4), linked against the MI355X library instead of the CPU
 * codec.  -r prints sizes, ratio and MB/s (MB = 1e6 B, wall clock).
 * -i (an addition): with -c also write the sidecar block
 * index <outfile>.idx; with -d decode with <infile>.idx instead of the GPU
 * index pass.
 */
#include <errno.h>
#include <getopt.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "snappy_amd.h"

static void usage(void)
{
    fprintf(stderr,
            "snappy [-c|-d|-b] [-r] [-i] [infile] [outfile]\n"
            "-c compress (MI355X)\n"
            "-b compress with the BST matcher (not supported on MI355X)\n"
            "-d decompress (MI355X)\n"
            "-r print results\n"
            "-i -c: also write outfile.idx (block index); -d: use infile.idx\n");
    exit(EXIT_FAILURE);
}

static FILE *open_or_die(const char *name, const char *mode)
{
    FILE *f = fopen(name, mode);
    if (!f) {
        fprintf(stderr, "cannot open %s: %s\n", name, strerror(errno));
        exit(EXIT_FAILURE);
    }
    return f;
}

static unsigned long long file_size(FILE *f)
{
    fseek(f, 0, SEEK_END);
    long s = ftell(f);
    fseek(f, 0, SEEK_SET);
    return s < 0 ? 0 : (unsigned long long)s;
}

int main(int argc, char *argv[])
{
    enum { M_COMPRESS, M_BST, M_DECOMPRESS } mode = M_COMPRESS;
    int show = 0, indexed = 0, opt;
    if (argc < 4) usage();
    while ((opt = getopt(argc, argv, "cbdri")) != -1) {
        if (opt == 'c') mode = M_COMPRESS;
        else if (opt == 'b') mode = M_BST;
        else if (opt == 'd') mode = M_DECOMPRESS;
        else if (opt == 'r') show = 1;
        else if (opt == 'i') indexed = 1;
        else usage();
    }
    if (indexed && mode == M_BST) usage();  /* -b writes no block index */
    const char *in_name = argv[argc - 2], *out_name = argv[argc - 1];
    FILE *in = open_or_die(in_name, "rb");
    FILE *out = open_or_die(out_name, "wb");
    unsigned long long in_size = file_size(in);
    FILE *idx = NULL;
    char name[4096] = "";
    if (indexed) {
        snprintf(name, sizeof(name), "%s.idx", mode == M_COMPRESS ? out_name : in_name);
        idx = open_or_die(name, mode == M_COMPRESS ? "wb" : "rb");
    }

    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    int rc = 0;
    if (mode == M_COMPRESS && idx) {
        rc = snappy_compress_file_indexed(in, in_size, out, idx);
    } else if (mode == M_COMPRESS) {
        snappy_compress(in, in_size, out);
        rc = snappy_amd_last_status();
    } else if (mode == M_BST) {
        rc = snappy_compress_bst(in, in_size, out);
    } else if (idx) {
        rc = snappy_decompress_file_indexed(in, idx, out);
    } else {
        rc = snappy_decompress(in, out);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    fclose(in);
    fclose(out);
    if (idx) fclose(idx);
    if (rc != 0 && idx && mode == M_COMPRESS) remove(name);  /* no partial index left behind */
    double secs = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
    if (show) {
        FILE *o = open_or_die(out_name, "rb");
        unsigned long long out_size = file_size(o);
        fclose(o);
        unsigned long long raw = mode == M_DECOMPRESS ? out_size : in_size;
        printf("input %llu bytes, output %llu bytes\n", in_size, out_size);
        if (mode != M_DECOMPRESS && out_size) printf("ratio %f\n", (double)in_size / (double)out_size);
        printf("%f s, %f MB/s (uncompressed bytes)\n", secs, secs > 0 ? raw / (secs * 1e6) : 0.0);
    }
    return rc == 0 ? 0 : 1;
}
