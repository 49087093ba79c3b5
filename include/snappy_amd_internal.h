/*
 * snappy_amd_internal.h -- host-buffer and FILE* entry points of the host
 * pipelines (snappy_pipeline.cpp, over the HIP shim snappy_device.hip) and of
 * the -b compressor (bst_host.c) that the C host layer (snappy_host.c) builds
 * the reference FILE* API on.  Exported for the host layer; not part of the
 * documented drop-in surface.
 */
#ifndef SNAPPY_AMD_INTERNAL_H
#define SNAPPY_AMD_INTERNAL_H
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#ifdef __cplusplus
extern "C" {
#endif
/* One SINGLE-layout stream of in[0..n) whose preamble encodes
 * header_value (snappy_compress writes its input_size argument, which the
 * reference never checks against the bytes read: snappy_compression.c:171). */
int snappy_amd_host_compress(const uint8_t *in, size_t n, uint64_t header_value, uint8_t *out, size_t cap,
                             size_t *out_len);
int snappy_amd_host_decompress(const uint8_t *in, size_t n, uint8_t *out, size_t cap, size_t *out_len);
/* the same with a sidecar block index (count entries) instead of the index pass */
int snappy_amd_host_decompress_idx(const uint8_t *in, size_t n, const uint64_t *idx, size_t count, uint8_t *out,
                                   size_t cap, size_t *out_len);
/* Streaming form of snappy_compress(): reads fin from its current position
 * to EOF in 64 MiB chunks, writes the same bytes as the whole-input call
 * (varint(header_value) ++ blocks) to fout, and (fidx != NULL) the sidecar
 * index of snappy_amd.h to fidx; *bytes_in = bytes read. */
int snappy_amd_host_compress_file(FILE *fin, uint64_t header_value, FILE *fout, FILE *fidx, uint64_t *bytes_in);
/* Pipelined snappy_decompress(): fin (a regular file, from its current
 * position to EOF) is read in 64 MiB chunks by several threads into pinned
 * staging and copied to HBM while the next chunk is read; the block index is
 * the sidecar's (idx/count, checked) or built on the GPU; the decoded bytes
 * come back in 64 MiB chunks written (positional writes when fout is a
 * regular file, fwrite otherwise) while the next chunk is copied down.
 * SNAPPY_AMD_ERR_UNSUPPORTED if fin is not a regular file (the caller then
 * reads it whole and uses snappy_amd_host_decompress[_idx]). */
int snappy_amd_host_decompress_file(FILE *fin, const uint64_t *idx, size_t count, FILE *fout);
/* snappy_compress_bst's stream: fin from its current position to EOF,
 * varint(header_value) ++ the BST-matcher blocks to fout (bst_host.c) */
int snappy_amd_bst_compress_file(FILE *fin, uint64_t header_value, FILE *fout);
#ifdef __cplusplus
}
#endif
#endif
