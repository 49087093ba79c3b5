/* Drop-in replacement of src/snappy_compression_tree.h:10 (tturturiello/lightweight-snappy).
 * The BST matcher (-b) is outside the GPU hot path:
 * libsnappy_amd.so writes the reference's -b stream byte for byte on host
 * threads (csrc/bst_host.c). */
#ifndef SNAPPY_SNAPPY_COMPRESSION_TREE_H
#define SNAPPY_SNAPPY_COMPRESSION_TREE_H
#include <stdio.h>
int snappy_compress_bst(FILE *file_input, unsigned long long input_size, FILE *file_compressed);
#endif
