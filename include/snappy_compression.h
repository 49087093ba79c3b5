/* Drop-in replacement of src/snappy_compression.h:8 (tturturiello/lightweight-snappy).
 * Implemented by libsnappy_amd.so on MI355X; see snappy_amd.h. */
#ifndef SNAPPY_SNAPPY_COMPRESSION_H
#define SNAPPY_SNAPPY_COMPRESSION_H
#include <stdio.h>
void snappy_compress(FILE *file_input, unsigned long long input_size, FILE *file_compressed);
#endif
