/* Drop-in replacement of src/snappy_decompression.h:15 (tturturiello/lightweight-snappy).
 * Implemented by libsnappy_amd.so on MI355X; see snappy_amd.h. */
#ifndef SNAPPY_SNAPPY_DECOMPRESSION_H
#define SNAPPY_SNAPPY_DECOMPRESSION_H
#include <stdio.h>
int snappy_decompress(FILE *file_input, FILE *file_decompressed);
#endif
