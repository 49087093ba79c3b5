/* Drop-in replacement of src/buffer_compression.h:8-16 (tturturiello/lightweight-snappy):
 * the byte-cursor helpers the reference's block loop is written with.  The MI355X codec
 * keeps its own cursors on the device; these host helpers live in the separate
 * libsnappy_amd_compat.so (not libsnappy_amd.so: their generic names could interpose on
 * an application's symbols), for code built against the reference header. */
#ifndef SNAPPY_BUFFER_COMPRESSION_H
#define SNAPPY_BUFFER_COMPRESSION_H
typedef struct buffer {
    char *current;          /* next byte */
    char *beginning;        /* start of the allocation */
    unsigned int bytes_left;
} Buffer;
/* zero-filled allocation of buffer_size bytes, cursor at its start (buffer_compression.c:10-14) */
void init_Buffer(Buffer *bf, unsigned int buffer_size);
/* advance the cursor, shrinking bytes_left (buffer_compression.c:22-25) */
void move_current(Buffer *bf, unsigned int offset);
/* rewind the cursor; bytes_left is left as is, as in the reference (buffer_compression.c:32-34) */
void reset(Buffer *bf);
#endif
