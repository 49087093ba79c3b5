/* libsnappy_amd_compat.so: the reference's Buffer cursor helpers
 * (include/buffer_compression.h; src/buffer_compression.c:10-34 semantics).
 * They are kept out of libsnappy_amd.so because their names (reset,
 * move_current, init_Buffer) could interpose on an application's own symbols;
 * only code written against the reference's buffer_compression.h links this. */
#include <stdlib.h>

#include "buffer_compression.h"

void init_Buffer(Buffer *bf, unsigned int buffer_size)
{
    char *p = (char *)calloc(buffer_size ? buffer_size : 1, 1);
    bf->beginning = bf->current = p;
    bf->bytes_left = p ? buffer_size : 0;
}

void move_current(Buffer *bf, unsigned int offset)
{
    bf->current += offset;
    bf->bytes_left -= offset;
}

void reset(Buffer *bf) { bf->current = bf->beginning; }
