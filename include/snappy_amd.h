/*
 * snappy_amd.h -- C ABI of the MI355X-native Snappy block codec.
 *
 * The drop-in entry points keep the reference signatures exactly
 * (declared again in snappy_compression.h / snappy_decompression.h /
 * snappy_compression_tree.h so src/cmd.c compiles unchanged):
 *
 *   snappy_compress      <- src/snappy_compression.h:8   (def .c:414-428)
 *   snappy_decompress    <- src/snappy_decompression.h:15 (def .c:345-363)
 *   snappy_compress_bst  <- src/snappy_compression_tree.h:10 (def .c:291-306)
 *
 * Added below them: an in-memory host-buffer API and a
 * device-resident (HBM pointer) batch API.  All compute runs in hand-written
 * HIP kernels for gfx950; there is no CPU fallback in this library.  (The
 * reference's -b BST compressor, a different algorithm with different output
 * and not the GPU path, runs on host threads: snappy_compress_bst.)  Every
 * function returns 0 (SNAPPY_AMD_OK) or a negative error code.
 */
#ifndef SNAPPY_AMD_H
#define SNAPPY_AMD_H

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------- */
#define SNAPPY_AMD_OK 0
#define SNAPPY_AMD_ERR_ARG (-1)        /* bad argument (NULL, chunk > 65536, ...) */
#define SNAPPY_AMD_ERR_HEADER (-2)     /* unreadable varint length preamble      */
#define SNAPPY_AMD_ERR_TRUNCATED (-3)  /* element runs past the end of its input  */
#define SNAPPY_AMD_ERR_OFFSET (-4)     /* copy offset 0 or before the block start */
#define SNAPPY_AMD_ERR_OVERRUN (-5)    /* element runs past the declared length   */
#define SNAPPY_AMD_ERR_CAPACITY (-6)   /* caller's output buffer too small        */
#define SNAPPY_AMD_ERR_DEVICE (-7)     /* HIP runtime error / no device           */
#define SNAPPY_AMD_ERR_IO (-8)         /* FILE* read/write failure                */
#define SNAPPY_AMD_ERR_UNSUPPORTED (-9)
#define SNAPPY_AMD_ERR_TIMEOUT (-10)   /* a block waited too long for an earlier one  */
#define SNAPPY_AMD_ERR_INDEX (-11)     /* a sidecar index that does not fit the stream */

/* Block size of the reference stream format (src/snappy_compression.c:9). */
#define SNAPPY_AMD_BLOCK 65536u

/* Stream layouts handled by the batch API. */
#define SNAPPY_AMD_SINGLE 0  /* one stream: varint(n) ++ 65536-byte blocks       */
#define SNAPPY_AMD_STREAMS 1 /* n cut into `chunk`-byte pieces, each one stream  */

/* ---- drop-in FILE* API (reference signatures) ------------------------ */
void snappy_compress(FILE *file_input, unsigned long long input_size, FILE *file_compressed);
int snappy_decompress(FILE *file_input, FILE *file_decompressed);
/* the -b mode: the reference's BST-matcher stream, byte for byte, computed by
 * a pool of host threads (<= 16, SNAPPY_AMD_BST_THREADS), one block each */
int snappy_compress_bst(FILE *file_input, unsigned long long input_size, FILE *file_compressed);

/* Status of the last snappy_compress / snappy_decompress call on this
 * thread (the reference signatures cannot return one). */
int snappy_amd_last_status(void);

/* The compile-time knobs of the library's gfx950 kernels, e.g.
 * "compress{measurement=0 k1r_dmax=10 ...} decode{measurement=0 k4_nofar=0 ...}".
 * measurement=1 marks a build that may write wrong bytes (timing experiments)
 * or carries statistics code: never a product library. */
const char *snappy_amd_build_config(void);

/* Sidecar block index (the stream format has no block
 * markers).  File layout, little-endian u64 words: SNAPPY_AMD_IDX_MAGIC, N
 * (decoded bytes), count = ceil(N/65536) + 1, then `count` block-index
 * entries in the format of snappy_amd_decompress_device below (byte offsets
 * from the start of the stream, its varint preamble included; the last entry
 * is the stream length).  With it, decoding skips the index pass. */
#define SNAPPY_AMD_IDX_MAGIC 0x3158444941504e53ull /* "SNPAIDX1" */
/* snappy_compress() that also writes the sidecar index of its output to idx */
int snappy_compress_file_indexed(FILE *file_input, unsigned long long input_size, FILE *file_compressed, FILE *idx);
/* snappy_decompress() using a sidecar index.  SNAPPY_AMD_ERR_INDEX if the
 * index is not this stream's own block index: a malformed file (magic, count,
 * an entry outside the stream or decreasing) is refused before any decoding;
 * an entry moved off an element boundary is refused by the decode (each
 * block's element chain must end exactly at the next entry), and a decode
 * that fails for any other reason is checked against the stream's own index
 * (GPU index pass): a different sidecar -> ERR_INDEX, the same -> the
 * stream's error, as snappy_decompress reports it.  Success implies the
 * sidecar was the stream's index and the output is snappy_decompress's. */
int snappy_decompress_file_indexed(FILE *file_input, FILE *idx, FILE *file_decompressed);

/* ---- varint preamble (src/varint.c) ---------------------------------- */
/* LEB128 of n into out (<= 10 bytes); returns bytes written. varint.c:12-20 */
uint32_t snappy_varint_encode(uint64_t n, uint8_t *out);
/* 64-bit LEB128 decode; returns bytes consumed or 0. (varint.c:28-42 uses
 * `int` and overflows at 2^31; this one does not.) */
uint32_t snappy_varint_decode(const uint8_t *in, size_t n, uint64_t *value);

/* ---- host-memory API -------------------------------------------------- */
/* Upper bound of snappy_compress output for n input bytes. */
size_t snappy_max_compressed_length(size_t n);
/* Same bytes as snappy_compress() on a FILE holding in[0..n); n == 0 gives
 * 0 bytes.  out must hold snappy_max_compressed_length(n). */
int snappy_compress_buffer(const uint8_t *in, size_t n, uint8_t *out, size_t *out_len);
/* Same bytes as snappy_compress_bst() on a FILE holding in[0..n) (the -b
 * stream; snappy_decompress_buffer decodes it).  out must hold
 * snappy_max_compressed_length(n); n == 0 gives 0 bytes. */
int snappy_compress_bst_buffer(const uint8_t *in, size_t n, uint8_t *out, size_t cap, size_t *out_len);
/* Decode one stream; *out_len = declared length. */
int snappy_decompress_buffer(const uint8_t *in, size_t n, uint8_t *out, size_t cap, size_t *out_len);
int snappy_uncompressed_length(const uint8_t *in, size_t n, uint64_t *len);

/* Threads and devices of the host-memory and FILE* calls above.  Each call
 * leases a pooled host context (its own streams, device scratch and pinned
 * staging) of the calling thread's device and returns it when it ends, so
 * calls from several threads run concurrently.  The device is the one set
 * here for the calling thread (-1: back to the default), else the
 * SNAPPY_AMD_DEVICE environment variable (read once), else 0. */
int snappy_amd_host_set_device(int device);
int snappy_amd_host_get_device(void);
/* Free every idle pooled host context (device scratch and pinned staging). */
int snappy_amd_host_release(void);
/* Idle host contexts in the pool (diagnostics). */
size_t snappy_amd_host_pool_size(void);

/* The host-memory API over several devices (a device may be listed more
 * than once).  Compress: the input's 65,536-byte blocks are split into one
 * contiguous range per device (the first range writes the preamble), each
 * compressed on its device by its own thread; once every range's size is
 * known (C1) each device copies its bytes to their place in out (C2).  The
 * bytes equal snappy_compress_buffer's; out must hold
 * snappy_max_compressed_length(n).  Decompress: the first device builds the
 * block index, every device decodes one range of blocks from its part of the
 * stream; a stream whose ranges are not self-contained (elements straddling a
 * range start, copies reaching an earlier range) is decoded whole on the
 * first device instead, so the results equal snappy_decompress_buffer's. */
int snappy_compress_buffer_multi(const int *devices, int ndev, const uint8_t *in, size_t n, uint8_t *out,
                                 size_t *out_len);
int snappy_decompress_buffer_multi(const int *devices, int ndev, const uint8_t *in, size_t n, uint8_t *out,
                                   size_t cap, size_t *out_len);

/* ---- device-resident batch API (all pointers are HBM) ----------------- */
typedef struct snappy_amd_ctx snappy_amd_ctx;

int snappy_amd_create(int device, snappy_amd_ctx **ctx);
void snappy_amd_destroy(snappy_amd_ctx *ctx);
/* Launch on this hipStream_t (NULL = the context's own stream, a blocking
 * stream: ordered after work queued on the legacy default stream). */
int snappy_amd_set_stream(snappy_amd_ctx *ctx, void *hip_stream);
void *snappy_amd_get_stream(snappy_amd_ctx *ctx);

/* Device bytes the context holds as scratch (token lists, segment records,
 * status words, staging of the host-buffer path, index scratch); it grows to
 * the largest call made and is kept. */
size_t snappy_amd_device_bytes(snappy_amd_ctx *ctx);
/* Release the scratch above (synchronises the context stream); the next call
 * allocates again.  The status words of a decode whose status has not been
 * read yet (decompress_device_async) are kept until it is read.  Used to make
 * room in HBM between phases (bench.py trims before C3, the all-gather of the
 * decoded shards, and between its sub-workloads). */
int snappy_amd_trim(snappy_amd_ctx *ctx);

/* Options of a context (snappy_amd_set_option). */
#define SNAPPY_AMD_OPT_SERIAL_INDEX 1 /* 1: index_device walks the stream with one wave
                                         (the chunk-parallel K5p pass otherwise) */
#define SNAPPY_AMD_OPT_K1R_EXTRA_LDS 2 /* bytes of extra dynamic LDS per K1r unit
                                          (occupancy experiments; default 0) */
int snappy_amd_set_option(snappy_amd_ctx *ctx, int option, int64_t value);

/* Number of units (blocks or streams) for n bytes in a layout. */
size_t snappy_amd_num_units(size_t n, uint32_t chunk, int layout);
/* Capacity d_out must have for compress_device. */
size_t snappy_amd_max_output(size_t n, uint32_t chunk, int layout);

/* Compress d_in[0..n).  layout SINGLE: one stream equal to snappy_compress()
 * (chunk ignored, blocks of 65536).  layout STREAMS: ceil(n/chunk)
 * independent streams, each equal to snappy_compress() of its chunk
 * (1 <= chunk <= 65536), concatenated.  d_offsets (nunits+1 u64, device)
 * receives each unit's byte offset in d_out -- the block index that lets
 * decompress_device run block-parallel.  *out_len (host) gets the total.
 * Asynchronous on the context stream except for the 8-byte total read. */
int snappy_amd_compress_device(snappy_amd_ctx *ctx, const void *d_in, size_t n, uint32_t chunk,
                               int layout, void *d_out, uint64_t *d_offsets, size_t *out_len);

/* Flags for the _ex forms. */
#define SNAPPY_AMD_NO_PREAMBLE 1u /* SINGLE layout: this buffer continues a stream
                                     (a rank > 0 shard): no varint preamble */

/* compress_device with an explicit preamble value and flags; a SINGLE-layout
 * stream sharded over ranks is rank 0 with header_value = the global length
 * and flags 0, every other rank with SNAPPY_AMD_NO_PREAMBLE (n must then be a
 * multiple of 65536 on every rank but the last). */
int snappy_amd_compress_device_ex(snappy_amd_ctx *ctx, const void *d_in, size_t n, uint32_t chunk, int layout,
                                  uint32_t flags, uint64_t header_value, void *d_out, uint64_t *d_offsets,
                                  size_t *out_len);

/* Block index entries (d_offsets, nunits+1 u64): bits [0,40) = byte offset in
 * the stream of the element holding the unit's first output byte; bits
 * [40,64) = how many output bytes of that element precede the unit (0 when
 * the element starts the unit -- always the case for streams this library
 * writes, whose entries are therefore plain offsets).  The last entry is the
 * stream's end.  Non-zero skips arise only in foreign SINGLE streams whose
 * elements cross 65,536-byte output boundaries (snappy_amd_index_device). */
#define SNAPPY_AMD_IDX_OFFSET_BITS 40

/* Decode what compress_device produced (or any stream whose block index is
 * given): n = total decoded bytes, d_offsets = the unit index.  SINGLE
 * layout decodes any valid stream: elements may straddle blocks and copies
 * may reach into earlier blocks (those blocks run in a second, ordered pass).
 * Returns the first failing unit's status (synchronises to read it). */
int snappy_amd_decompress_device(snappy_amd_ctx *ctx, const void *d_comp, const uint64_t *d_offsets,
                                 size_t n, uint32_t chunk, int layout, void *d_out);

/* Same as decompress_device without the status read-back (fully async);
 * fetch the status later with snappy_amd_decompress_status. */
int snappy_amd_decompress_device_async(snappy_amd_ctx *ctx, const void *d_comp, const uint64_t *d_offsets,
                                       size_t n, uint32_t chunk, int layout, void *d_out);
int snappy_amd_decompress_status(snappy_amd_ctx *ctx);
/* decompress with the flags/preamble value of compress_device_ex; sync = 1
 * reads back the status, 0 leaves it for snappy_amd_decompress_status. */
int snappy_amd_decompress_device_ex(snappy_amd_ctx *ctx, const void *d_comp, const uint64_t *d_offsets, size_t n,
                                    uint32_t chunk, int layout, uint32_t flags, uint64_t header_value, void *d_out,
                                    int sync);

/* Build the block index of a SINGLE-layout stream already in HBM (e.g. a
 * file produced by the reference or another encoder): d_offsets gets
 * ceil(N/65536)+1 entries (format above), *n_out the declared length N.
 * max_units = the entries d_offsets can hold (SNAPPY_AMD_ERR_CAPACITY if the
 * stream needs more).
 * SNAPPY_AMD_ERR_UNSUPPORTED only if a straddling element starts past 2^40
 * bytes or covers a boundary more than 2^24 - 1 bytes after its start. */
int snappy_amd_index_device(snappy_amd_ctx *ctx, const void *d_comp, size_t clen, uint64_t *d_offsets,
                            size_t max_units, size_t *n_out);

/* Kernel timing of the last compress/decompress call, measured with HIP
 * events on the launch stream: K1 (block compress), K3 (scan + gather),
 * K4 (block decode), milliseconds. */
int snappy_amd_last_timings(snappy_amd_ctx *ctx, float *k1_ms, float *k3_ms, float *k4_ms);
/* 1 = record the events above on every call (default 0). */
int snappy_amd_enable_timing(snappy_amd_ctx *ctx, int on);

#ifdef __cplusplus
}
#endif
#endif
