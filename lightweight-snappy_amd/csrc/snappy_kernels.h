// snappy_kernels.h -- private declarations shared by the HIP kernels and
// the extern "C" device shim.  Not part of the public C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SNAPPY_LAYOUT_SINGLE 0
#define SNAPPY_LAYOUT_STREAMS 1
#define SNAPPY_BLOCK 65536u

// which units carry a varint preamble
#define SNAPPY_HDR_NONE 0        // a SINGLE-layout shard continuing a stream
#define SNAPPY_HDR_FIRST_UNIT 1  // unit 0 = start of a SINGLE stream
#define SNAPPY_HDR_EVERY_UNIT 2  // STREAMS layout: every unit is a stream

// per-unit status values (same numbers as SNAPPY_AMD_ERR_* in snappy_amd.h)
#define SNAPPY_ST_OK 0
#define SNAPPY_ST_HEADER (-2)
#define SNAPPY_ST_TRUNCATED (-3)
#define SNAPPY_ST_OFFSET (-4)
#define SNAPPY_ST_OVERRUN (-5)
#define SNAPPY_ST_CAPACITY (-6)
#define SNAPPY_ST_UNSUPPORTED (-9)
#define SNAPPY_ST_TIMEOUT (-10)   // K4 pass 2: a unit waited too long for an earlier one
#define SNAPPY_ST_INDEX (-11)     // K4 (SINGLE): the unit's element chain does not end at the next index entry
#define SNAPPY_ST_DEFER 2         // K4 pass 1: the unit copies from earlier units (pass 2 decodes it;
                                  // meanwhile its status is DEFER + output bytes already in HBM)

namespace snappy_amd {

__global__ void k1r_match_units(const uint8_t *__restrict__ in, uint64_t n, uint32_t unit, uint32_t hdr_mode,
                                uint64_t header_value, uint2 *__restrict__ tokens, uint32_t tok_cap,
                                uint32_t *__restrict__ ntok_out, uint32_t *__restrict__ sizes,
                                uint32_t *__restrict__ seg_off, uint32_t segs);
__global__ void k1r_match_units64(const uint8_t *__restrict__ in, uint64_t n, uint32_t unit, uint32_t hdr_mode,
                                uint64_t header_value, uint2 *__restrict__ tokens, uint32_t tok_cap,
                                uint32_t *__restrict__ ntok_out, uint32_t *__restrict__ sizes,
                                uint32_t *__restrict__ seg_off, uint32_t segs);
__global__ void k2_emit_units(const uint8_t *__restrict__ in, uint64_t n, uint32_t unit, uint32_t hdr_mode,
                              uint64_t header_value, const uint2 *__restrict__ tokens, uint32_t tok_cap,
                              const uint32_t *__restrict__ ntok, const uint32_t *__restrict__ seg_off, uint32_t segs,
                              const uint64_t *__restrict__ offsets, uint8_t *__restrict__ out);
// K2 segments: 256 tokens (4 per lane); waves per unit
#ifndef SNAPPY_K2_SEG
#define SNAPPY_K2_SEG 256u
#endif
#ifndef SNAPPY_K2_WAVES
#define SNAPPY_K2_WAVES 8u
#endif
// register-resident K1r handles units up to this size (128 VGPRs x 64 lanes x 4 B)
#define SNAPPY_K1R_MAX_UNIT 32768u

__global__ void k3_scan(const uint32_t *__restrict__ sizes, uint64_t count, uint64_t *__restrict__ offsets,
                        uint64_t *__restrict__ total);
// one-wave K3 for launches of at most SNAPPY_K3_WAVE_MAX units
__global__ void k3_scan_wave(const uint32_t *__restrict__ sizes, uint64_t count, uint64_t *__restrict__ offsets,
                             uint64_t *__restrict__ total);
#define SNAPPY_K3_WAVE_MAX 8192u
// K4: comp is 4-byte aligned, the stream starts at comp + bias (bias < 4).
// K4 pass 1: every unit; allow_back = 1 for SINGLE-layout streams (straddling
// elements and copies into earlier blocks are legal: such units end with
// status SNAPPY_ST_DEFER, for pass 2, and set status[units + 1])
__global__ void k4_decompress_units(const uint8_t *__restrict__ comp, const uint64_t *__restrict__ offsets,
                                    uint64_t n, uint32_t unit, uint32_t hdr_mode, uint64_t header_value,
                                    uint32_t allow_back, uint32_t bias, uint8_t *__restrict__ out,
                                    int32_t *__restrict__ status);
// K4 pass 2: the DEFER units, in ticket order (status[units] = ticket counter,
// status[units + 1] = pass 1's defer flag; both 0 before pass 1)
__global__ void k4_decompress_back(const uint8_t *__restrict__ comp, const uint64_t *__restrict__ offsets,
                                   uint64_t n, uint32_t unit, uint32_t hdr_mode, uint64_t header_value,
                                   uint32_t bias, uint8_t *__restrict__ out,
                                   int32_t *__restrict__ status);
#ifndef SNAPPY_K5_CHUNK
#define SNAPPY_K5_CHUNK 16384
#endif
constexpr uint32_t K5_CHUNK = SNAPPY_K5_CHUNK;  // K5p chunk of compressed stream (K5_S in the kernels)
__global__ void k5a_chunk_walk(const uint8_t *__restrict__ comp, uint64_t clen, uint64_t *__restrict__ X,
                               uint64_t *__restrict__ O, uint32_t *__restrict__ P);
__global__ void k5b1_compose(const uint32_t *__restrict__ P, uint32_t nchunks, uint64_t *__restrict__ F);
__global__ void k5b_carry(const uint8_t *__restrict__ comp, uint64_t clen, uint32_t nchunks,
                          const uint64_t *__restrict__ X, const uint64_t *__restrict__ O, const uint64_t *__restrict__ F,
                          uint64_t *__restrict__ BE, uint64_t *__restrict__ BB, uint64_t *__restrict__ Ent,
                          uint64_t *__restrict__ Base, int64_t *__restrict__ result);
__global__ void k5b3_fill(const uint8_t *__restrict__ comp, uint64_t clen, const uint32_t *__restrict__ P,
                          uint32_t nchunks, const uint64_t *__restrict__ BE, const uint64_t *__restrict__ BB,
                          uint64_t *__restrict__ Ent, uint64_t *__restrict__ Base);
__global__ void k5c_mark(const uint8_t *__restrict__ comp, uint64_t clen, const uint64_t *__restrict__ Ent,
                         const uint64_t *__restrict__ Base, uint64_t *__restrict__ offsets, uint64_t max_units,
                         int32_t *__restrict__ cst, uint64_t *__restrict__ fin);
__global__ void k5d_result(uint32_t nchunks, const int32_t *__restrict__ cst, int64_t *__restrict__ result,
                           uint64_t *__restrict__ offsets, uint64_t max_units);
__global__ void k5_index_stream(const uint8_t *__restrict__ comp, uint64_t clen, uint64_t *__restrict__ offsets,
                                uint64_t max_units, int64_t *__restrict__ result);

}  // namespace snappy_amd
