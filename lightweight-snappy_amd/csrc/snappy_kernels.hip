// snappy_kernels.hip -- hand-written CDNA4 (gfx950) kernels of the Snappy
// block codec.  One wave64 per independent unit (a 65,536-byte block of a
// single stream, or one <=65,536-byte stream of the STREAMS layout).
//
//   K1 k1_compress_units   per-unit LZ77 match finder + element emit
//                          (reference: src/snappy_compression.c:384-403 and
//                          helpers :61-165, :229-329)
//   K3 k3_scan / k3_gather exclusive scan of unit sizes -> block index, then
//                          compaction of the fixed-stride scratch into one
//                          contiguous stream (replaces the per-block fwrite,
//                          src/snappy_compression.c:334-336)
//   K4 k4_decompress_units tag-dispatch decode of one unit into an LDS window
//                          (src/snappy_decompression.c:290-333)
//   K5 k5_index_stream     block index of a foreign single stream
//
// Data layout in LDS (K1): [u16 hash table, 4096 entries][unit input bytes
// + 16 zero pad].  The table holds block-relative positions; 0 is a valid
// candidate, exactly as in the reference (snappy_compression.c:259-265).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "snappy_kernels.h"

namespace snappy_amd {

constexpr uint32_t kTable = 4096;
constexpr uint32_t kMul = 0x1e35a7bdu;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Little-endian dword starting at byte q of a dword-aligned byte buffer.
__device__ __forceinline__ uint32_t le32_at(const uint32_t *w, uint32_t q)
{
    const uint32_t a = w[q >> 2];
    const uint32_t b = w[(q >> 2) + 1];
    return __builtin_amdgcn_alignbyte(b, a, q & 3);
}

// Big-endian load of src/snappy_compression.c:239-241.
__device__ __forceinline__ uint32_t be32_at(const uint32_t *w, uint32_t q)
{
    return __builtin_bswap32(le32_at(w, q));
}

__device__ __forceinline__ uint32_t varint_put(uint64_t v, uint8_t *out, uint32_t lane)
{
    // every lane computes the same encoding; lanes < len store one byte each
    uint32_t len = 1;
    uint64_t t = v;
    while (t >= 128) { t >>= 7; len++; }
    if (lane < len) {
        uint8_t b = (uint8_t)((v >> (7 * lane)) & 0x7F);
        if (lane + 1 < len) b |= 0x80;
        out[lane] = b;
    }
    return len;
}

// Literal element, src/snappy_compression.c:95-120: tag (len-1)<<2 for
// len-1 < 60, else tag (59+k)<<2 followed by len-1 in k LE bytes.
__device__ __forceinline__ uint32_t emit_literal(uint8_t *ob, uint32_t o, const uint8_t *inb, uint32_t start,
                                                 uint32_t len, uint32_t lane)
{
    const uint32_t m = len - 1;
    uint32_t hl, hdr;
    if (m < 60) { hl = 1; hdr = m << 2; }
    else if (m < 256) { hl = 2; hdr = (60u << 2) | (m << 8); }
    else { hl = 3; hdr = (61u << 2) | (m << 8); }
    const uint32_t total = hl + len;
    for (uint32_t b = 0; b < total; b += 64) {
        const uint32_t i = b + lane;
        if (i < total) {
            const uint32_t sh = (i < hl ? i : 0) * 8;
            ob[o + i] = i < hl ? (uint8_t)(hdr >> sh) : inb[start + i - hl];
        }
    }
    return o + total;
}

// Copy split 64/60 (src/snappy_compression.c:153-165) and piece encoding
// (:131-145): copy-1 iff len < 12 && off < 2048, else copy-2; never copy-4.
__device__ __forceinline__ uint32_t emit_copy(uint8_t *ob, uint32_t o, uint32_t len, uint32_t off, uint32_t lane)
{
    const uint32_t n64 = len > 68 ? (len - 68 + 63) >> 6 : 0;
    const uint32_t rem = len - 64 * n64;
    const uint32_t has60 = rem > 64 ? 1u : 0u;
    const uint32_t last = has60 ? rem - 60 : rem;
    const uint32_t offb = ((off & 0xFF) << 8) | (((off >> 8) & 0xFF) << 16);
    const uint32_t c64 = 0xFEu | offb;  // ((64-1)<<2)|2
    const uint32_t c60 = 0xEEu | offb;  // ((60-1)<<2)|2
    uint32_t lastb, lastl;
    if (last < 12 && off < 2048) {
        lastl = 2;
        lastb = ((((off >> 8) << 5) + ((last - 4) << 2) + 1) & 0xFF) | ((off & 0xFF) << 8);
    } else {
        lastl = 3;
        lastb = (((last - 1) << 2) | 2) | offb;
    }
    const uint32_t body = 3 * (n64 + has60);
    const uint32_t total = body + lastl;
    for (uint32_t b = 0; b < total; b += 64) {
        const uint32_t i = b + lane;
        if (i < total) {
            uint32_t v;
            if (i < body) {
                const uint32_t piece = i / 3;
                const uint32_t k = i - 3 * piece;
                v = (piece < n64 ? c64 : c60) >> (8 * k);
            } else {
                v = lastb >> (8 * (i - body));
            }
            ob[o + i] = (uint8_t)v;
        }
    }
    return o + total;
}

// ---------------------------------------------------------------------------
// K1: one wave per unit.  All control state is wave-uniform (SGPRs); the
// lanes cooperate on staging, match extension (64 bytes per ballot) and
// element emission.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k1_compress_units(const uint8_t *__restrict__ in, uint64_t n, uint32_t unit,
                                                        uint32_t hdr_mode, uint64_t header_value, uint32_t vec_ok,
                                                        uint8_t *__restrict__ scratch, uint64_t stride,
                                                        uint32_t *__restrict__ sizes)
{
    extern __shared__ uint32_t lds[];
    uint16_t *table = reinterpret_cast<uint16_t *>(lds);
    uint32_t *inw = lds + kTable / 2;
    uint8_t *inb = reinterpret_cast<uint8_t *>(inw);

    const uint32_t lane = threadIdx.x;
    const uint32_t u = blockIdx.x;
    const uint64_t base = (uint64_t)u * unit;
    const uint32_t L = (uint32_t)((n - base) < unit ? (n - base) : unit);
    const uint8_t *src = in + base;

    // Stage the unit into LDS: 16 B per lane per step (1 KiB per wave op).
    if (vec_ok) {
        const uint32_t L16 = L & ~15u;
        for (uint32_t i = lane * 16; i < L16; i += 1024)
            *reinterpret_cast<u32x4 *>(inb + i) = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(src + i));
        for (uint32_t i = L16 + lane; i < L; i += 64) inb[i] = src[i];
    } else {
        for (uint32_t i = lane; i < L; i += 64) inb[i] = src[i];
    }
    if (lane < 16) inb[L + lane] = 0;
    for (uint32_t i = lane; i < kTable / 2; i += 64) lds[i] = 0;
    __syncthreads();

    uint8_t *ob = scratch + (uint64_t)u * stride;
    uint32_t o = 0;
    if (hdr_mode == SNAPPY_HDR_EVERY_UNIT) o = varint_put(L, ob, lane);
    else if (hdr_mode == SNAPPY_HDR_FIRST_UNIT && u == 0) o = varint_put(header_value, ob, lane);

    // set_htable_size, src/snappy_compression.c:198-204
    uint32_t T = 256, lg = 8;
    while (T < kTable && T < L) { T <<= 1; lg++; }
    const uint32_t shift = 32 - lg;

    uint32_t p = 1, skip = 33, lit = 0;  // start_new_literal + append_literal
    while (!(L - p < (skip >> 5) + 15)) {  // is_block_end :229-232
        const uint32_t cur = rfl(be32_at(inw, p));
        const uint32_t h = (cur * kMul) >> shift;
        const uint32_t cand = rfl(table[h]);
        const uint32_t cv = rfl(be32_at(inw, cand));
        if (cv == cur) {  // found_match :259-265
            if (p > lit) o = emit_literal(ob, o, inb, lit, p - lit, lane);
            skip = 32;
            uint32_t len = 4;  // find_copy_length :61-72, limit = block end
            for (;;) {
                const uint32_t q = p + len + lane;
                const bool ok = q < L && inb[q] == inb[cand + len + lane];
                const uint64_t bad = __ballot(!ok);
                if (bad) { len += (uint32_t)__builtin_ctzll(bad); break; }
                len += 64;
            }
            o = emit_copy(ob, o, len, p - cand, lane);
            table[h] = (uint16_t)p;  // emit_copy :328
            p += len;
            lit = p;
        } else {  // update_hash_table :303-307, append_literal :283-287
            const uint32_t prev = rfl(be32_at(inw, p - 1));
            table[(prev * kMul) >> shift] = (uint16_t)(p - 1);
            table[h] = (uint16_t)p;
            p += skip >> 5;
            skip++;
        }
    }
    if (L > lit) o = emit_literal(ob, o, inb, lit, L - lit, lane);  // exhaust_input + emit_literal
    if (lane == 0) sizes[u] = o;
}

// ---------------------------------------------------------------------------
// K3a: exclusive scan of unit sizes -> offsets[0..count], total.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k3_scan(const uint32_t *__restrict__ sizes, uint64_t count,
                                                uint64_t *__restrict__ offsets, uint64_t *__restrict__ total)
{
    __shared__ uint64_t part[1024];
    const uint32_t t = threadIdx.x;
    const uint64_t per = (count + 1023) / 1024;
    const uint64_t b0 = t * per < count ? t * per : count;
    const uint64_t b1 = b0 + per < count ? b0 + per : count;
    uint64_t s = 0;
    for (uint64_t i = b0; i < b1; i++) s += sizes[i];
    part[t] = s;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        const uint64_t v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint64_t run = t ? part[t - 1] : 0;
    for (uint64_t i = b0; i < b1; i++) { offsets[i] = run; run += sizes[i]; }
    if (t == 1023) { offsets[count] = part[1023]; *total = part[1023]; }
}

// ---------------------------------------------------------------------------
// K3b: gather each unit's bytes from its 16-aligned scratch slot to its
// (byte-aligned) place in the output.  Destination writes are dword-aligned;
// the source side is realigned with v_alignbyte.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k3_gather(const uint8_t *__restrict__ scratch, uint64_t stride,
                                                 const uint32_t *__restrict__ sizes,
                                                 const uint64_t *__restrict__ offsets, uint8_t *__restrict__ out)
{
    const uint32_t u = blockIdx.x;
    const uint32_t t = threadIdx.x;
    const uint8_t *src = scratch + (uint64_t)u * stride;
    const uint32_t *srcw = reinterpret_cast<const uint32_t *>(src);
    uint8_t *dst = out + offsets[u];
    const uint32_t len = sizes[u];
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 3);
    uint32_t head = (4 - mis) & 3;
    if (head > len) head = len;
    if (t < head) dst[t] = src[t];
    const uint32_t nw = (len - head) >> 2;
    uint32_t *dstw = reinterpret_cast<uint32_t *>(dst + head);
    for (uint32_t k = t; k < nw; k += 256) dstw[k] = le32_at(srcw, head + 4 * k);
    const uint32_t tail0 = head + 4 * nw;
    if (t < len - tail0) dst[tail0 + t] = src[tail0 + t];
}

// ---------------------------------------------------------------------------
// K4: one wave per unit.  LDS: [decoded window: unit bytes][compressed unit].
// Tag dispatch of src/snappy_decompression.c:290-333 with bounds checks; a
// copy whose source lies before the unit start is an error here (the
// reference compressor never emits one; K5 detects them in foreign streams).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k4_decompress_units(const uint8_t *__restrict__ comp,
                                                          const uint64_t *__restrict__ offsets, uint64_t n,
                                                          uint32_t unit, uint32_t hdr_mode, uint64_t header_value,
                                                          uint32_t comp_cap,
                                                          uint8_t *__restrict__ out, int32_t *__restrict__ status)
{
    extern __shared__ uint32_t lds[];
    const uint32_t lane = threadIdx.x;
    const uint32_t u = blockIdx.x;
    const uint32_t win = (unit + 15) & ~15u;
    uint8_t *ob = reinterpret_cast<uint8_t *>(lds);
    uint32_t *cw = lds + win / 4 + 4;

    const uint64_t c0 = offsets[u], c1 = offsets[u + 1];
    const uint64_t base = (uint64_t)u * unit;
    const uint32_t want = (uint32_t)((n - base) < unit ? (n - base) : unit);
    int32_t st = SNAPPY_ST_OK;
    if (c1 < c0 || c1 - c0 > comp_cap) {
        if (lane == 0) status[u] = SNAPPY_ST_TRUNCATED;
        return;
    }
    const uint32_t clen = (uint32_t)(c1 - c0);

    // Stage compressed bytes: aligned dwords covering [c0 & ~3, c1); the
    // unit's byte i then sits at cb[mis + i].
    const uint32_t mis = (uint32_t)(c0 & 3);
    const uint64_t a0 = c0 - mis;
    const uint32_t span = clen + mis;
    const uint32_t nfull = span >> 2;
    const uint32_t *gw = reinterpret_cast<const uint32_t *>(comp + a0);
    for (uint32_t k = lane; k < nfull; k += 64) cw[k] = __builtin_nontemporal_load(gw + k);
    if (lane == 0) {
        uint32_t w = 0;
        for (uint32_t i = nfull * 4; i < span; i++) w |= (uint32_t)comp[a0 + i] << (8 * (i - nfull * 4));
        cw[nfull] = w;
        cw[nfull + 1] = 0;
        cw[nfull + 2] = 0;
    }
    __syncthreads();
    const uint8_t *cb = reinterpret_cast<const uint8_t *>(cw) + mis;

    uint32_t ip = 0, op = 0;
    // varint preamble: every STREAMS unit, and block 0 of a SINGLE stream
    if (hdr_mode == SNAPPY_HDR_EVERY_UNIT || (hdr_mode == SNAPPY_HDR_FIRST_UNIT && u == 0)) {
        const uint64_t expect = hdr_mode == SNAPPY_HDR_EVERY_UNIT ? want : header_value;
        uint64_t v = 0;
        uint32_t k = 0;
        bool done = false;
        for (; k < 10 && k < clen; k++) {
            const uint32_t byte = rfl(le32_at(cw, mis + k) & 0xFF);
            v |= (uint64_t)(byte & 0x7F) << (7 * k);
            if (!(byte & 0x80)) { done = true; k++; break; }
        }
        if (!done || v != expect) st = SNAPPY_ST_HEADER;
        ip = k;
    }

    while (st == SNAPPY_ST_OK && op < want) {
        if (ip >= clen) { st = SNAPPY_ST_TRUNCATED; break; }
        const uint32_t w = rfl(le32_at(cw, mis + ip));
        const uint32_t tag = w & 0xFF;
        uint32_t len, off;
        if ((tag & 3) == 0) {
            len = (tag >> 2) + 1;
            ip += 1;
            if (len > 60) {
                const uint32_t k = len - 60;
                if (ip + k > clen) { st = SNAPPY_ST_TRUNCATED; break; }
                const uint32_t x = rfl(le32_at(cw, mis + ip));
                len = (k == 4 ? x : (x & ((1u << (8 * k)) - 1))) + 1;
                ip += k;
            }
            if (len > clen - ip) { st = SNAPPY_ST_TRUNCATED; break; }
            if (len > want - op) { st = SNAPPY_ST_OVERRUN; break; }
            for (uint32_t b = lane; b < len; b += 64) ob[op + b] = cb[ip + b];
            ip += len;
            op += len;
            continue;
        }
        if ((tag & 3) == 1) {
            len = ((tag >> 2) & 7) + 4;
            off = ((tag >> 5) << 8) | ((w >> 8) & 0xFF);
            ip += 2;
        } else if ((tag & 3) == 2) {
            len = (tag >> 2) + 1;
            off = (w >> 8) & 0xFFFF;
            ip += 3;
        } else {
            len = (tag >> 2) + 1;
            off = rfl(le32_at(cw, mis + ip + 1));
            ip += 5;
        }
        if (ip > clen) { st = SNAPPY_ST_TRUNCATED; break; }
        if (off == 0 || off > op) { st = SNAPPY_ST_OFFSET; break; }
        if (len > want - op) { st = SNAPPY_ST_OVERRUN; break; }
        // byte-serial overlap semantics (snappy_decompression.c:273-280):
        // out[op+i] = out[op-off + i mod off]
        if (lane < len) {
            const uint32_t i = off >= len ? lane : lane % off;
            const uint8_t v = ob[op - off + i];
            ob[op + lane] = v;
        }
        op += len;
    }
    __syncthreads();

    // write the window out (unit-aligned destination)
    uint8_t *dst = out + base;
    if (((reinterpret_cast<uintptr_t>(dst) | want) & 15) == 0) {
        for (uint32_t i = lane * 16; i < want; i += 1024)
            *reinterpret_cast<u32x4 *>(dst + i) = *reinterpret_cast<const u32x4 *>(ob + i);
    } else {
        const uint32_t mis2 = (uint32_t)(reinterpret_cast<uintptr_t>(dst) & 3);
        uint32_t head = (4 - mis2) & 3;
        if (head > want) head = want;
        if (lane < head) dst[lane] = ob[lane];
        const uint32_t nw = (want - head) >> 2;
        uint32_t *dw = reinterpret_cast<uint32_t *>(dst + head);
        for (uint32_t k = lane; k < nw; k += 64) dw[k] = le32_at(lds, head + 4 * k);
        const uint32_t t0 = head + 4 * nw;
        if (lane < want - t0) dst[t0 + lane] = ob[t0 + lane];
    }
    if (lane == 0) status[u] = st;
}

// ---------------------------------------------------------------------------
// K5: block index of a SINGLE-layout stream (one wave).  The stream is
// walked through a 512-byte register window (two coalesced dword loads per
// lane); tag bytes come out of the window with v_readlane.  Records the
// compressed offset of every element that starts at a multiple of 65,536
// decoded bytes; flags elements that straddle such a boundary.
// result[0] = status, result[1] = declared length N, result[2] = units.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t win_byte(uint32_t w0, uint32_t w1, uint32_t rel)
{
    const uint32_t dw = rel >> 2;
    const uint32_t v = dw < 64 ? __builtin_amdgcn_readlane(w0, dw & 63) : __builtin_amdgcn_readlane(w1, dw & 63);
    return (v >> (8 * (rel & 3))) & 0xFF;
}

__global__ __launch_bounds__(64) void k5_index_stream(const uint8_t *__restrict__ comp, uint64_t clen,
                                                      uint64_t *__restrict__ offsets, uint64_t max_units,
                                                      int64_t *__restrict__ result)
{
    const uint32_t lane = threadIdx.x;
    uint64_t wbase = ~0ull;
    uint32_t w0 = 0, w1 = 0;
    auto fetch = [&](uint64_t pos) -> uint32_t {
        const uint64_t want_base = pos & ~3ull;
        if (wbase == ~0ull || pos < wbase || pos + 8 > wbase + 512) {
            wbase = want_base;
            const uint64_t q0 = wbase + 4 * lane, q1 = q0 + 256;
            uint32_t a = 0, b = 0;
            for (uint32_t k = 0; k < 4; k++) {
                if (q0 + k < clen) a |= (uint32_t)comp[q0 + k] << (8 * k);
                if (q1 + k < clen) b |= (uint32_t)comp[q1 + k] << (8 * k);
            }
            w0 = a;
            w1 = b;
        }
        return win_byte(w0, w1, (uint32_t)(pos - wbase));
    };

    int64_t st = SNAPPY_ST_OK;
    uint64_t N = 0, ip = 0;
    uint32_t k = 0;
    bool done = false;
    for (; k < 10 && ip < clen; k++) {
        const uint32_t byte = fetch(ip++);
        N |= (uint64_t)(byte & 0x7F) << (7 * k);
        if (!(byte & 0x80)) { done = true; break; }
    }
    if (!done) st = SNAPPY_ST_HEADER;
    const uint64_t units = (N + SNAPPY_BLOCK - 1) / SNAPPY_BLOCK;
    if (st == SNAPPY_ST_OK && units > max_units) st = SNAPPY_ST_CAPACITY;
    uint64_t op = 0, unit = 0;
    if (st == SNAPPY_ST_OK && lane == 0 && units) offsets[0] = 0;
    unit = 1;
    while (st == SNAPPY_ST_OK && op < N) {
        if (ip >= clen) { st = SNAPPY_ST_TRUNCATED; break; }
        const uint32_t tag = fetch(ip);
        uint64_t len;
        switch (tag & 3) {
        case 0:
            len = (tag >> 2) + 1;
            ip += 1;
            if (len > 60) {
                const uint32_t kk = (uint32_t)len - 60;
                if (ip + kk > clen) { st = SNAPPY_ST_TRUNCATED; break; }
                len = 0;
                for (uint32_t i = 0; i < kk; i++) len |= (uint64_t)fetch(ip + i) << (8 * i);
                len += 1;
                ip += kk;
            }
            ip += len;
            break;
        case 1: len = ((tag >> 2) & 7) + 4; ip += 2; break;
        case 2: len = (tag >> 2) + 1; ip += 3; break;
        default: len = (tag >> 2) + 1; ip += 5; break;
        }
        if (st != SNAPPY_ST_OK) break;
        if (ip > clen) { st = SNAPPY_ST_TRUNCATED; break; }
        // element [op, op+len) must not straddle a 65,536 boundary
        const uint64_t next_boundary = unit * SNAPPY_BLOCK;
        if (op < next_boundary && op + len > next_boundary && next_boundary < N) {
            st = SNAPPY_ST_UNSUPPORTED;
            break;
        }
        op += len;
        if (op == next_boundary && op < N) {
            if (lane == 0) offsets[unit] = ip;
            unit++;
        }
        if (op > N) { st = SNAPPY_ST_OVERRUN; break; }
    }
    if (lane == 0) {
        if (st == SNAPPY_ST_OK) offsets[units] = ip;
        result[0] = st;
        result[1] = (int64_t)N;
        result[2] = (int64_t)units;
    }
}

}  // namespace snappy_amd
