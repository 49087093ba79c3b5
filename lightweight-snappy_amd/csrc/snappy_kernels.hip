// snappy_kernels.hip -- hand-written CDNA4 (gfx950) kernels of the Snappy
// block codec.  One wave64 per independent unit (a 65,536-byte block of a
// single stream, or one <=65,536-byte stream of the STREAMS layout).
//
//   K1r k1r_match_units(64) per-unit LZ77 match finder -> tokens
//                          (reference: src/snappy_compression.c:384-403 and
//                          helpers :61-72, :229-329)
//   K3  k3_scan            exclusive scan of unit sizes -> block index
//   K2  k2_emit_units      tokens -> Snappy elements at their final offsets
//                          (:95-165; replaces the per-block fwrite :334-336)
//   K4  k4_decompress_*    tag-dispatch decode, block-parallel
//                          (src/snappy_decompression.c:290-363)
//   K5  k5_* / k5a-d       block index of a foreign single stream (K5a, K5b1-3, K5c, K5d)
//
// The hash table holds block-relative positions; 0 is a valid candidate,
// exactly as in the reference (snappy_compression.c:259-265).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#include "snappy_kernels.h"

// The Makefile builds this file twice: SNAPPY_TU=1 emits the compress kernels
// (K1r, K2, K3), SNAPPY_TU=2 the decode kernels (K4, K5), so each object is
// compiled with the instruction scheduler measured fastest for its kernels.
// SNAPPY_TU unset (tools/isa.sh, variant builds) emits all of them.
#ifndef SNAPPY_TU
#define SNAPPY_TU 0
#endif
#define SNAPPY_TU_COMPRESS (SNAPPY_TU != 2)
#define SNAPPY_TU_DECODE (SNAPPY_TU != 1)

// Measurement-only knobs whose kernels write WRONG bytes (they time what a
// piece of work costs by skipping it): a product build cannot set them.  The
// shipped library reports its knobs through snappy_amd_build_config(), which
// tests/test_abi.py and the GPU tests check.
#if ((defined(SNAPPY_K2_NOLIT) && SNAPPY_K2_NOLIT) || defined(SNAPPY_K4_NOFAR)) && !defined(SNAPPY_MEASUREMENT_BUILD)
#error "SNAPPY_K2_NOLIT / SNAPPY_K4_NOFAR write wrong output: measurement builds only (-DSNAPPY_MEASUREMENT_BUILD)"
#endif

namespace snappy_amd {

// v_writelane_b32 (no clang builtin in this toolchain): the LLVM intrinsic by name
__device__ int amdgcn_writelane(int val, int lanesel, int old) __asm("llvm.amdgcn.writelane.i32");


constexpr uint32_t kTable = 4096;
constexpr uint32_t kMul = 0x1e35a7bdu;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

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

// Probe position of the k-th consecutive miss after (p, skip):
// p_k = p + sum_{j<k} ((skip + j) >> 5) = p + F(skip + k) - F(skip), with
// F(m) = sum_{i<m} (i >> 5) = 16 q (q - 1) + (m & 31) q, q = m >> 5.
__device__ __forceinline__ uint32_t skipsum(uint32_t m)
{
    const uint32_t q = m >> 5;
    return 16 * q * (q - 1) + (m & 31) * q;
}

// ---------------------------------------------------------------------------
// K1r: register-resident match finder (one wave per unit).
//
//  * The unit lives in VGPRs: register r, lane l holds big-endian dword
//    64 r + l (128 VGPRs v2..v129 hold 32 KiB).  65,536-byte blocks keep a
//    ring of their last 128 256-byte segments there instead (segment s in
//    register s % 128, loaded ahead of the probe window; measured on the text
//    workload only 1.4 % of candidate checks reach further back, and those read
//    global memory), so both kernels run 3 waves per SIMD.  A wave-uniform
//    register index goes through s_set_gpr_idx_on.  Any 64 consecutive dwords
//    d..d+63 sit in registers R = d / 64 and R + 1: merged by one lane select
//    they are a rotation of the wanted lanes, undone by one ds_bpermute.
//  * The hash table lives in LDS as 4096 u16 positions + 4096 u8 tags of the
//    4 bytes there (12 KiB).  A probe whose tag differs is a miss decided
//    without touching the input; equal tags are verified against the bytes,
//    so the probe/insert sequence of src/snappy_compression.c:384-403 is
//    reproduced bit for bit.
//  * Position window: lane l <-> position q0 + l holds the BE32 there (`bv`),
//    its hash and tag (`hv`), the nearest earlier window lane with the same
//    hash (DPP wave_shr chain, up to DMAX back) and the table entry of its
//    slot (`ent`, re-read after every round's inserts).
//  * Lane-space rounds (step-1 probes, i.e. skip < 64: the text regime): the
//    probes p, p + 1, ... ARE window lanes p - q0, ...  Lane l's candidate is
//    its table entry unless a lane in [p - 1 - q0, l) has the same hash (the
//    round's misses insert exactly those positions): then that lane.  One
//    ballot finds the first probable hit; the lanes before it are exact
//    misses, inserted by one lane-ordered write (the highest lane wins a
//    shared slot, which is the serial order); the hit is verified and its
//    length found by 16 lanes comparing 64 bytes per step.
//  * Larger steps (skip >= 61, incompressible data) use W = 4 speculative
//    probes at their closed-form positions with explicit conflict stops.
//  * Output is a token list (4 bytes each: offset | (length - 4) << 16 |
//    literal gap << 24, escapes in a second array), the unit's exact encoded
//    size and every 256th token's output offset / input position; K3 places
//    every unit, K2 writes the bytes.
// 12 KiB LDS and <= 168 VGPRs -> 12 units per CU (3 waves per SIMD), both
// kernels.
// ---------------------------------------------------------------------------
typedef uint32_t v32 __attribute__((ext_vector_type(32)));
typedef uint32_t __attribute__((aligned(1))) u32u;
typedef uint16_t __attribute__((aligned(1))) u16u;

[[maybe_unused]] constexpr uint32_t kTagMul = 0x9E3779B1u;
constexpr uint32_t kRegs = 128;  // VGPRs holding a 32 KiB unit (64 dwords each), + 1 zero spare
// Register r (wave-uniform) of the resident unit.  g0..g3 are pinned to
// v2..v129 by the asm constraints, so the relative move (s_set_gpr_idx_on,
// SRC0) is exact whatever else the allocator does.  s_set_gpr_idx_on writes
// m0, a register the compiler reserves (writelane lane selects) and does not
// take as an asm clobber.  The statements leave m0 holding the index: the
// built code object is checked to set m0 again before any later read of it
// (tools/check_asm_waits.py check_m0, run by tests/test_abi.py).
// SNAPPY_REGIDX_M0_SAVE 1 saves and restores m0 inside each statement instead
// (A/B, outputs identical: K1r +1.1 %, K1r64 +0.5 %, profiles/r06w_*).
#ifndef SNAPPY_REGIDX_M0_SAVE
#define SNAPPY_REGIDX_M0_SAVE 0
#endif
#if SNAPPY_REGIDX_M0_SAVE
#define REGIDX_M0_DECL uint32_t _m0;
#define REGIDX_M0_SAVE "s_mov_b32 %[m0s], m0\n\t"
#define REGIDX_M0_REST "\n\ts_mov_b32 m0, %[m0s]"
#define REGIDX_M0_OUT , [m0s] "=&s"(_m0)
#define REGIDX_M0_ONLY [m0s] "=&s"(_m0)
#else
#define REGIDX_M0_DECL
#define REGIDX_M0_SAVE ""
#define REGIDX_M0_REST ""
#define REGIDX_M0_OUT
#define REGIDX_M0_ONLY
#endif
#define REG_OF_V(r)                                                                                 \
    ({                                                                                              \
        uint32_t _v;                                                                                \
        REGIDX_M0_DECL                                                                              \
        asm volatile(REGIDX_M0_SAVE "s_set_gpr_idx_on %[ri], gpr_idx(SRC0)\n\tv_mov_b32 %[ov], v2\n\t"     \
                     "s_set_gpr_idx_off" REGIDX_M0_REST                                            \
                     : [ov] "=&v"(_v) REGIDX_M0_OUT                                                  \
                     : [ri] "s"((uint32_t)(r)), "{v[2:33]}"(g0), "{v[34:65]}"(g1), "{v[66:97]}"(g2),      \
                       "{v[98:129]}"(g3));                                                          \
        _v;                                                                                         \
    })
// BIG (65,536-byte blocks): the 128 registers are a ring over the block's
// 256-byte segments -- segment s lives in register s % 128 while it is one of
// the last 128 loaded (ring_to in k1r_body); older candidates are read from
// global memory.  s_set_gpr_idx DST mode writes a ring register in place.
// g0..g3 are only ever read through asm that names v2..v129, so the write is
// modelled as a use: tied in/out operands make the allocator copy the 128
// registers (hundreds of spills).  The kernels are checked to keep g0..g3 in
// place with no VGPR spills (tests/test_abi.py::test_kernel_register_budget).
#define REG_SET_V(r, val)                                                                            \
    do {                                                                                             \
        REGIDX_M0_DECL                                                                               \
        asm volatile(REGIDX_M0_SAVE "s_set_gpr_idx_on %[ri], gpr_idx(DST)\n\tv_mov_b32 v2, %[xv]\n\t"       \
                     "s_set_gpr_idx_off" REGIDX_M0_REST                                             \
                     : REGIDX_M0_ONLY                                                                \
                     : [ri] "s"((uint32_t)(r)), [xv] "v"(val), "{v[2:33]}"(g0), "{v[34:65]}"(g1),        \
                       "{v[66:97]}"(g2), "{v[98:129]}"(g3) : "memory");                              \
    } while (0)
#define REG_OF(r)                                                                                   \
    ({                                                                                              \
        const uint32_t _rr = (r);                                                                   \
        uint32_t _rv;                                                                               \
        if constexpr (BIG) _rv = REG_OF_V(_rr & (kRegs - 1));                                       \
        else _rv = REG_OF_V(_rr);                                                                   \
        _rv;                                                                                        \
    })

// registers r and r + 1 of the resident unit with one s_set_gpr_idx_on region
// (SRC0 of both moves is indexed); r + 1 = 128 of a 32 KiB unit reads v130,
// which holds no unit data (see DW_LANES)
#define REG_PAIR_V(r, lo, hi)                                                                        \
    do {                                                                                             \
        REGIDX_M0_DECL                                                                               \
        asm volatile(REGIDX_M0_SAVE "s_set_gpr_idx_on %[ri], gpr_idx(SRC0)\n\tv_mov_b32 %[olo], v2\n\t"      \
                     "v_mov_b32 %[ohi], v3\n\ts_set_gpr_idx_off" REGIDX_M0_REST                        \
                     : [olo] "=&v"(lo), [ohi] "=&v"(hi) REGIDX_M0_OUT                                  \
                     : [ri] "s"((uint32_t)(r)), "{v[2:33]}"(g0), "{v[34:65]}"(g1), "{v[66:97]}"(g2),      \
                       "{v[98:129]}"(g3));                                                           \
    } while (0)
#define REG_PAIR(r, lo, hi)                                                                          \
    do {                                                                                             \
        const uint32_t _pr = (r);                                                                    \
        if constexpr (BIG) { /* ring registers r, r + 1 (mod 128) */                                 \
            const uint32_t _pq = _pr & (kRegs - 1);                                                  \
            if (__builtin_expect(_pq != kRegs - 1, 1)) REG_PAIR_V(_pq, lo, hi);                      \
            else { lo = REG_OF_V(kRegs - 1); hi = REG_OF_V(0); }                                     \
        } else {                                                                                     \
            REG_PAIR_V(_pr, lo, hi);                                                                 \
        }                                                                                            \
    } while (0)

// lane i <- big-endian dword d + i of the unit (d wave-uniform): registers
// R = d / 64 and R + 1 merged at lane d % 64 hold the 64 dwords rotated by
// d % 64; one ds_bpermute puts them in order (it reads lane addr[7:2], so
// the rotation needs no masking: tools/micro/lds_packed3.hip)
#define DW_LANES(dd)                                                                                 \
    ({                                                                                               \
        const uint32_t _d = (dd);                                                                    \
        const uint32_t _R = _d >> 6, _l0 = _d & 63;                                                  \
        /* R + 1 = 128 (v130, 32 KiB units) holds no unit data: those lanes lie past the */          \
        /* unit end, where every caller ignores them (past-L compares are clamped) */              \
        uint32_t _r0, _r1;                                                                           \
        REG_PAIR(_R, _r0, _r1);                                                                      \
        const uint32_t _m = lane >= _l0 ? _r0 : _r1;                                                 \
        (uint32_t)__builtin_amdgcn_ds_bpermute((int)((_d + lane) << 2), (int)_m); /* addr[7:2] */   \
    })

// DPP across the whole wave: wave_shl:1 (lane l <- l + 1) and wave_shr:1
// (lane l <- l - 1); lanes with no source get 0
__device__ __forceinline__ uint32_t wave_shl1(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, true);
}

// big-endian funnel by bytes: the 32 bits starting k bytes (0..3) into the
// 64-bit big-endian hi:lo, one v_perm_b32 (selector bytes 4-k..7-k)
__device__ __forceinline__ uint32_t perm_sel(uint32_t k) { return 0x07060504u - k * 0x01010101u; }
__device__ __forceinline__ uint32_t funnel_bytes(uint32_t hi, uint32_t lo, uint32_t sel)
{
    return __builtin_amdgcn_perm(hi, lo, sel);
}

// bit d (1 <= d <= D) set iff lane l - d carries the same x as lane l (x != 0)
template <uint32_t D>
__device__ __forceinline__ uint32_t same_x_bits(uint32_t x)
{
    uint32_t xs = x, bits = 0;
#pragma unroll
    for (uint32_t d = 1; d <= D; d++) {
        xs = wave_shr1(xs);
        bits |= (xs == x) ? (1u << d) : 0u;
    }
    return bits;
}

__device__ __forceinline__ uint32_t varint_len(uint64_t v)
{
    uint32_t len = 1;
    while (v >= 128) { v >>= 7; len++; }
    return len;
}

// encoded size of a literal of n bytes (src/snappy_compression.c:95-120)
__device__ __forceinline__ uint32_t literal_bytes(uint32_t n)
{
    return n + (n <= 60 ? 1 : (n <= 256 ? 2 : 3));
}

// encoded size of a copy (src/snappy_compression.c:131-165)
__device__ __forceinline__ uint32_t copy_bytes(uint32_t len, uint32_t off)
{
    const uint32_t n64 = len > 68 ? (len - 68 + 63) >> 6 : 0;
    const uint32_t rem = len - 64 * n64;
    const uint32_t has60 = rem > 64 ? 1u : 0u;
    const uint32_t last = has60 ? rem - 60 : rem;
    return 3 * (n64 + has60) + ((last < 12 && off < 2048) ? 2 : 3);
}

// Conflicts of the W-probe rounds (large steps): lane k must not read a slot
// an earlier lane writes (h_k in {h_j, a_j}), nor have its a-insert
// overwritten by an earlier lane's h-insert of another position (a_k == h_j,
// p_j != p_k - 1).  eqm(x) = all-ones iff x == 0, for x < 2^31.  Lanes with no
// source lane see 0 (bound_ctrl), which can only add false conflicts; lane 0
// is never flagged (the caller masks it), so every round makes progress.
__device__ __forceinline__ uint32_t eqm(uint32_t x) { return (uint32_t)((int32_t)(x - 1) >> 31); }

template <int N>
__device__ __forceinline__ uint32_t shz(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x110 + N, 0xF, 0xF, true);
}

template <int N>
__device__ __forceinline__ uint32_t tconf_step(uint32_t h, uint32_t a, uint32_t notdup)
{
    const uint32_t hs = shz<N>(h), as = shz<N>(a);
    if constexpr (N == 1) return eqm(h ^ hs) | eqm(h ^ as) | (eqm(a ^ hs) & notdup);
    else return eqm(h ^ hs) | eqm(h ^ as) | eqm(a ^ hs);
}

template <int W>
__device__ __forceinline__ uint32_t tconf(uint32_t h, uint32_t a, uint32_t notdup)
{
    static_assert(W >= 1 && W <= 4, "W-probe rounds speculate at most 4 probes");
    uint32_t c = 0;
    if constexpr (W > 1) c |= tconf_step<1>(h, a, notdup);
    if constexpr (W > 2) c |= tconf_step<2>(h, a, notdup);
    if constexpr (W > 3) c |= tconf_step<3>(h, a, notdup);
    return c;
}

#ifndef SNAPPY_K1R_DMAX
#define SNAPPY_K1R_DMAX 13  // lane-space rounds: same-hash distances resolved per window (8/10/12/14/16
                            // measured, profiles/r03h_ab_k1r_dmax_rmin_*; with the round-5 asm loop at
                            // its best loop placement 8 / 9 / 10: 12.46 / 12.37 / 12.23 ms per GiB,
                            // profiles/r05zw_*; round 6 at RMIN 2: 11 / 13 / 14 / 16 -> 12.31-12.32 /
                            // 12.26-12.27 / 12.34-12.37 / 12.52-12.58, profiles/r06m_*)
#endif
#ifndef SNAPPY_K1R_DMAX64
#define SNAPPY_K1R_DMAX64 12  // K1r64 (65,536-byte blocks): round 6 at RMIN 2, 10 / 12 / 13 / 14 ->
                              // 14.07-14.09 / 14.03-14.04 / 14.42 / 14.12-14.13 ms per GiB (r06m_*)
#endif
#ifndef SNAPPY_K1R_LSMIN
#define SNAPPY_K1R_LSMIN 4  // lane-space rounds while at least this many step-1 probes remain
#endif
#ifndef SNAPPY_K1R_RMIN
#define SNAPPY_K1R_RMIN 2  // refresh the window when fewer probe lanes remain (round 6, DMAX 13 / 12:
                           // 1 / 2 / 3 / 4 / 6 -> 12.17 / 12.13-12.17 / 12.15-12.18 / 12.19-12.22 /
                           // 12.33 ms per GiB, 64 KiB blocks 13.90 / 13.90-13.92 / 13.93 / 13.95 /
                           // 14.11, profiles/r06l_*).  Any RMIN >= 1 keeps a window's tokens <= 16
                           // (62 probe positions, >= 4 bytes per match), so pend <= 48 + 16 = 64
#endif
#ifndef SNAPPY_K1R_WINDOW
#define SNAPPY_K1R_WINDOW 4  // W-probe rounds
#endif


#if defined(SNAPPY_K1R_LSTAMPS) || defined(SNAPPY_K1R_RSTAMPS)
#define MSTAMP(var)                                                                         \
    do {                                                                                    \
        __builtin_amdgcn_sched_barrier(0);                                                  \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(var)::"memory");        \
        __builtin_amdgcn_sched_barrier(0);                                                  \
    } while (0)
#endif
// SNAPPY_K1R_RSTAMPS (measurement build): the window refresh's cycles (token
// flush and window move separately) against the whole loop's, with the asm
// round loop in place (the LSTAMPS / STATS builds run the C++ round instead)
#if defined(SNAPPY_K1R_RSTAMPS)
#define RSTAMP(var) MSTAMP(var)
#else
#define RSTAMP(var) do { } while (0)
#endif
#if defined(SNAPPY_K1R_LSTAMPS)
#define LSTAMP(var) MSTAMP(var)
#define LSEG(i, a, b) seg[i] += (b) - (a)
#else
#define LSTAMP(var) do { } while (0)
#define LSEG(i, a, b) do { } while (0)
#endif

// K2 segments (K1r records each one's output offset and input position): 256
// tokens; K2 walks a segment in passes of kK2Pass tokens, kK2Per per lane (2: 80
// VGPRs, 6 waves per SIMD; a 256-token pass needs 114, 4 waves: 7 % slower)
#ifndef SNAPPY_K2_PASS
#define SNAPPY_K2_PASS 128u
#endif
constexpr uint32_t kK2Seg = SNAPPY_K2_SEG;
constexpr uint32_t kK2Pass = SNAPPY_K2_PASS;
[[maybe_unused]] constexpr uint32_t kK2Per = kK2Pass / 64;
static_assert(kK2Pass % 64 == 0 && kK2Seg % kK2Pass == 0, "K2: passes of 64 k tokens dividing a segment");

// Wave-wide inclusive add-scan in DPP (row_shr 1/2/4/8 inside 16-lane rows,
// then row_bcast:15 / row_bcast:31 across rows): no LDS round trips.
template <uint32_t CTRL, uint32_t ROWS>
__device__ __forceinline__ uint32_t dpp0(uint32_t x)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xF, true);
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x)
{
    x += dpp0<0x111, 0xF>(x);
    x += dpp0<0x112, 0xF>(x);
    x += dpp0<0x114, 0xF>(x);
    x += dpp0<0x118, 0xF>(x);
    x += dpp0<0x142, 0xA>(x);
    x += dpp0<0x143, 0xC>(x);
    return x;
}

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t lane, uint32_t *total)
{
    (void)lane;
    const uint32_t x = wave_incl_scan(v);
    *total = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
    return x - v;
}

// The lane data carry the in-window predecessor's tag (pdnz), so the hit test
// selects the candidate's tag and compares it once with the lane's (16-bit
// field: a lane past the window has bit 24 of its word set and never matches)
// -- two VALU instead of three (V16: 64 KiB blocks 15.04-15.08 -> 14.51 ms per
// GiB, 32 KiB streams at matched loop placement 12.56 -> 12.34-12.36;
// profiles/r05za_*, r05zs_*)

template <bool BIG>
__device__ __forceinline__ void k1r_body(const uint8_t *__restrict__ in, uint64_t n, uint32_t unit,
                                         uint32_t hdr_mode, uint64_t header_value,
                                         uint2 *__restrict__ tokens, uint32_t tok_cap,
                                         uint32_t *__restrict__ ntok_out, uint32_t *__restrict__ sizes,
                                         uint32_t *__restrict__ seg_off, uint32_t segs)
{
    constexpr int W = SNAPPY_K1R_WINDOW;
    constexpr uint32_t DMAX = BIG ? SNAPPY_K1R_DMAX64 : SNAPPY_K1R_DMAX;
    static_assert(SNAPPY_K1R_LSMIN >= 4 && SNAPPY_K1R_LSMIN <= 32, "lane-space rounds need skip < 64 - 3");
    static_assert(DMAX >= 2 && DMAX <= 16, "DMAX: 2..16 (kcap <= 15 keeps the lane masks in range)");
    // 12 KiB: 4096 packed 3-byte records (u16 position, u8 tag) at byte 3 * slot:
    // one unaligned ds_read_b32 fetches position | tag << 16 (bits 24..31 are
    // the next record's), a ds_write_b16 + ds_write_b8_d16_hi store one; the
    // highest lane wins a record shared within one instruction pair
    // (tools/micro/lds_packed3.hip).  12 units/CU (with the VGPR limit).
    // The same 12 KiB as two aligned arrays: u16 positions at byte 2 * slot and
    // u8 tags at kTagBase + slot, so no table access is unaligned (the packed
    // 3-byte records measured SQ_LDS_UNALIGNED_STALL 8.5e9 per 1 GiB launch:
    // the LDS spent most of its active cycles stalled on them).  A record's
    // address is that of its position (`adr` = 2 * slot); its tag sits at
    // adr / 2 + kTagBase.  Reads: ds_read_u16 + ds_read_u8; writes:
    // ds_write_b16 + ds_write_b8_d16_hi, each highest-lane-wins on its own
    // address, so a record shared within one write pair is the same lane's.
    // slot kTable: a record nobody reads, the target of non-inserting lanes (one
    // per lane instead -- no same-address writes -- measured 2.6 % slower: 16.86
    // against 16.42 ms per GiB of 32 KiB text streams)
    constexpr uint32_t kSlots = kTable + 1;
    constexpr uint32_t kTagBase = 2 * kSlots + 6;
    __shared__ __attribute__((aligned(16))) uint8_t tbl_[kTagBase + kSlots + 7];
    constexpr uint32_t kDummy = 2 * kTable;
    auto *const tbl = (__attribute__((address_space(3))) uint8_t *)tbl_;
    // (the two halves are loaded into one register as a 2 x u16 vector, so the
    // backend can use ds_read_u16_d16 + ds_read_u8_d16_hi: no VALU joins them,
    // so no wait is forced where the read is issued)
#define TBL_READ3(adr)                                                                              \
    ({                                                                                             \
        const uint32_t _a = (adr);                                                                 \
        u16x2 _v;                                                                                  \
        _v.x = *(__attribute__((address_space(3))) uint16_t *)(tbl + _a);                          \
        _v.y = (uint16_t)tbl[(_a >> 1) + kTagBase];                                                \
        __builtin_bit_cast(uint32_t, _v);                                                          \
    })
#define TBL_WRITE3(adr, word)                                                                       \
    do {                                                                                           \
        const uint32_t _a = (adr), _w = (word);                                                    \
        *(__attribute__((address_space(3))) uint16_t *)(tbl + _a) = (uint16_t)_w;                   \
        tbl[(_a >> 1) + kTagBase] = (uint8_t)(_w >> 16);                                           \
    } while (0)
#define TBL_ADR(h) (2 * (h))
// lane-space rounds: position and tag as two registers (nothing joins the two
// loads, so their wait sits at the first use, not where they are issued)
#define TBL_READ_ENT(adr)                                                                           \
    do {                                                                                           \
        const uint32_t _a = (adr);                                                                 \
        ent = *(__attribute__((address_space(3))) uint16_t *)(tbl + _a);                           \
        ent_t = tbl[(_a >> 1) + kTagBase];                                                         \
    } while (0)
#define TBL_READ(h) TBL_READ3(2 * (h))
#define TBL_WRITE(s, word) TBL_WRITE3(2 * (s), word)
// The tag: the 8 product bits below the table index, ((v *
// kMul) >> (shift - 8)) & 0xFF, instead of a second multiply (any function of
// the 4 bytes filters candidates: equal bytes give equal tags, and a tag
// collision is verified like any hit)
#define TAG_OF(v) __builtin_amdgcn_ubfe((v) * kMul, shift - 8, 8)
// an insert group: the lanes where cond holds write their record; the others
// write the dummy record (one instruction stream, no exec change: masking
// them off measured 3 % slower, profiles/r03j_ab_k1r_masked_*)
#define TBL_INSERT(cond) TBL_WRITE3((cond) ? adr : kDummy, word)
// Lanes communicate through the table: a read must see every earlier write of
// the wave, including other lanes' (LDS executes a wave's accesses in order).
// C++ sees no such dependence, so every write group is followed by a compiler
// barrier that keeps later reads after it.
#define LDS_ORDER() asm volatile("" ::: "memory")
// tag bits 16..23 of an entry against those of a hash|tag word
#define TAG_EQ(e, w) ((((e) ^ (w)) & 0xFF0000u) == 0)
    const uint32_t lane = threadIdx.x;
    const uint32_t u = blockIdx.x;
    const uint64_t base = (uint64_t)u * unit;
    const uint32_t L = (uint32_t)((n - base) < unit ? (n - base) : unit);
    const uint8_t *src = in + base;
#ifdef SNAPPY_K1R_STATS
    const uint64_t t_start = clock64();
    (void)t_start;
#endif

    // unit -> registers, big-endian dwords, zero past the end
    v32 g0, g1, g2, g3;
    const bool aligned = ((reinterpret_cast<uintptr_t>(src) & 3) == 0);
    // big-endian dword k (per lane) of the unit, zero past its end
    auto load_dw = [&](uint32_t k) -> uint32_t {
        const uint32_t b = 4 * k;
        uint32_t w = 0;
        if (b + 4 <= L && aligned) {
            w = __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(src + b));
        } else if (b < L) {
            for (uint32_t k = 0; k < 4; k++)
                if (b + k < L) w |= (uint32_t)src[b + k] << (8 * k);
        }
        return __builtin_bswap32(w);
    };
    auto load_word = [&](uint32_t i) -> uint32_t { return load_dw(64 * i + lane); };
#pragma unroll
    for (int i = 0; i < (int)kRegs; i++) {
        const uint32_t w = load_word(i);
        if (i < 32) g0[i] = w;
        else if (i < 64) g1[i - 32] = w;
        else if (i < 96) g2[i - 64] = w;
        else g3[i - 96] = w;
    }

    // BIG: segments [seg_hi - 128, seg_hi) are resident in the ring registers;
    // segment seg_hi is prefetched into LDS by an LDS-DMA load (global_load_lds)
    // as soon as the ring moves, so the next advance finds it there instead of
    // waiting on a global load
    uint32_t seg_hi = kRegs;
#ifdef SNAPPY_K1R_STATS
    uint32_t n_farc = 0, n_reload = 0;  // BIG: candidate gathers from global memory, segments loaded synchronously
#define K1R_COUNT(x) (x)++
#else
#define K1R_COUNT(x) do { } while (0)
#endif
    __shared__ uint32_t ring_stage[64];
    uint32_t staged = 0;  // BIG: 1 + the segment in ring_stage, 0 = none
    auto stage = [&](uint32_t sg) {
        if constexpr (BIG) {
            staged = 0;
            if (aligned && 256 * (sg + 1) <= L) {
                // scalar base + lane offset (the builtin would keep a 64-bit per-lane
                // address live and spill); the compiler does not track this load:
                // ring_to waits vmcnt(0) before the LDS read
                const uint32_t lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t *)ring_stage;
                // (lane offset computed inside: hoisted, it would hold a VGPR for the whole kernel)
                uint32_t m0_save, voff;  // m0 is reserved to the compiler (writelane lane selects): restore it
                asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\tv_lshlrev_b32 %1, 2, %3\n\t"
                             "global_load_lds_dword %1, %4\n\ts_mov_b32 m0, %0"
                             : "=&s"(m0_save), "=&v"(voff)
                             : "s"(lds), "v"(lane), "s"(src + 256 * sg)
                             : "memory");
                staged = sg + 1;
            }
        }
    };
    stage(seg_hi);
    // make segments < need resident (a long jump reloads at most the last 128).
    // PF (the window refresh, which moves the ring one segment at a time): take
    // the staged segment and stage the next; match extension loads directly.
    auto ring_to = [&](uint32_t need, auto pf) {
        if constexpr (BIG) {
            if (__builtin_expect(need <= seg_hi, 1)) return;
            uint32_t sg = need - seg_hi > kRegs ? need - kRegs : seg_hi;
            if (decltype(pf)::value && staged == sg + 1) {  // the DMA was issued an advance ago
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const uint32_t lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t *)ring_stage;
                uint32_t w;
                asm volatile("v_lshl_add_u32 %0, %1, 2, %2\n\tds_read_b32 %0, %0\n\ts_waitcnt lgkmcnt(0)"
                             : "=&v"(w) : "v"(lane), "s"(lds) : "memory");
                REG_SET_V(sg & (kRegs - 1), __builtin_bswap32(w));
                sg++;
            }
            for (; sg < need; sg++) {
                K1R_COUNT(n_reload);
                REG_SET_V(sg & (kRegs - 1), load_word(sg));
            }
            seg_hi = need;
            if (decltype(pf)::value) stage(seg_hi);  // REG_SET_V consumed the LDS read: the DMA may overwrite it
        }
    };
    // lane i <- big-endian dword dd + i: from the registers, or (BIG, a segment
    // that left the ring) from global memory
#define CAND_LANES(dd)                                                                             \
    ({                                                                                             \
        const uint32_t _cd = (dd);                                                                 \
        uint32_t _cv;                                                                              \
        if constexpr (BIG) {                                                                       \
            if (__builtin_expect((_cd >> 6) + kRegs >= seg_hi, 1)) _cv = DW_LANES(_cd);             \
            else { K1R_COUNT(n_farc); _cv = load_dw(_cd + lane); }                                  \
        } else {                                                                                   \
            _cv = DW_LANES(_cd);                                                                   \
        }                                                                                          \
        _cv;                                                                                       \
    })

    uint32_t T = 256, lg = 8;  // set_htable_size :198-204
    while (T < kTable && T < L) { T <<= 1; lg++; }
    const uint32_t shift = 32 - lg;

    // never-set slots mean position 0 (snappy_compression.c:259-265): tag of BE32(0)
    const uint32_t cur0 = __builtin_amdgcn_readfirstlane(REG_OF(0));
    const uint32_t init = TAG_OF(cur0) << 16;
    for (uint32_t i = lane; i < kTable; i += 64) TBL_WRITE(i, init);
    __syncthreads();

    // tokens, 4 bytes each: offset | (length - 4) << 16 | gap << 24, gap = the
    // literal bytes before the copy; a length or gap that does not fit 8 bits
    // (255 = escape) puts gap | length << 16 in the same slot of a second array
    // (after all units' words), written only for those tokens
    uint32_t *tok = reinterpret_cast<uint32_t *>(tokens) + (uint64_t)u * tok_cap;
    uint32_t *tok_full = reinterpret_cast<uint32_t *>(tokens) + ((uint64_t)gridDim.x + u) * tok_cap;
    uint32_t tka = 0, tkb = 0;  // pending tokens: lane t < pend holds token nt + t
    uint32_t nt = 0, pend = 0;
    // encoded size so far (header, literals, copies: src/snappy_compression.c:95-165)
    // and the end of the last flushed token; K2 segments start every kK2Seg tokens
    uint32_t acc = 0, cend = 0;
    if (hdr_mode == SNAPPY_HDR_EVERY_UNIT) acc = varint_len(L);
    else if (hdr_mode == SNAPPY_HDR_FIRST_UNIT && u == 0) acc = varint_len(header_value);
    // K2 segment k (tokens kK2Seg k ..): its output offset in the unit and the
    // input position where its first token's literal starts
    uint32_t *const segu = seg_off + 2 * (uint64_t)u * segs;
    auto flush_tokens = [&]() {
        const bool has = lane < pend;
        const uint32_t pos = tka & 0xFFFF, len = tka >> 16, end = pos + len;
        // lane l <- end of lane l - 1; lane 0 keeps cend (no bound_ctrl: the old value stays)
        const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp((int)cend, (int)end, 0x138, 0xF, 0xF, false);
        const uint32_t litn = pos - prev;
        if (has) {
            const uint32_t lc = len - 4 < 255 ? len - 4 : 255u, gc = litn < 255 ? litn : 255u;
            tok[nt + lane] = tkb | (lc << 16) | (gc << 24);
            if (lc == 255 || gc == 255) tok_full[nt + lane] = litn | (len << 16);
        }
        const uint32_t b = has ? (litn ? literal_bytes(litn) : 0u) + copy_bytes(len, tkb) : 0u;
        uint32_t tot;
        const uint32_t ex = wave_excl_scan(b, lane, &tot);
        if (has && ((nt + lane) & (kK2Seg - 1)) == 0)
            *reinterpret_cast<uint2 *>(segu + 2 * ((nt + lane) / kK2Seg)) = make_uint2(acc + ex, prev);
        if (pend) cend = __builtin_amdgcn_readlane(end, pend - 1);
        acc += tot;
        nt += pend;
        pend = 0;
    };

    // ---- position window at q0 (see the header): dv = dwords q0/4 .. q0/4 + 63,
    // rotated: dword q0/4 + i sits at lane (dr + i) % 64 (ds_bpermute wraps addr[7:2])
    uint32_t q0 = 0, d0 = 0, dr = 0, dv = 0, bv = 0, hv = 0;
    uint32_t pdl1 = 0, pdc = 0;               // lane-space data: predecessor lane + 1, its position
    // the slot's entry and its tag as the loads' own types: a widened copy would
    // make the compiler zero-extend (and wait for) a load where it is issued
    uint16_t ent = 0;
    uint8_t ent_t = 0;
    uint32_t adr = 0, word = 0;               // the lane's table record address and its insert word
    uint32_t pdnz = 0;  // the predecessor's tag
    uint64_t m_win = 0, m_win17 = 0;
    bool lsw = false;  // the lane-space data describe the current window
// SNAPPY_K1R_WIN_ALIGN: a window's per-lane BE32 by v_alignbit from (p - 1) / 4
// (as the round loop's pa funnel, V6) instead of v_perm with a per-lane
// selector from a 32-bit multiply; 32 KiB units only (A/B, outputs identical,
// profiles/r05zj_*: 32 KiB streams 12.64 -> 12.55-12.57 ms per GiB, but 64 KiB
// blocks 14.06 -> 14.41 in K1r64's schedule)
#ifndef SNAPPY_K1R_WIN_ALIGN
#define SNAPPY_K1R_WIN_ALIGN 1
#endif
#define WINDOW_AT(qq)                                                                              \
    do {                                                                                           \
        q0 = (qq);                                                                                 \
        ring_to((q0 >> 8) + 2, std::true_type{}); /* BIG: the window's segments and the next */    \
        d0 = q0 >> 2;                                                                              \
        dr = d0 & 63;                                                                              \
        {                                                                                          \
            uint32_t _r0, _r1;                                                                     \
            REG_PAIR(d0 >> 6, _r0, _r1);                                                           \
            dv = lane >= dr ? _r0 : _r1;                                                           \
        }                                                                                          \
        if (SNAPPY_K1R_WIN_ALIGN == 2 || (SNAPPY_K1R_WIN_ALIGN && !BIG)) { \
            /* the dwords from (p - 1) / 4 funnelled by v_alignbit with the lane's */              \
            /* shift -8 p (bits 4:0; 0 takes the second dword, the one at p) */                    \
            const uint32_t _p = q0 + lane;                                                          \
            const uint32_t _k = (_p - 1) >> 2; /* rotated by dr = d0 % 64 */                       \
            const uint32_t _a = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(_k << 2), (int)dv);   \
            const uint32_t _b = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((_k + 1) << 2), (int)dv); \
            bv = __builtin_amdgcn_alignbit(_a, _b, 0u - (_p << 3));                                  \
        } else {                                                                                   \
            const uint32_t _k = d0 + (((q0 & 3) + lane) >> 2); /* rotated by dr = d0 % 64 */     \
            const uint32_t _a = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(_k << 2), (int)dv);   \
            const uint32_t _b = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((_k + 1) << 2), (int)dv); \
            bv = funnel_bytes(_a, _b, perm_sel((q0 + lane) & 3));                                 \
        }                                                                                          \
        {                                                                                          \
            const uint32_t _pr = bv * kMul;                                                        \
            hv = (_pr >> shift) | (__builtin_amdgcn_ubfe(_pr, shift - 8, 8) << 16);                \
        }                                                                                          \
    } while (0)
// A window refresh reads the new window's table entries as soon as the
// addresses are known (their LDS round trip overlaps the lane data), not after
// it (the later read: +2.9-3.2 % at every loop placement, profiles/r06q_*)
#define WINDOW_LS(qq)                                                                              \
    do {                                                                                           \
        WINDOW_AT(qq);                                                                             \
        adr = TBL_ADR(hv & 0xFFFF);                                                                \
        TBL_READ_ENT(adr); /* in flight during the lane data below */                             \
        const uint32_t _bits = same_x_bits<DMAX>((hv & 0xFFFF) + 1);                               \
        const uint32_t _pd = _bits ? (uint32_t)__builtin_ctz(_bits) : 0u;                          \
        /* lane - pd + 1, or lane - 1 at pd = 1: pdl1 >= lane0 also implies lane > lane0 */      \
        pdl1 = _bits ? lane - _pd + 1 - (_pd == 1 ? 1u : 0u) : 0xFFFFFF00u; /* signed: below every lane0 */ \
        pdc = q0 + lane - _pd;                                                                     \
        const uint32_t _hp = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane - _pd) << 2), (int)hv); \
        /* the predecessor's tag */                                                                \
        pdnz = (_hp >> 16) & 0xFFu;                                                                \
        /* probe lanes: <= 62 and not past is_block_end (L - p >= 16, 17 at skip 64) */           \
        const int32_t _w16 = (int32_t)(L - 16 - q0), _w17 = (int32_t)(L - 17 - q0);              \
        const bool _inw = (int32_t)lane <= _w16 && lane <= 62;                                     \
        m_win = __ballot(_inw);                                                                    \
        m_win17 = __ballot((int32_t)lane <= _w17 && lane <= 62);                                   \
        word = (q0 + lane) | (hv & 0xFF0000u);                                                     \
        if (!_inw) word |= 1u << 24; /* the asm hit test sees the window mask in the lane data */   \
        lsw = true; /* the caller reads ent */                                                     \
    } while (0)

    // find_copy_length :61-72 after found_match :259-265: common prefix of the
    // bytes at pf (pf - q0 <= 62: its dwords come from dv) and cand
    // (registers); lanes 0..15 compare 64 bytes, then 252 per pass
    // common prefix continued from len (all bytes before it equal), 252 bytes per pass
    auto match_len_from = [&](uint32_t pf, uint32_t cand, uint32_t len) -> uint32_t {
            for (;;) {
                if (pf + len >= L) break;
                const uint32_t qa = pf + len, qb = cand + len;
                ring_to((qa >> 8) + 2, std::false_type{});
                const uint32_t a0 = DW_LANES(qa >> 2), b0 = CAND_LANES(qb >> 2);
                const uint32_t va = funnel_bytes(a0, wave_shl1(a0), perm_sel(qa & 3));
                const uint32_t vb = funnel_bytes(b0, wave_shl1(b0), perm_sel(qb & 3));
                const uint32_t yy = lane < 63 ? (va ^ vb) : 0;  // lane 63 lacks its successor
                const uint64_t bb = __ballot(yy != 0);
                if (bb) {
                    const uint32_t m = (uint32_t)__builtin_ctzll(bb);
                    len += 4 * m + ((uint32_t)__builtin_clz(__builtin_amdgcn_readlane(yy, m)) >> 3);
                    break;
                }
                len += 252;
            }
        return len;
    };
    auto match_len = [&](uint32_t pf, uint32_t cand) -> uint32_t {
        const uint32_t pa = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((pf >> 2) + lane) << 2), (int)dv);
        const uint32_t ca = CAND_LANES(cand >> 2);
        const uint32_t pv = funnel_bytes(pa, wave_shl1(pa), perm_sel(pf & 3));
        const uint32_t cv = funnel_bytes(ca, wave_shl1(ca), perm_sel(cand & 3));
        const uint32_t y = pv ^ cv;
        const uint64_t bad = __ballot(y != 0) & 0xFFFFull;
        if (bad) {
            const uint32_t m = (uint32_t)__builtin_ctzll(bad);
            return 4 * m + ((uint32_t)__builtin_clz(__builtin_amdgcn_readlane(y, m)) >> 3);
        }
        return match_len_from(pf, cand, 64);
    };
    // emit_copy :323-329 as a token (the caller inserts pf into the table)
    // (pend < 64 on entry: lane-space windows flush at refresh when more than
    // 48 are pending -- a window of <= 62 probe positions holds <= 16 matches --
    // and W-probe rounds flush when 64 are pending)
    auto put_token = [&](uint32_t pf, uint32_t len, uint32_t off) {
        tka = (uint32_t)amdgcn_writelane((int)(pf | (len << 16)), (int)pend, (int)tka);
        tkb = (uint32_t)amdgcn_writelane((int)off, (int)pend, (int)tkb);
        pend++;
    };
    // lane-space rounds defer a match's token into the next round, where its
    // writelanes fill the wait for the verification gather (dka/dkb, dkn = 0/1;
    // with dkn = 0 the writelanes hit lane pend, which the next token overwrites)
    uint32_t dka = 0, dkb = 0, dkn = 0;
    auto drain_token = [&]() {
        tka = (uint32_t)amdgcn_writelane((int)dka, (int)pend, (int)tka);
        tkb = (uint32_t)amdgcn_writelane((int)dkb, (int)pend, (int)tkb);
        pend += dkn;
        dkn = 0;
    };

#ifdef SNAPPY_K1R_RSTAMPS
    const uint64_t t_loop = clock64();
    uint64_t rs_flush = 0, rs_win = 0, rs_asm = 0;
    uint32_t rs_n = 0, rs_nfl = 0, rs_nasm = 0, rs_code[6] = {0, 0, 0, 0, 0, 0};
#endif
#ifdef SNAPPY_K1R_STATS
    const uint64_t t_loop = clock64();
    uint32_t n_probe = 0, n_match = 0, n_round = 0, n_refresh = 0;
#endif

    // ---- k1r_asm_rounds: the lane-space round of the C++ loop below (32 KiB
    // units), hand-scheduled as one loop: drain the deferred token, hit ballot,
    // first hit f and its candidate c, the 64 bytes at pf = q0 + f and at c
    // gathered (ds_bpermute; c's registers by s_set_gpr_idx), the inserts of
    // lanes lo0..f (lane-ordered, highest lane wins a slot), the next round's
    // entries read while the verification runs, the match length from the
    // first differing byte; a round without a hit inserts its nk probes.  It
    // leaves the loop with `code`: 1 = skip past the step-1 range or
    // is_block_end, 2 = the window must move (refresh), 3 = the next round's
    // probes reach a step of 2 (skip > 64 - DMAX: the C++ round), and mid-round
    // (inserts done, entries read) 4 = 64 or more equal bytes (C++ extends the
    // match), 5 = a tag collision (C++ finishes the miss).  Everything the
    // compiler schedules around it -- waits, DPP, cross-lane reads -- is
    // written out with its wait states: a VALU-written SGPR or VCC is read by
    // VALU two states later (v_cndmask, v_readlane sources); LDS results are
    // waited for by count (pa, ca before the two entry reads); it exits with
    // lgkmcnt(0), so `ent`/`ent_t` are complete when the compiler reads them.
    // m0 (the writelane lane select) is saved and restored.  The loop always
    // advances p (a match by >= 4, a missing round by nk >= 1), so it ends.
    // A/B on 1 GiB of 32 KiB text streams, outputs identical (profiles/
    // r04b_ab_k1r_asm_rounds_text32k.log): the C++ round 15.98-16.02 ms, this
    // loop 15.85-15.86 ms; a variant that drains the token at the loop top
    // 16.21-16.23, one that gathers at the first probe before the hit ballot
    // (60 % of text matches are there) 17.49-17.52 (its extra LDS traffic and
    // issue cost more than the latency it hides).  SNAPPY_K1R_CXX_ROUNDS keeps
    // the C++ round (the statistics and stamp builds always do).
#if !defined(SNAPPY_K1R_STATS) && !defined(SNAPPY_K1R_LSTAMPS) && !defined(SNAPPY_K1R_CXX_ROUNDS)
#define K1R_ASM_ROUNDS 1
#else
#define K1R_ASM_ROUNDS 0
#endif
#if K1R_ASM_ROUNDS
// Round 5 took the loop through A/B variants V2-V20 (1 GiB of 32 KiB streams and
// of 64 KiB blocks each, outputs checked identical; DESIGN.md 4.2 lists them, the
// logs are profiles/r05e_* .. r05zk_*).  What stayed, in the order the round runs:
//  * the hit test: the candidate of every lane (in-window predecessor or table
//    entry) and its tag compared in one SDWA compare (the lane data carry the
//    predecessor's tag, V16); a lane past the window has bit 24 of its
//    word set, so it never matches (V6); the hit branch on the SCC of the s_and
//    that makes the hit mask (V2)
//  * pa: the dwords at pf gathered from (pf - 1) / 4 and funnelled by v_alignbit
//    with the shift -8 pf from v_mul_i32_i24 (bits 4:0; 0 takes the second
//    dword, the one at pf) (V6, V10)
//  * ca: the candidate's register pair R, R + 1 selected by one v_cndmask with
//    s_set_gpr_idx on SRC0 and SRC1 (lanes >= l0 take R; V15); K1r64 reads ring
//    registers (c / 256) mod 128: a candidate whose segment left the ring is
//    gathered from the input (global_load_dword, byte-swapped to the ring's
//    big-endian dwords; V19), the wrap pair 127 / 0 by a select of v129 / v2
//    without a register index (round 6; it left for the C++ round before:
//    64 KiB blocks 14.11 -> 14.14-14.18 ms per GiB unpinned, within the loop
//    placement's +-2 %, profiles/r06e_ab_*)
//  * the previous round's token drained into tka / tkb during the gathers, its
//    first word by one s_pack_ll_b32_b16 (V9); lo0 = lane0 - (lane0 < f) by
//    s_subb (V5)
//  * the wait for pa and ca alone; the inserts of lanes lo0 .. f under an exec
//    mask from one s_bfm_b64 (at most DMAX + 1 lanes, so the 6-bit size never
//    wraps; no dummy-record writes: V13) and the next round's entry reads issued
//    after it, behind the funnels (V18)
//  * the prefix length per lane as (clz(xor) >> 3) | 4 lane, read back from the
//    first differing dword (V3, V7); skip is not reset by a hit round (a pending
//    token implies skip 32, V8); the clamp to the block end only on the exit path
// Each masked insert restores exec to its value where the statement runs (sx,
// read by the compiler: the statement runs in uniform control flow with all
// 64 lanes live, and exec cannot be declared clobbered).
// SNAPPY_K1R_PAD32 / SNAPPY_K1R_PAD64: the loop's first instruction placed
// at byte 4*PAD of a 64-byte line (-1: wherever the code before it ends).  The
// same loop code placed 4 bytes apart measured 1.8 % apart (profiles/r05zn_*,
// r05zo_*), so the placement is pinned to the measured best instead of being
// left to the code around the statement.  The padding (s_nop) runs once per
// entry into the asm loop.  Re-swept with DMAX 13 / 12 and RMIN 2 (profiles/
// r06n_*): PAD32 0..15 -> 12.18 (2) to 12.79 (13) ms per GiB; PAD64 -1 13.93,
// 0..14 even 14.00-14.55.  With SNAPPY_K1R_X45 (r06x_*): PAD32 0 best (12.13-12.20;
// 12.20-12.53 elsewhere), PAD64 -1 best (13.85-13.88; 13.92-14.53 pinned).
#ifndef SNAPPY_K1R_PAD32
#define SNAPPY_K1R_PAD32 2  // with SNAPPY_K1R_EARLY_DK (profiles/r06ag_*, r06ah_*)
#endif
#ifndef SNAPPY_K1R_PAD64
#define SNAPPY_K1R_PAD64 0  // with SNAPPY_K1R64_HALF32 (profiles/r06aa_*, r06ad_*)
#endif
#ifndef SNAPPY_K1R_PAD64A  // K1r64's first-32-KiB loop (SNAPPY_K1R64_HALF32; -1 with EARLY_DK, r06ah_*)
#define SNAPPY_K1R_PAD64A -1
#endif
#ifndef SNAPPY_K1R64_HALF32
#define SNAPPY_K1R64_HALF32 1
#endif
#define K1R_STR2(x) #x
#define K1R_STR(x) K1R_STR2(x)
#define K1R_LOOP_PLACE(pad) ".if " K1R_STR(pad) " >= 0\n.p2align 6\n.rept " K1R_STR(pad) "\ns_nop 0\n.endr\n.endif\n"
#define K1R_CAND32 "s_lshr_b32 %[s0], %[c], 8\n\t"
// K1r64: residency as one compare of c against the first resident position
// (seghi = (seg_hi - 128) * 256; r05b_ab_k4_k1r64_cand_text64k.log: 18.70 ->
// 18.08 ms per GiB), the segment's register by one s_bfe
#define K1R_CAND64                                                                                  \
    "s_cmp_lt_u32 %[c], %[seghi]\n\t"                                                              \
    "s_cbranch_scc1 L%=_far\n\t"                                                                   \
    "s_bfe_u32 %[s0], %[c], 0x70008\n\t"                                                           \
    "s_cmp_eq_u32 %[s0], 127\n\t"                                                                  \
    "s_cbranch_scc1 L%=_wrap\n\t" /* the wrap pair 127 / 0: gathered below, no register index */
#define K1R_SEGHI64(seg_hi) "s"(((seg_hi) - kRegs) << 8)
#define K1R_HIT_PREDTAG                                                                             \
    "v_cndmask_b32_sdwa %[t1], %[pdc], %[ent], vcc dst_sel:DWORD dst_unused:UNUSED_PAD "             \
    "src0_sel:DWORD src1_sel:WORD_0\n\t" /* the candidate of every lane */                          \
    "v_cndmask_b32_e32 %[t0], %[pdnz], %[entt], vcc\n\t" /* and its tag */                          \
    "v_cmp_eq_u32_sdwa %[hm], %[t0], %[word] src0_sel:DWORD src1_sel:WORD_1\n\t"
#define K1R_HIT32 K1R_HIT_PREDTAG
#define K1R_HIT64 K1R_HIT_PREDTAG
#define K1R_DRAIN                                                                                   \
    K1R_DRAIN_PACK                                                                                  \
    "s_mov_b32 m0, %[pend]\n\t" /* (gfx950 refuses two SGPRs in a v_writelane: m0 stays) */          \
    "v_writelane_b32 %[tka], %[dka], m0\n\t"                                                        \
    "v_writelane_b32 %[tkb], %[dkb], m0\n\t"                                                        \
    "s_add_u32 %[pend], %[pend], %[dkn]\n\t"
#define K1R_SKIPFIX "s_cmp_eq_u32 %[dkn], 0\n\ts_cselect_b32 %[skip], %[skip], 32\n\t"
// the round's inserts (lanes lo0 .. f, or the misses' lanes) under an exec mask,
// exec restored to its value at the statement (sx), then the next round's entries
#define K1R_INSERTS(cnt, lo)                                                                        \
    "s_bfm_b64 exec, " cnt ", " lo "\n\t"                                                          \
    "ds_write_b16 %[adr], %[word]\n\t"                                                              \
    "ds_write_b8_d16_hi %[adrt], %[word] offset:%[tagb]\n\t"                                        \
    "s_mov_b64 exec, %[sx]\n\t"                                                                     \
    "ds_read_u16 %[ent], %[adr]\n\t" /* the next round's entries */                                  \
    "ds_read_u8 %[entt], %[adrt] offset:%[tagb]\n\t"
// the match length: lane s1 (the first differing dword of the 64 bytes, -1 if
// none in lanes 0-31) gives 4 s1 + the byte.  SNAPPY_K1R_X45: one unsigned test
// of len - 4 > 59 leaves for both rare ends (>= 64 equal bytes: s1 > 15, or -1,
// whose lane 63 reads >= 252; a tag collision: len < 4), told apart at the exit:
// one compare and one branch fewer per hit round, K1r 12.18-12.24 -> 12.11-12.17 ms
// per GiB and K1r64 13.94-13.98 -> 13.82-13.86, each at its best loop placement
// (profiles/r06x_*, r06y_*, outputs identical)
#ifndef SNAPPY_K1R_X45
#define SNAPPY_K1R_X45 1
#endif
// SNAPPY_K1R_PACK_DRAIN: a hit round leaves its token as pf (dka) and the length
// (dlen, the read-back's own register) and the next round's drain packs them
// (one s_pack in the drain, one s_mov of pf in the gather wait's shadow) instead
// of an s_pack on the tail after the length read-back; every exit that keeps a
// token pending packs it itself (the leaving path) or hands it to C++ (codes 4/5).
// Slower at every loop placement (A/B, outputs identical, 68 GPU tests green,
// profiles/r06aj_*: K1r 12.04 -> 12.18 at best, K1r64 13.49-13.51 -> 13.67 at
// best: the pack now sits on the next round's drain before its writelanes), so off
#ifndef SNAPPY_K1R_PACK_DRAIN
#define SNAPPY_K1R_PACK_DRAIN 0
#endif
#if SNAPPY_K1R_PACK_DRAIN
#define K1R_LEN "%[dlen]"
#define K1R_DRAIN_PACK "s_pack_ll_b32_b16 %[dka], %[dka], %[dlen]\n\t"
#define K1R_DKA_SHADOW "s_mov_b32 %[dka], %[pf]\n\t"
#define K1R_DKA_TAIL
#define K1R_DLEN_DECL uint32_t _dlen = dka >> 16; /* the pending token's length */
#define K1R_DLEN_OP [dlen] "+s"(_dlen),
#else
#define K1R_LEN "%[s0]"
#define K1R_DRAIN_PACK
#define K1R_DKA_SHADOW
#define K1R_DKA_TAIL "s_pack_ll_b32_b16 %[dka], %[pf], %[s0]\n\t"
#define K1R_DLEN_DECL
#define K1R_DLEN_OP
#endif
#if SNAPPY_K1R_X45
#define K1R_LENCHECK                                                                                \
    "v_readlane_b32 " K1R_LEN ", %[t2], %[s1]\n\t"                                                 \
    "s_add_u32 %[s2], " K1R_LEN ", -4\n\t"                                                          \
    "s_cmp_gt_u32 %[s2], 59\n\t"                                                                    \
    "s_cbranch_scc1 L%=_x4\n\t"
#define K1R_X4 "s_cmp_lt_u32 " K1R_LEN ", 4\n\ts_cbranch_scc1 L%=_x5\n\ts_mov_b32 %[code], 4\n\ts_branch L%=_end\n"
#else
#define K1R_LENCHECK                                                                                \
    "s_cmp_gt_u32 %[s1], 15\n\t"                                                                    \
    "s_cbranch_scc1 L%=_x4\n\t"                                                                    \
    "v_readlane_b32 %[s0], %[t2], %[s1]\n\t"                                                       \
    "s_cmp_lt_u32 %[s0], 4\n\t" /* (pf <= L - 16: the clamp below never makes it < 4) */           \
    "s_cbranch_scc1 L%=_x5\n\t"
#define K1R_X4 "s_mov_b32 %[code], 4\n\ts_branch L%=_end\n"
#endif
// SNAPPY_K1R_EARLY_INS: a hit round's inserts and next entry reads issued as
// soon as the insert range is known, before the wait for the gathers, which
// then waits for pa and ca alone (lgkmcnt(4): one wave's LDS operations
// complete in order; the K1r64 far path's ca is a global load, so there the
// count leaves pa's four successors); 0: after the funnels (round 5's V18).
// Measured slower at every loop placement (A/B, outputs identical, 68 GPU tests
// green on it, profiles/r06z_*: K1r 12.09-12.12 -> 12.18 at best, 12.26-12.59
// elsewhere; K1r64 equal), so off
#ifndef SNAPPY_K1R_EARLY_INS
#define SNAPPY_K1R_EARLY_INS 0
#endif
#if SNAPPY_K1R_EARLY_INS
#define K1R_INS_EARLY K1R_INSERTS("%[s2]", "%[s0]")
#define K1R_INS_LATE
#define K1R_GATHER_WAIT "s_waitcnt lgkmcnt(4)\n\t" /* pa and ca; the inserts and entry reads stay in flight */
#else
#define K1R_INS_EARLY
#define K1R_INS_LATE K1R_INSERTS("%[s2]", "%[s0]")
#define K1R_GATHER_WAIT "s_waitcnt lgkmcnt(0)\n\t" /* pa and ca */
#endif
// the miss round's way on: SNAPPY_K1R_NOHIT2 tests the common case first --
// lane0 <= lim0 = min(62 - RMIN, L - 16 - q0) (window and block end in one
// signed compare, as the hit path) and skip <= skipmax -- and tells the rare
// ends apart after it; 0: the four tests in turn.  Two compares and two branches
// fewer per miss round, yet slower at every loop placement (A/B, outputs
// identical, profiles/r06ae_*: K1r 12.10-12.13 -> 12.16-12.45 ms per GiB, K1r64
// 13.57 -> 13.58-13.69), so off
#ifndef SNAPPY_K1R_NOHIT2
#define SNAPPY_K1R_NOHIT2 0
#endif
#if SNAPPY_K1R_NOHIT2
#define K1R_NOHIT_TAIL(T)                                                                           \
    "s_cmp_le_i32 %[lane0], %[lim0]\n\t"                                                           \
    "s_cbranch_scc0 L%=_nx" T "\n\t"                                                              \
    "s_cmp_le_u32 %[skip], %[skipmax]\n\t"                                                         \
    "s_cbranch_scc1 L%=_top" T "\n\t"                                                             \
    "s_cmp_gt_u32 %[skip], %[lsmax]\n\t"                                                           \
    "s_cbranch_scc1 L%=_x1\n\t"                                                                    \
    "s_branch L%=_x3\n"                                                                            \
    "L%=_nx" T ":\n\t"                                                                            \
    "s_cmp_gt_u32 %[skip], %[lsmax]\n\t"                                                           \
    "s_cbranch_scc1 L%=_x1\n\t"                                                                    \
    "s_cmp_gt_u32 %[p], %[lm16]\n\t"                                                               \
    "s_cbranch_scc1 L%=_x1\n\t"                                                                    \
    "s_branch L%=_x2\n"
#else
#define K1R_NOHIT_TAIL(T)                                                                           \
    "s_cmp_gt_u32 %[skip], %[lsmax]\n\t"                                                           \
    "s_cbranch_scc1 L%=_x1\n\t"                                                                    \
    "s_cmp_gt_u32 %[p], %[lm16]\n\t"                                                               \
    "s_cbranch_scc1 L%=_x1\n\t"                                                                    \
    "s_cmp_gt_u32 %[lane0], %[l0max]\n\t"                                                          \
    "s_cbranch_scc1 L%=_x2\n\t"                                                                    \
    "s_cmp_le_u32 %[skip], %[skipmax]\n\t"                                                         \
    "s_cbranch_scc1 L%=_top" T "\n"
#endif
// SNAPPY_K1R_EARLY_DK: a hit round's token offset written right after the drain
// that consumed the previous one (in the gather wait's shadow) instead of on the
// tail after the length read-back.  (The pending flag stays on the tail: the
// code-5 exit's skip fix reads the previous round's.)  A/B, outputs identical,
// 68 GPU tests green, at each build's best placements (profiles/r06ag_*, r06ah_*):
// K1r 12.11-12.13 -> 12.04-12.08 ms per GiB, K1r64 13.55-13.60 -> 13.49-13.51
#ifndef SNAPPY_K1R_EARLY_DK
#define SNAPPY_K1R_EARLY_DK 1
#endif
#if SNAPPY_K1R_EARLY_DK
#define K1R_DK_EARLY "s_sub_u32 %[dkb], %[pf], %[c]\n\t"
#define K1R_DK_LATE "s_mov_b32 %[dkn], 1\n\t"
#else
#define K1R_DK_EARLY
#define K1R_DK_LATE "s_sub_u32 %[dkb], %[pf], %[c]\n\ts_mov_b32 %[dkn], 1\n\t"
#endif
// one round loop of the asm statement (labels suffixed with T)
#define K1R_ROUND_BODY(CAND, HIT, T)                                                                \
            "L%=_top" T ":\n\t"                                                                          \
            "s_lshl_b64 %[valid], %[dmask], %[lane0]\n\t"                                           \
            "v_cmp_gt_i32_e32 vcc, %[lane0], %[pdl1]\n\t" /* vcc = not in-round */                  \
            "s_waitcnt lgkmcnt(0)\n\t"                                                              \
            HIT                                                                                     \
            "s_and_b64 %[hm], %[hm], %[valid]\n\t"                                                  \
            "s_cbranch_scc0 L%=_nohit" T "\n\t" /* SCC = (hm != 0) */                                     \
            "s_ff1_i32_b64 %[f], %[hm]\n\t"                                                         \
            "v_readlane_b32 %[c], %[t1], %[f]\n\t"                                                  \
            "s_add_u32 %[pf], %[q0], %[f]\n\t"                                                      \
            "v_add3_u32 %[t2], %[pf], -1, %[lane4]\n\t" /* dwords from (pf - 1) / 4 */              \
            "ds_bpermute_b32 %[t2], %[t2], %[dv]\n\t" /* pa: dwords at pf */                        \
            CAND                                                                                    \
            "s_bfe_u32 %[s1], %[c], 0x60002\n\t"                                                    \
            "v_cmp_le_u32_e32 vcc, %[s1], %[lane]\n\t" /* lanes >= l0 take register R */           \
            "v_add_u32_e32 %[t1], %[c], %[lane4]\n\t"                                               \
            "s_set_gpr_idx_on %[s0], gpr_idx(SRC0,SRC1)\n\t"                                        \
            "v_cndmask_b32_e32 %[t3], v3, v2, vcc\n\t"                                              \
            "s_set_gpr_idx_off\n\t"                                                                 \
            "ds_bpermute_b32 %[t3], %[t1], %[t3]\n\t" /* ca: dwords at c */                         \
            "L%=_farret" T ":\n\t"                                                                       \
            K1R_DRAIN /* the previous round's token, during the gathers */                         \
            K1R_DK_EARLY                                                                            \
            K1R_DKA_SHADOW                                                                          \
            "s_cmp_lt_u32 %[lane0], %[f]\n\t"                                                       \
            "s_subb_u32 %[s0], %[lane0], 0\n\t" /* lo0 */                                           \
            "v_mul_i32_i24_e64 %[t0], %[pf], -8\n\t" /* pa's funnel shift */                        \
            "s_sub_u32 %[s2], %[f], %[s0]\n\t"                                                      \
            "s_add_u32 %[s2], %[s2], 1\n\t" /* lanes lo0 .. f insert */                             \
            K1R_INS_EARLY                                                                           \
            "s_and_b32 %[s3], %[c], 3\n\t"                                                          \
            "s_mul_i32 %[s3], %[s3], 0xfefefeff\n\t"                                                \
            "s_add_i32 %[s3], %[s3], 0x7060504\n\t" /* ca's perm selector */                        \
            K1R_GATHER_WAIT                                                                         \
            "v_mov_b32_dpp %[t1], %[t2] wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"     \
            "v_mov_b32_dpp %[t4], %[t3] wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"     \
            "v_alignbit_b32 %[t2], %[t2], %[t1], %[t0]\n\t"                                         \
            "v_perm_b32 %[t3], %[t3], %[t4], %[s3]\n\t"                                             \
            K1R_INS_LATE                                                                            \
            "v_cmp_ne_u32_e32 vcc, %[t2], %[t3]\n\t"                                                \
            "v_xor_b32_e32 %[t2], %[t2], %[t3]\n\t"                                                 \
            "v_ffbh_u32_e32 %[t2], %[t2]\n\t"                                                       \
            "v_bfe_u32 %[t2], %[t2], 3, 2\n\t"                                                      \
            "v_lshl_or_b32 %[t2], %[lane], 2, %[t2]\n\t" /* the prefix length if this dword differs */ \
            "s_ff1_i32_b32 %[s1], vcc_lo\n\t"                                                       \
            K1R_LENCHECK                                                                            \
            "s_add_u32 %[lane0], %[f], " K1R_LEN "\n\t"                                             \
            K1R_DKA_TAIL                                                                            \
            K1R_DK_LATE                                                                             \
            "s_cmp_le_i32 %[lane0], %[lim0]\n\t" /* implies pf + len <= L - 16: no clamp */         \
            "s_cbranch_scc1 L%=_top" T "\n\t"                                                            \
            "s_sub_u32 %[s2], %[L], %[pf]\n\t" /* leaving: the length clamped to the block end */ \
            "s_min_u32 " K1R_LEN ", " K1R_LEN ", %[s2]\n\t"                                          \
            "s_add_u32 %[p], %[pf], " K1R_LEN "\n\t"                                                \
            "s_sub_u32 %[lane0], %[p], %[q0]\n\t"                                                   \
            "s_lshl_b32 %[s1], " K1R_LEN ", 16\n\t"                                                 \
            "s_or_b32 %[dka], %[s1], %[pf]\n\t"                                                     \
            "s_cmp_gt_u32 %[p], %[lm16]\n\t"                                                        \
            "s_cbranch_scc1 L%=_x1\n\t"                                                             \
            "s_branch L%=_x2\n"                                                                     \
            "L%=_nohit" T ":\n\t"                                                                        \
            K1R_SKIPFIX                                                                             \
            "s_and_b64 %[valid], %[valid], %[mwin]\n\t"                                             \
            "s_bcnt1_i32_b64 %[s0], %[valid]\n\t" /* nk misses: lanes lane0 - 1 .. lane0 + nk - 1 */ \
            K1R_DRAIN                                                                               \
            "s_mov_b32 %[dkn], 0\n\t"                                                               \
            "s_add_i32 %[s1], %[lane0], -1\n\t"                                                     \
            "s_add_u32 %[s2], %[skip], %[s0]\n\t"                                                   \
            "s_add_i32 %[s3], %[s2], -1\n\t"                                                        \
            "s_add_u32 %[c], %[s0], 1\n\t" /* (c is free on this path) */                          \
            K1R_INSERTS("%[c]", "%[s1]") /* lanes lane0 - 1 .. lane0 - 1 + nk */                    \
            "s_lshr_b32 %[s3], %[s3], 5\n\t" /* the last probe steps by 2 at skip 64 */             \
            "s_add_u32 %[lane0], %[s1], %[s0]\n\t" /* lane0 - 1 + nk + the step-2 probe */          \
            "s_add_u32 %[lane0], %[lane0], %[s3]\n\t"                                               \
            "s_add_u32 %[p], %[q0], %[lane0]\n\t"                                                   \
            "s_mov_b32 %[skip], %[s2]\n\t"                                                          \
            K1R_NOHIT_TAIL(T)
// SNAPPY_K1R64_HALF32: K1r64's asm statement holds a second round loop with the
// 32 KiB candidate step, entered while no segment past the first 128 is loaded
// (seghi == 0: registers 0..127 hold segments 0..127, nothing is far or wrapped;
// a pair past register 127 reads v130 only for bytes past the 64 the round
// compares, as in K1r): five scalar instructions and two branches fewer per hit
// round over the first half of each block.  A/B on 1 GiB of 64 KiB blocks,
// outputs identical, 68 GPU tests green: K1r64 13.78-13.82 -> 13.52-13.56 ms per
// GiB with both loops' placements swept (PAD64 0, PAD64A 0; profiles/r06aa_*,
// r06ad_*); random and repeat equal
#if SNAPPY_K1R64_HALF32
#define K1R64_HALF_SEL "s_cmp_eq_u32 %[seghi], 0\n\ts_cbranch_scc1 L%=_topa\n"
// (the first loop's miss path falls through to the code-3 exit: branch there)
#define K1R64_HALF_LOOP "s_branch L%=_x3\n" K1R_LOOP_PLACE(SNAPPY_K1R_PAD64A) K1R_ROUND_BODY(K1R_CAND32, K1R_HIT64, "a")
#else
#define K1R64_HALF_SEL ""
#define K1R64_HALF_LOOP ""
#endif
#define K1R_ASM_ROUNDS_STMT(code, fx, cx, e32, et32, CAND, SEGHI, HIT, PAD, DUAL_SEL, DUAL_LOOP)    \
    do {                                                                                            \
        uint32_t _m0s, _pf, _s0, _s1, _s2, _s3, _t0, _t1, _t2, _t3, _t4;                            \
        K1R_DLEN_DECL                                                                               \
        uint64_t _valid, _hm;                                                                       \
        asm volatile(                                                                               \
            "s_mov_b32 %[m0s], m0\n\t"                                                              \
            "s_cmp_gt_u32 %[skip], %[skipmax]\n\t" /* a step of 2 within DMAX probes: C++ round */   \
            "s_cbranch_scc1 L%=_x3\n"                                                               \
            DUAL_SEL                                                                                \
            K1R_LOOP_PLACE(PAD)                                                                     \
            K1R_ROUND_BODY(CAND, HIT, "")                                                           \
            DUAL_LOOP                                                                               \
            "L%=_x3:\n\ts_mov_b32 %[code], 3\n\ts_branch L%=_end\n"                                 \
            "L%=_x1:\n\ts_mov_b32 %[code], 1\n\ts_branch L%=_end\n"                                 \
            "L%=_x2:\n\ts_mov_b32 %[code], 2\n\ts_branch L%=_end\n"                                 \
            "L%=_x4:\n\t" K1R_X4                                                                   \
            "L%=_far:\n\t" /* K1r64: the candidate's 256 bytes from the input */                    \
            "s_and_b32 %[s1], %[c], -4\n\t"                                                         \
            "v_add_u32_e32 %[t1], %[s1], %[lane4]\n\t"                                              \
            "global_load_dword %[t3], %[t1], %[srcb]\n\t"                                           \
            "s_mov_b32 %[s1], 0x10203\n\t"                                                          \
            "s_waitcnt vmcnt(0)\n\t"                                                                \
            "v_perm_b32 %[t3], %[t3], %[t3], %[s1]\n\t" /* big-endian, as the ring registers */    \
            "s_branch L%=_farret\n"                                                                 \
            "L%=_wrap:\n\t" /* K1r64: registers 127 (v129, lanes >= l0) and 0 (v2) */               \
            "s_bfe_u32 %[s1], %[c], 0x60002\n\t"                                                    \
            "v_cmp_le_u32_e32 vcc, %[s1], %[lane]\n\t"                                              \
            "v_add_u32_e32 %[t1], %[c], %[lane4]\n\t"                                               \
            "s_nop 0\n\t"                                                                            \
            "v_cndmask_b32_e32 %[t3], v2, v129, vcc\n\t"                                            \
            "ds_bpermute_b32 %[t3], %[t1], %[t3]\n\t"                                               \
            "s_branch L%=_farret\n"                                                                 \
            "L%=_x5:\n\ts_mov_b32 %[code], 5\n"                                                     \
            "L%=_end:\n\t"                                                                          \
            K1R_SKIPFIX                                                                             \
            "s_mov_b32 m0, %[m0s]\n\t"                                                              \
            "s_waitcnt lgkmcnt(0)"                                                                  \
            : [p] "+s"(p), [skip] "+s"(skip), [lane0] "+s"(lane0), [pend] "+s"(pend), [dka] "+s"(dka), \
              [dkb] "+s"(dkb), [dkn] "+s"(dkn), K1R_DLEN_OP [code] "=&s"(code), [f] "=&s"(fx),         \
              [c] "=&s"(cx),                                                                        \
              [m0s] "=&s"(_m0s), [pf] "=&s"(_pf), [s0] "=&s"(_s0), [s1] "=&s"(_s1), [s2] "=&s"(_s2),   \
              [s3] "=&s"(_s3), [valid] "=&s"(_valid), [hm] "=&s"(_hm), [ent] "+v"(e32),                \
              [entt] "+v"(et32), [tka] "+v"(tka), [tkb] "+v"(tkb), [t0] "=&v"(_t0), [t1] "=&v"(_t1),  \
              [t2] "=&v"(_t2), [t3] "=&v"(_t3), [t4] "=&v"(_t4)                                        \
            : [q0] "s"(q0), [L] "s"(L), [lm16] "s"(L - 16), [mwin] "s"(m_win), [seghi] SEGHI,         \
              [lim0] "s"(__builtin_elementwise_min((int32_t)(62 - SNAPPY_K1R_RMIN), (int32_t)L - 16 - (int32_t)q0)), \
              [dv] "v"(dv),                                                                         \
              [pdl1] "v"(pdl1), [pdc] "v"(pdc), [pdnz] "v"(pdnz), [adr] "v"(adr), [adrt] "v"(adr >> 1), \
              [word] "v"(word), [lane] "v"(lane), [lane4] "v"(lane << 2), [srcb] "s"(src),            \
              [sx] "s"(__builtin_amdgcn_read_exec()), /* exec here (the compiler reads it once) */     \
              [skipmax] "i"(64 - DMAX), [dmask] "i"((1u << DMAX) - 1), [lsmax] "i"(64 - SNAPPY_K1R_LSMIN), \
              [l0max] "i"(62 - SNAPPY_K1R_RMIN), [tagb] "i"(kTagBase), "{v[2:33]}"(g0), "{v[34:65]}"(g1), \
              "{v[66:97]}"(g2), "{v[98:129]}"(g3)                                                      \
            : "vcc", "scc", "memory");                                                              \
    } while (0)
#endif
#if defined(SNAPPY_K1R_LSTAMPS)
    uint64_t seg[6] = {0, 0, 0, 0, 0, 0};
    uint64_t s0, s1, s2, s3, s4, s5, s6;
#endif
    uint32_t p = 1, skip = 33;
    while (!(L - p < (skip >> 5) + 15)) {  // is_block_end :229-232
#ifdef SNAPPY_K1R_STATS
        n_round++;
#endif
        if (skip <= 64 - SNAPPY_K1R_LSMIN) {
            // ---------------- lane-space rounds until a step > 1 or the block end.
            // The common round (a hit, verified, no refresh) is one straight-line
            // path: the rare cases branch out of it (__builtin_expect).
            auto refresh = [&]() {
                LSTAMP(s5);
#ifdef SNAPPY_K1R_STATS
                n_refresh++;
#endif
#ifdef SNAPPY_K1R_RSTAMPS
                uint64_t r0, r1, r2;
                const bool rfl = pend + dkn > 48;
                if constexpr (BIG) {  // (the product's order: the move first, see below)
                    RSTAMP(r0);
                    WINDOW_LS(p - 1);
                    RSTAMP(r1);
                    if (rfl) flush_tokens();
                    RSTAMP(r2);
                    rs_win += r1 - r0;
                    rs_flush += r2 - r1;
                } else {
                    RSTAMP(r0);
                    if (rfl) flush_tokens();
                    RSTAMP(r1);
                    WINDOW_LS(p - 1);
                    RSTAMP(r2);
                    rs_flush += r1 - r0;
                    rs_win += r2 - r1;
                }
                rs_n++;
                rs_nfl += rfl;
                if (false)
#endif
                // the deferred token stays pending (drained by the next round): count it.
                // BIG: the window move waits vmcnt(0) for its staged LDS-DMA, and vmcnt
                // counts stores too (in issue order): flush after the move, so that
                // wait never covers this refresh's token stores
                if constexpr (BIG) {
                    const bool fl = pend + dkn > 48;
                    WINDOW_LS(p - 1);
                    if (fl) flush_tokens();
                } else
                {
                    if (pend + dkn > 48) flush_tokens();
                    WINDOW_LS(p - 1);
                }
                LSTAMP(s6);
                LSEG(5, s5, s6);
            };
            uint32_t lane0 = p - q0;
            bool went = false;
            if (!lsw || lane0 + SNAPPY_K1R_RMIN > 62) {
                refresh();
                lane0 = 1;
                went = true;
            }
            // the round's table entries: read right after the round's inserts, so the
            // read is in flight during the verification (each path that writes the table
            // again, and a refresh, reads again); the entry registers have the loads' own
            // u16 / u8 types, or the compiler zero-extends -- and waits for -- each load
            // where it is issued (round 3: that wait made this order 8 % slower; now
            // text32k 16.19 -> 16.18 ms, 64 KiB blocks 19.37 -> 19.20, profiles/r03s2b_*,
            // against reading at the round's end)
            if (!went) TBL_READ_ENT(adr);
            for (;;) {
#if K1R_ASM_ROUNDS
                {
                    // the common rounds as one hand-scheduled loop (k1r_asm_rounds below)
                    uint32_t code, fx, cx;
                    uint32_t e32 = ent, et32 = ent_t;
#ifdef SNAPPY_K1R_RSTAMPS
                    uint64_t ra0, ra1;
                    RSTAMP(ra0);
#endif
                    if constexpr (BIG)
                        K1R_ASM_ROUNDS_STMT(code, fx, cx, e32, et32, K1R_CAND64, K1R_SEGHI64(seg_hi), K1R_HIT64, SNAPPY_K1R_PAD64,
                                            K1R64_HALF_SEL, K1R64_HALF_LOOP);
                    else
                        K1R_ASM_ROUNDS_STMT(code, fx, cx, e32, et32, K1R_CAND32, "i"(0), K1R_HIT32, SNAPPY_K1R_PAD32, "", "");
#ifdef SNAPPY_K1R_RSTAMPS
                    RSTAMP(ra1);
                    rs_asm += ra1 - ra0;
                    rs_nasm++;
                    rs_code[code < 6 ? code : 0]++;
#endif
                    ent = (uint16_t)e32;
                    ent_t = (uint8_t)et32;
                    if (code == 1) break;  // skip past the step-1 range, or is_block_end
                    if (code == 2) {       // the window needs to move
                        refresh();
                        lane0 = 1;
                        continue;
                    }
                    if (code >= 4) {  // the round stopped after its inserts: finish it here
                        const uint32_t f = fx, pf = q0 + fx, c = cx;
                        uint32_t np;
                        if (code == 4) {  // 64 or more equal bytes: extend the match
                            uint32_t len = __builtin_elementwise_min(match_len_from(pf, c, 64), L - pf);
                            dka = pf | (len << 16);
                            dkb = pf - c;
                            dkn = 1;
                            np = pf + len;
                            skip = 32;
                        } else {  // tag collision: a miss (as in the C++ round below)
                            dkn = 0;
                            if (f == lane0) {
                                TBL_INSERT(lane - (lane0 - 1) <= 1);
                                LDS_ORDER();
                                TBL_READ_ENT(adr);
                            }
                            np = pf + ((skip + f - lane0) >> 5);
                            skip += f - lane0 + 1;
                        }
                        p = np;
                        if (!(skip <= 64 - SNAPPY_K1R_LSMIN && p <= L - 16)) break;
                        lane0 = p - q0;
                        if (lane0 + SNAPPY_K1R_RMIN > 62) {
                            refresh();
                            lane0 = 1;
                        }
                        continue;
                    }
                    // code 3: a round whose probes reach a step of 2 (skip > 64 - DMAX) runs below
                }
#endif
                LSTAMP(s0);
                drain_token();  // the previous round's match: one writelane pair per round
                // probe k = lane - lane0 for k <= kcap: step 1 before it ((skip + k - 1) >> 5 == 1),
                // predecessors within DMAX; inside the window and before is_block_end (m_win);
                // the probe at skip + k == 64 (only when 64 - skip < DMAX) needs L - p_k >= 17
                // (one-sided branch: the common case costs a compare and a branch)
                uint64_t valid = (((1ull << DMAX) - 1) << lane0) & m_win;
                if (__builtin_expect(skip > 64 - DMAX, 0)) {
                    const uint32_t kcap = 64 - skip;
                    valid = ((2ull << kcap) - 1) << lane0;
                    if (lane0 + kcap < 64) valid &= ~((1ull << (lane0 + kcap)) & ~m_win17);
                    valid &= m_win;
                }
                // lane l > lane0 takes the in-round candidate when its nearest same-hash lane is >= lane0 - 1;
                // the hit test selects per lane (VALU) so one ballot carries it to SALU
                const bool inr = (int32_t)pdl1 >= (int32_t)lane0;
                const uint32_t hitnz = (inr ? pdnz : (uint32_t)ent_t) ^ ((word >> 16) & 0xFFu);
                const uint64_t hm = __ballot(hitnz == 0) & valid;
                const uint32_t candv = inr ? pdc : ent;
                const uint32_t f = (uint32_t)__builtin_ctzll(hm);
                LSTAMP(s1);
                LSEG(0, s0, s1);
                uint32_t np;
                if (__builtin_expect(hm != 0, 1)) {
                    const uint32_t pf = q0 + f;
                    const uint32_t c = __builtin_amdgcn_readlane(candv, f) & 0xFFFF;
                    // find_copy_length :61-72 after found_match :259-265: lanes 0..15
                    // compare the 64 bytes at pf (dwords from dv) and c (registers)
                    const uint32_t pa = (uint32_t)__builtin_amdgcn_ds_bpermute(
                        (int)(((pf >> 2) + lane) << 2), (int)dv);
                    const uint32_t ca = CAND_LANES(c >> 2);
                    __builtin_amdgcn_sched_barrier(0);
                    // the inserts known before the verdict: misses p_k - 1, p_k and the
                    // probe at f (miss or match) -- all of [lane0 - 1, f] unless f is the
                    // first probe (its p - 1 is inserted only if it misses); other lanes
                    // write the dummy record
                    const uint32_t lo0 = f > lane0 ? lane0 - 1 : lane0;
                    TBL_INSERT(lane - lo0 <= f - lo0);
                    LDS_ORDER();
                    TBL_READ_ENT(adr);  // the next round's entries, in flight during the verification
                    LSTAMP(s2);
                    LSEG(1, s1, s2);
                    const uint32_t pv = funnel_bytes(pa, wave_shl1(pa), perm_sel(pf & 3));
                    const uint32_t cv = funnel_bytes(ca, wave_shl1(ca), perm_sel(c & 3));
                    const uint32_t y = pv ^ cv;
                    const uint64_t bad = __ballot(y != 0) & 0xFFFFull;
                    // per lane: the prefix length if its dword holds the first mismatch
                    const uint32_t lenv = 4 * lane + ((uint32_t)__builtin_clz(y | 1) >> 3);
                    // read before the test: with bad == 0 the lane index is garbage and len is replaced
                    uint32_t len = __builtin_amdgcn_readlane(lenv, (uint32_t)__builtin_ctzll(bad) & 63);
                    if (__builtin_expect(bad == 0, 0)) len = match_len_from(pf, c, 64);
                    LSTAMP(s3);
                    LSEG(2, s2, s3);
#ifdef SNAPPY_K1R_STATS
                    n_probe += f - lane0 + 1;
#endif
                    // every path defines the deferred token (dkn says whether it counts):
                    // no loop-carried "keep" value, so no register copies at the latch
                    len = __builtin_elementwise_min(len, L - pf);  // the compare never runs past the block
                    dka = pf | (len << 16);
                    dkb = pf - c;
                    if (__builtin_expect(len >= 4, 1)) {
#ifdef SNAPPY_K1R_STATS
                        n_match++;
#endif
                        dkn = 1;
                        np = pf + len;
                        skip = 32;
                    } else {  // tag collision: a miss (append_literal :283-287 steps by skip >> 5)
                        dkn = 0;
                        if (f == lane0) {  // its p - 1, then p again (the later write wins)
                            TBL_INSERT(lane - (lane0 - 1) <= 1);
                            LDS_ORDER();
                            TBL_READ_ENT(adr);
                        }
                        np = pf + ((skip + f - lane0) >> 5);
                        skip += f - lane0 + 1;
                    }
                } else {
                    LSTAMP(s3);
                    dka = dkb = dkn = 0;
                    const uint32_t nk = (uint32_t)__builtin_popcountll(valid);  // lanes lane0 .. lane0 + nk - 1
                    // update_hash_table :303-307: p_k - 1 and p_k of every miss, lane order
                    TBL_INSERT(lane - (lane0 - 1) <= nk);
                    LDS_ORDER();
                    TBL_READ_ENT(adr);
                    np = q0 + lane0 + nk - 1 + ((skip + nk - 1) >> 5);  // the last probe steps by 2 at skip 64
                    skip += nk;
#ifdef SNAPPY_K1R_STATS
                    n_probe += nk;
#endif
                }
                p = np;
                LSTAMP(s4);
                LSEG(3, s3, s4);
                LSEG(4, s0, s4);
#ifdef SNAPPY_K1R_STATS
                n_round++;
#endif
                // is_block_end at skip < 64; steps > 1 continue in W-probe rounds
                if (__builtin_expect(!(skip <= 64 - SNAPPY_K1R_LSMIN && p <= L - 16), 0)) break;
                lane0 = p - q0;
                if (__builtin_expect(lane0 + SNAPPY_K1R_RMIN > 62, 0)) {
                    refresh();
                    lane0 = 1;
                }
            }
            drain_token();
#ifdef SNAPPY_K1R_STATS
            n_round--;
#endif
            continue;
        }
        // ---------------- W-probe round (steps > 1)
#ifdef SNAPPY_K1R_STATS
        if constexpr (!BIG) n_farc++;  // (32 KiB units have no far gathers: the slot counts W-probe rounds)
#endif
        lsw = false;
        if (p - 1 < q0 || p + 12 > q0 + 64) WINDOW_AT(p - 1);
        // lane k = k-th probe if all earlier miss, at its closed-form position
        const uint32_t sk = skip + lane;
        const uint32_t pk = p + skipsum(sk) - skipsum(skip);
        const uint32_t bend = (sk >> 5) + 15;
        // invalid: lane >= W, block end (is_block_end), or past the window
        const uint32_t inval = (uint32_t)(((int32_t)(W - 1 - lane)) >> 31) |
                               (uint32_t)(((int32_t)(L - pk) - (int32_t)bend) >> 31) |
                               (uint32_t)(((int32_t)(q0 + 64) - (int32_t)(pk + 12)) >> 31);
        const uint32_t ik = inval ? 1 : pk - q0;
        const uint32_t hvp = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(ik << 2), (int)hv);
        const uint32_t hvq = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((ik - 1) << 2), (int)hv);
        const uint32_t h = hvp & 0xFFFF, a = hvq & 0xFFFF;
        const uint32_t e = TBL_READ(h);
        // previous lane stepped by 1 iff its skip counter was 32..63
        const uint32_t notdup = ~eqm(((sk - 1) >> 5) ^ 1);
        const uint32_t conflict = tconf<W>(h, a, notdup) & ~eqm(lane);
        const uint32_t hit = TAG_EQ(e, hvp) ? 0xFFFFFFFFu : 0u;
        const uint64_t stop = __ballot((inval | conflict | hit) != 0);
        const uint32_t f = (uint32_t)__builtin_ctzll(stop);
        // lanes before f are exact misses: update_hash_table :303-307
        if (lane < f) {
            TBL_WRITE(a, (pk - 1) | (hvq & 0xFFFF0000u));
            TBL_WRITE(h, pk | (hvp & 0xFFFF0000u));
        }
        LDS_ORDER();
        const uint64_t hits = __ballot((hit & ~(inval | conflict)) != 0);
#ifdef SNAPPY_K1R_STATS
        n_probe += f + ((hits >> f) & 1);
#endif
        uint32_t next_f = f;  // probes consumed if no match
        if ((hits >> f) & 1) {
            const uint32_t pf = __builtin_amdgcn_readlane(pk, f);
            const uint32_t cand = __builtin_amdgcn_readlane(e, f) & 0xFFFF;
            const uint32_t hf = __builtin_amdgcn_readlane(hvp, f);
            uint32_t len = match_len(pf, cand);
            if (len >= 4) {  // verified: found_match :259-265
                if (len > L - pf) len = L - pf;
#ifdef SNAPPY_K1R_STATS
                n_match++;
#endif
                if (pend == 64) flush_tokens();
                put_token(pf, len, pf - cand);
                TBL_WRITE(hf & 0xFFFF, pf | (hf & 0xFFFF0000u));  // emit_copy :328
                LDS_ORDER();
                skip = 32;
                p = pf + len;
                continue;
            }
            // tag collision: lane f is a miss as well
            const uint32_t af = __builtin_amdgcn_readlane(hvq, f);
            TBL_WRITE(af & 0xFFFF, (pf - 1) | (af & 0xFFFF0000u));
            TBL_WRITE(hf & 0xFFFF, pf | (hf & 0xFFFF0000u));
            LDS_ORDER();
            next_f = f + 1;
        }
        // f (or f + 1) misses consumed; f stops at a conflict, the window
        // edge or the block end and is retried exactly as the next lane 0
        p = skip + next_f <= 64 ? p + next_f : p + skipsum(skip + next_f) - skipsum(skip);
        skip += next_f;
    }
#undef WINDOW_AT
#undef WINDOW_LS
#undef TAG_OF
#undef TBL_READ
#undef TBL_WRITE
#undef TBL_READ3
#undef TBL_WRITE3
#undef TBL_ADR
#undef TBL_READ_ENT
#undef TBL_INSERT
#undef TAG_EQ
#undef LDS_ORDER
#undef CAND_LANES
#undef K1R_COUNT
    // BIG: the last stage() may still be writing ring_stage; drain it before the
    // workgroup's LDS can be released (tools/check_asm_waits.py checks every path)
    if constexpr (BIG) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    flush_tokens();
    // the tail literal is pseudo-token nt (src/snappy_compression.c:292-297)
    if (lane == 0) {
        if ((nt & (kK2Seg - 1)) == 0) *reinterpret_cast<uint2 *>(segu + 2 * (nt / kK2Seg)) = make_uint2(acc, cend);
        ntok_out[u] = nt;
        sizes[u] = acc + (L > cend ? literal_bytes(L - cend) : 0u);
    }
#ifdef SNAPPY_K1R_RSTAMPS
    if (lane == 0) {
        uint64_t *st = reinterpret_cast<uint64_t *>(tokens + (uint64_t)gridDim.x * tok_cap) + 4 * (uint64_t)u;
        st[0] = clock64() - t_loop;
        st[1] = rs_flush | (rs_asm << 24);  // (a unit's flush cycles < 2^24)
        st[2] = rs_win | ((uint64_t)rs_nasm << 40);
        st[3] = rs_n | ((uint64_t)rs_nfl << 16) | ((uint64_t)rs_code[3] << 32) | ((uint64_t)(rs_code[4] + rs_code[5]) << 48);
    }
#endif
#ifdef SNAPPY_K1R_STATS
    if (lane == 0) {
        uint64_t *st = reinterpret_cast<uint64_t *>(tokens + (uint64_t)gridDim.x * tok_cap) + 4 * (uint64_t)u;
        st[0] = clock64() - t_loop;
#if defined(SNAPPY_K1R_LSTAMPS)
        st[1] = seg[0] | (seg[1] << 32);
        st[3] = seg[2] | (seg[3] << 32);
        st[2] = seg[4] | (seg[5] << 32);
#else
        st[1] = n_farc | ((uint64_t)n_reload << 32);
        st[2] = n_probe | ((uint64_t)n_round << 32);
        st[3] = n_match | ((uint64_t)n_refresh << 32);
#endif
    }
#endif
}

#if SNAPPY_TU_COMPRESS
__global__ __launch_bounds__(64, 3) void k1r_match_units(const uint8_t *__restrict__ in, uint64_t n, uint32_t unit,
                                                          uint32_t hdr_mode, uint64_t header_value,
                                                          uint2 *__restrict__ tokens, uint32_t tok_cap,
                                                          uint32_t *__restrict__ ntok_out,
                                                          uint32_t *__restrict__ sizes,
                                                          uint32_t *__restrict__ seg_off, uint32_t segs)
{
    k1r_body<false>(in, n, unit, hdr_mode, header_value, tokens, tok_cap, ntok_out, sizes, seg_off, segs);
}
#endif

// 65,536-byte blocks (the reference's MAX_BLOCK_SIZE): a 32 KiB register
// ring over the block, three waves per SIMD
#if SNAPPY_TU_COMPRESS
__global__ __launch_bounds__(64, 3) void k1r_match_units64(const uint8_t *__restrict__ in, uint64_t n, uint32_t unit,
                                                            uint32_t hdr_mode, uint64_t header_value,
                                                            uint2 *__restrict__ tokens, uint32_t tok_cap,
                                                            uint32_t *__restrict__ ntok_out,
                                                            uint32_t *__restrict__ sizes,
                                                            uint32_t *__restrict__ seg_off, uint32_t segs)
{
    k1r_body<true>(in, n, unit, hdr_mode, header_value, tokens, tok_cap, ntok_out, sizes, seg_off, segs);
}
#endif

// ---------------------------------------------------------------------------
// K2: token list -> Snappy bytes at the unit's final offset (after K3's scan),
// one wave per unit, one token per lane: literal header + literal bytes (read
// from the input) + copy pieces, exactly as write_literal / write_copy lay
// them out (src/snappy_compression.c:95-165).  The last pseudo-token carries
// the tail literal.
// ---------------------------------------------------------------------------
// exclusive add-scan over lanes 0..31 only (lanes 32..63 undefined), total of lanes 0..31
__device__ __forceinline__ uint32_t wave_excl_scan32(uint32_t v, uint32_t *total)
{
    uint32_t x = v;
    x += dpp0<0x111, 0xF>(x);
    x += dpp0<0x112, 0xF>(x);
    x += dpp0<0x114, 0xF>(x);
    x += dpp0<0x118, 0xF>(x);
    x += dpp0<0x142, 0xA>(x);
    *total = (uint32_t)__builtin_amdgcn_readlane((int)x, 31);
    return x - v;
}

template <typename P>
__device__ __forceinline__ void put_copy(P *o, uint32_t len, uint32_t off)
{
    while (len > 68) {
        o[0] = 0xFE; o[1] = (uint8_t)off; o[2] = (uint8_t)(off >> 8);
        o += 3; len -= 64;
    }
    if (len > 64) {
        o[0] = 0xEE; o[1] = (uint8_t)off; o[2] = (uint8_t)(off >> 8);
        o += 3; len -= 60;
    }
    if (len < 12 && off < 2048) {
        o[0] = (uint8_t)((((off >> 8) << 5) + ((len - 4) << 2) + 1));
        o[1] = (uint8_t)off;
    } else {
        o[0] = (uint8_t)(((len - 1) << 2) | 2); o[1] = (uint8_t)off; o[2] = (uint8_t)(off >> 8);
    }
}

// the element bytes of one token (literal header + payload + copy pieces) at w;
// literal bytes come from src + s0 (global); litn <= 16 by five independent dword
// loads realigned with v_alignbyte, longer literals are left to the caller
template <typename P>
__device__ __forceinline__ void put_element(P *w, const uint8_t *__restrict__ src, uint32_t s0, uint32_t litn,
                                            uint32_t hl, uint32_t len, uint32_t off, bool wide_ok)
{
    if (hl == 1) w[0] = (uint8_t)((litn - 1) << 2);
    else if (hl == 2) { w[0] = 60 << 2; w[1] = (uint8_t)(litn - 1); }
    else if (hl == 3) { w[0] = 61 << 2; w[1] = (uint8_t)(litn - 1); w[2] = (uint8_t)((litn - 1) >> 8); }
    if (litn <= 16) {
        if (wide_ok) {
            const uintptr_t sa = reinterpret_cast<uintptr_t>(src + s0);
            const uint32_t sh = (uint32_t)(sa & 3);
            const uint32_t *aw = reinterpret_cast<const uint32_t *>(sa - sh);
            const uint32_t d0 = aw[0], d1 = aw[1], d2 = aw[2], d3 = aw[3], d4 = aw[4];
            const uint32_t r[4] = {__builtin_amdgcn_alignbyte(d1, d0, sh), __builtin_amdgcn_alignbyte(d2, d1, sh),
                                   __builtin_amdgcn_alignbyte(d3, d2, sh), __builtin_amdgcn_alignbyte(d4, d3, sh)};
#pragma unroll
            for (uint32_t j = 0; j < 16; j++)
                if (j < litn) w[hl + j] = (uint8_t)(r[j >> 2] >> (8 * (j & 3)));
        } else {
            for (uint32_t j = 0; j < litn; j++) w[hl + j] = src[s0 + j];
        }
    }
    if (len) put_copy(w + hl + litn, len, off);
}

// K2: tokens -> bytes at the unit's final offset (write_literal :95-120,
// write_copy :153-165).  gridDim.y waves per unit, wave y taking segments y,
// y + gridDim.y, ... of kK2Seg tokens (K1r recorded each segment's output
// offset and input position, so segments are independent), each segment in
// passes of kK2Pass tokens (kK2Per consecutive per lane) with two memory round
// trips (the token words, then every short literal's source dwords).  The
// pass is assembled in LDS (byte writes are cheap there) and leaves as aligned
// dword stores; larger passes (long copies / literals) write HBM directly.
// 4 KiB holds a text segment (~2 KiB of output) and keeps K2 at 32 waves per CU
#ifndef SNAPPY_K2_STAGE
#define SNAPPY_K2_STAGE 4096
#endif
constexpr uint32_t kK2Stage = SNAPPY_K2_STAGE;

// put_element into the LDS stage without exec-mask branches: every store is
// issued by every lane, lanes without a byte to store hit their own dummy
// slot (stage + kK2Stage + 4 lane); full literal dwords as unaligned ds_write_b32
// lw: the five source dwords of a short literal, loaded by the caller (all the
// wave's literal loads in one round trip), sh = its source address & 3
__device__ __forceinline__ void put_element_lds(__attribute__((address_space(3))) uint8_t *stage, uint32_t at,
                                                const uint8_t *__restrict__ src, uint32_t s0, uint32_t litn,
                                                uint32_t hl, uint32_t len, uint32_t off, bool wide_ok, bool live,
                                                uint32_t lane, const uint32_t *lw, uint32_t sh)
{
    const uint32_t dum = kK2Stage + 4 + 4 * lane;  // past the stage and its 3 alignment bytes
#define K2_ST8(cond, adr, v) stage[(cond) ? (adr) : dum] = (uint8_t)(v)
    // literal header (write_literal :95-120)
    const uint32_t lm1 = litn - 1;
    K2_ST8(live && hl >= 1, at, hl == 1 ? lm1 << 2 : (hl == 2 ? 60u << 2 : 61u << 2));
    K2_ST8(live && hl >= 2, at + 1, lm1);
    K2_ST8(live && hl == 3, at + 2, lm1 >> 8);
    const uint32_t lp = at + hl;
    if (litn <= 16) {
        if (wide_ok) {
            const uint32_t r0 = __builtin_amdgcn_alignbyte(lw[1], lw[0], sh), r1 = __builtin_amdgcn_alignbyte(lw[2], lw[1], sh);
            const uint32_t r2 = __builtin_amdgcn_alignbyte(lw[3], lw[2], sh), r3 = __builtin_amdgcn_alignbyte(lw[4], lw[3], sh);
#define K2_ST32(k, r) *(__attribute__((address_space(3))) u32u *)(stage + (live && 4 * (k) + 4 <= litn ? lp + 4 * (k) : dum)) = (r)
            K2_ST32(0, r0); K2_ST32(1, r1); K2_ST32(2, r2); K2_ST32(3, r3);
#undef K2_ST32
            const uint32_t fb = litn & ~3u, rem = litn & 3u;
            const uint32_t rt = fb == 0 ? r0 : (fb == 4 ? r1 : (fb == 8 ? r2 : r3));
            K2_ST8(live && rem > 0, lp + fb, rt);
            K2_ST8(live && rem > 1, lp + fb + 1, rt >> 8);
            K2_ST8(live && rem > 2, lp + fb + 2, rt >> 16);
        } else if (live) {
            for (uint32_t j = 0; j < litn; j++) stage[lp + j] = src[s0 + j];
        }
    }
    // copy (write_copy :153-165): one piece when len <= 64, the split otherwise
    const uint32_t cp = lp + litn;
    if (len <= 64) {
        const bool c1 = len < 12 && off < 2048;
        const bool has = live && len != 0;
        K2_ST8(has, cp, c1 ? (((off >> 8) << 5) + ((len - 4) << 2) + 1) : (((len - 1) << 2) | 2));
        K2_ST8(has, cp + 1, off);
        K2_ST8(has && !c1, cp + 2, off >> 8);
    } else if (live) {
        put_copy(stage + cp, len, off);
    }
#undef K2_ST8
}

// the whole wave copies literal k (long: > 16 bytes) of every lane/slot in
// longs into the LDS stage; 8 byte loads per lane in flight per round trip
__device__ __forceinline__ void k2_long_literals(__attribute__((address_space(3))) uint8_t *w,
                                                 const uint8_t *__restrict__ src, uint64_t longs, uint32_t litn,
                                                 uint32_t s0v, uint32_t d0v, uint32_t lane)
{
    while (longs) {
        const uint32_t k = (uint32_t)__builtin_ctzll(longs);
        longs &= longs - 1;
        const uint32_t ln = __builtin_amdgcn_readlane(litn, k);
        const uint32_t s0 = __builtin_amdgcn_readlane(s0v, k);
        const uint32_t d0 = __builtin_amdgcn_readlane(d0v, k);
        for (uint32_t j0 = 0; j0 < ln; j0 += 512) {
            uint8_t v[8];
#pragma unroll
            for (uint32_t q = 0; q < 8; q++) {
                const uint32_t j = j0 + 64 * q + lane;
                v[q] = j < ln ? src[s0 + j] : 0;
            }
#pragma unroll
            for (uint32_t q = 0; q < 8; q++) {
                const uint32_t j = j0 + 64 * q + lane;
                if (j < ln) w[d0 + j] = v[q];
            }
        }
    }
}

// the same straight to HBM: byte head up to an aligned destination dword, then
// aligned dword stores of source dwords realigned by v_alignbyte (8 loads per
// lane in flight, 1 KiB per round trip), byte tail; end = in + n bounds reads
__device__ __forceinline__ void k2_long_literals(uint8_t *w, const uint8_t *__restrict__ src,
                                                 const uint8_t *__restrict__ end, uint64_t longs, uint32_t litn,
                                                 uint32_t s0v, uint32_t d0v, uint32_t lane)
{
    while (longs) {
        const uint32_t k = (uint32_t)__builtin_ctzll(longs);
        longs &= longs - 1;
        const uint32_t ln = __builtin_amdgcn_readlane(litn, k);
        const uint8_t *s = src + __builtin_amdgcn_readlane(s0v, k);
        uint8_t *d = w + __builtin_amdgcn_readlane(d0v, k);
        uint32_t head = (uint32_t)((4 - (reinterpret_cast<uintptr_t>(d) & 3)) & 3);
        if (head > ln) head = ln;
        if (lane < head) d[lane] = s[lane];
        const uint32_t nw = (ln - head) >> 2;
        const uint8_t *sb = s + head;
        const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(sb) & 3);
        const uint32_t *sa = reinterpret_cast<const uint32_t *>(sb - sh);
        uint32_t *dw = reinterpret_cast<uint32_t *>(d + head);
        for (uint32_t k0 = 0; k0 < nw; k0 += 256) {
            uint32_t lo[4], hi[4];
#pragma unroll
            for (uint32_t q = 0; q < 4; q++) {
                const uint32_t kk = k0 + 64 * q + lane;
                lo[q] = hi[q] = 0;
                if (kk < nw) {
                    lo[q] = sa[kk];
                    if (sh) {
                        const uint8_t *pb = reinterpret_cast<const uint8_t *>(sa + kk + 1);
                        if (pb + 4 <= end) hi[q] = sa[kk + 1];
                        else for (uint32_t t = 0; t < sh; t++) hi[q] |= (uint32_t)pb[t] << (8 * t);
                    }
                }
            }
#pragma unroll
            for (uint32_t q = 0; q < 4; q++) {
                const uint32_t kk = k0 + 64 * q + lane;
                if (kk < nw) dw[kk] = __builtin_amdgcn_alignbyte(hi[q], lo[q], sh);
            }
        }
        const uint32_t t0 = head + 4 * nw;
        if (lane < ln - t0) d[t0 + lane] = s[t0 + lane];
    }
}

// SNAPPY_K2_PREFETCH: token words one pass ahead (see the pass loop)
// (A/B on 1 GiB, outputs identical, profiles/r05u_ab_k2_prefetch_*: K3 + K2 per
// GiB 0.932-0.936 -> 0.910-0.911 ms on 32 KiB streams, 0.900-0.902 -> 0.861-0.864
// on 64 KiB blocks with the register cap below; uncapped it needs 82 VGPRs, 5
// waves per SIMD, and is slower: 0.984-0.985)
#ifndef SNAPPY_K2_PREFETCH
#define SNAPPY_K2_PREFETCH 1
#endif
// measurement only (wrong output): K2 reads no literal bytes from the input, the
// upper bound of what literals staged by K1r could save K2
#ifndef SNAPPY_K2_NOLIT
#define SNAPPY_K2_NOLIT 0
#endif
// 1: no register cap (80 VGPRs, 6 waves/SIMD with 128-token passes); capping at
// 7 or 8 waves spills and measured slower (1.18 / 1.22 against 0.979
// ms of K3 + K2 per GiB of text)
// (with the prefetch: 6, i.e. 80 VGPRs, the same occupancy as before it)
#ifndef SNAPPY_K2_WAVES_PER_EU
#define SNAPPY_K2_WAVES_PER_EU (SNAPPY_K2_PREFETCH ? 6 : 1)
#endif
#if SNAPPY_TU_COMPRESS
__global__ __launch_bounds__(64, SNAPPY_K2_WAVES_PER_EU) void k2_emit_units(const uint8_t *__restrict__ in, uint64_t n, uint32_t unit,
                                                    uint32_t hdr_mode, uint64_t header_value,
                                                    const uint2 *__restrict__ tokens, uint32_t tok_cap,
                                                    const uint32_t *__restrict__ ntok,
                                                    const uint32_t *__restrict__ seg_off, uint32_t segs,
                                                    const uint64_t *__restrict__ offsets, uint8_t *__restrict__ out)
{
    __shared__ __attribute__((aligned(16))) uint8_t stage_[kK2Stage + 4 + 4 * 64 + 16];  // + alignment, per-lane dummies
    auto *const stage = (__attribute__((address_space(3))) uint8_t *)stage_;
    const uint32_t lane = threadIdx.x;
    const uint32_t u = blockIdx.x;
    const uint32_t nt = ntok[u];
    const uint64_t base = (uint64_t)u * unit;
    const uint32_t L = (uint32_t)((n - base) < unit ? (n - base) : unit);
    const uint8_t *src = in + base;
    uint8_t *dst = out + offsets[u];
    // 4-byte tokens (K1r: offset | (length - 4) << 16 | gap << 24, escapes in tok_full)
    const uint32_t *tok = reinterpret_cast<const uint32_t *>(tokens) + (uint64_t)u * tok_cap;
    const uint32_t *tok_full = reinterpret_cast<const uint32_t *>(tokens) + ((uint64_t)gridDim.x + u) * tok_cap;
    if (blockIdx.y == 0) {
        if (hdr_mode == SNAPPY_HDR_EVERY_UNIT) varint_put(L, dst, lane);
        else if (hdr_mode == SNAPPY_HDR_FIRST_UNIT && u == 0) varint_put(header_value, dst, lane);
    }
#if SNAPPY_K2_PREFETCH
    // the next pass's token words (and the next segment's record) are loaded one
    // pass ahead, so their round trip overlaps this pass's literal loads
    uint32_t kwn[kK2Per];
    auto load_kw = [&](uint32_t c, uint32_t *k) {
#pragma unroll
        for (uint32_t i = 0; i < kK2Per; i++) {
            const uint32_t t = c + kK2Per * lane + i;
            k[i] = tok[t < nt ? t : 0u];
        }
    };
    auto load_se = [&](uint32_t sg) {
        return *reinterpret_cast<const uint2 *>(seg_off + 2 * ((uint64_t)u * segs + (sg * kK2Seg <= nt ? sg : 0u)));
    };
    if (blockIdx.y * kK2Seg <= nt) load_kw(blockIdx.y * kK2Seg, kwn);
    uint2 sen = load_se(blockIdx.y);
#endif
    for (uint32_t sg = blockIdx.y; sg * kK2Seg <= nt; sg += gridDim.y) {
    // K1r's table: the segment's output offset and the input position where
    // its first literal starts (the end of the previous segment's last token)
#if SNAPPY_K2_PREFETCH
    const uint2 se = sen;
    sen = load_se(sg + gridDim.y);
#else
    const uint2 se = *reinterpret_cast<const uint2 *>(seg_off + 2 * ((uint64_t)u * segs + sg));
#endif
    uint32_t o = se.x, carry = se.y;
    for (uint32_t c = sg * kK2Seg; c < (sg + 1) * kK2Seg && c <= nt; c += kK2Pass) {

    uint32_t gap[kK2Per], len[kK2Per], off[kK2Per], pe[kK2Per], litn[kK2Per], hl[kK2Per], sz[kK2Per];
    bool live[kK2Per];
    uint32_t lspan = 0;  // input bytes covered by the lane's tokens (literal + copy)
    // the lane's token words in one round trip (a lane past the end re-reads word 0:
    // no branch, so no load waits for the one before it), then the rare escapes
    uint32_t kw[kK2Per];
#if SNAPPY_K2_PREFETCH
#pragma unroll
    for (uint32_t i = 0; i < kK2Per; i++) kw[i] = kwn[i];
    {
        uint32_t cn = c + kK2Pass;
        if (!(cn < (sg + 1) * kK2Seg && cn <= nt)) cn = (sg + gridDim.y) * kK2Seg;
        if (cn <= nt) load_kw(cn, kwn);
    }
#else
#pragma unroll
    for (uint32_t i = 0; i < kK2Per; i++) {
        const uint32_t t = c + kK2Per * lane + i;
        kw[i] = tok[t < nt ? t : 0u];
    }
#endif
#pragma unroll
    for (uint32_t i = 0; i < kK2Per; i++) {
        const uint32_t t = c + kK2Per * lane + i;
        const bool has = t < nt;  // else the pseudo-token (the tail literal) or nothing
        live[i] = t <= nt;
        const uint32_t k = has ? kw[i] : 0xFFFFFFFFu;
        const uint32_t lc = (k >> 16) & 0xFF, gc = k >> 24;
        off[i] = has ? k & 0xFFFF : 0u;
        gap[i] = has ? gc : 0u;
        len[i] = has ? lc + 4 : 0u;
        if (has && (lc == 255 || gc == 255)) {
            const uint32_t f = tok_full[t];
            gap[i] = f & 0xFFFF;
            len[i] = f >> 16;
        }
        lspan += gap[i] + len[i];
    }
    uint32_t span_tot;
    uint32_t cur = carry + wave_excl_scan(lspan, lane, &span_tot);
    uint32_t lsum = 0;
#pragma unroll
    for (uint32_t i = 0; i < kK2Per; i++) {
        const uint32_t t = c + kK2Per * lane + i;
        pe[i] = cur;  // where the token's literal starts
        litn[i] = t < nt ? gap[i] : (t == nt ? L - cur : 0u);
        cur += gap[i] + len[i];
        hl[i] = litn[i] ? (litn[i] <= 60 ? 1 : (litn[i] <= 256 ? 2 : 3)) : 0;
        sz[i] = hl[i] + litn[i] + ((live[i] && len[i]) ? copy_bytes(len[i], off[i]) : 0);
        lsum += sz[i];
    }
    uint32_t total;
    uint32_t rel = wave_excl_scan(lsum, lane, &total);
    const bool staged = total <= kK2Stage;
    // the stage is laid out at the destination's alignment (stage byte sb + x is
    // output byte dst + o + x), so the copy-out below reads aligned LDS dwords
    const uint32_t sb = staged ? (uint32_t)(reinterpret_cast<uintptr_t>(dst + o) & 3) : 0u;
    uint64_t longs[kK2Per];
    uint32_t d0v[kK2Per];
    // every short literal's source dwords in one round trip: lanes with none read
    // the unit's first token words (in bounds, ignored)
    uint32_t lw[kK2Per][5], lsh[kK2Per];
    bool wide[kK2Per];
#pragma unroll
    for (uint32_t i = 0; i < kK2Per; i++) {
        wide[i] = base + pe[i] + 20 <= n;  // the aligned 20-byte read ends inside in[0, n)
        const bool ld = !SNAPPY_K2_NOLIT && staged && wide[i] && live[i] && litn[i] != 0 && litn[i] <= 16;
        const uintptr_t sa = reinterpret_cast<uintptr_t>(src + pe[i]);
        lsh[i] = (uint32_t)(sa & 3);
        const auto *aw = reinterpret_cast<const __attribute__((address_space(1))) uint32_t *>(
            ld ? sa - lsh[i] : reinterpret_cast<uintptr_t>(tok));
#pragma unroll
        for (uint32_t j = 0; j < 5; j++) lw[i][j] = aw[j];
    }
#pragma unroll
    for (uint32_t i = 0; i < kK2Per; i++) {
        const bool wide_ok = wide[i];
        if (staged) put_element_lds(stage, rel + sb, src, pe[i], litn[i], hl[i], len[i], off[i], wide_ok, live[i], lane,
                                    lw[i], lsh[i]);
        else if (live[i]) put_element(dst + o + rel, src, pe[i], litn[i], hl[i], len[i], off[i], wide_ok);
        longs[i] = __ballot(live[i] && litn[i] > 16);
        d0v[i] = rel + sb + hl[i];
        rel += sz[i];
    }
#pragma unroll
    for (uint32_t i = 0; i < kK2Per && !SNAPPY_K2_NOLIT; i++) {
        if (staged) k2_long_literals(stage, src, longs[i], litn[i], pe[i], d0v[i], lane);
        else k2_long_literals(dst + o, src, in + n, longs[i], litn[i], pe[i], d0v[i], lane);
    }
    if (staged) {
        __builtin_amdgcn_wave_barrier();
        // stage[sb, sb + total) -> dst + o: byte head to a dword boundary, aligned
        // dwords (aligned in LDS too: sb + head is a multiple of 4), byte tail
        uint8_t *g = dst + o;
        uint32_t head = (4 - sb) & 3;
        if (head > total) head = total;
        if (lane < head) g[lane] = stage[sb + lane];
        const uint32_t nw = (total - head) >> 2;
        uint32_t *gw = reinterpret_cast<uint32_t *>(g + head);
        const auto *sw = reinterpret_cast<const __attribute__((address_space(3))) uint32_t *>(stage + sb + head);
        for (uint32_t k = lane; k < nw; k += 64) gw[k] = sw[k];
        const uint32_t tail0 = head + 4 * nw;
        if (lane < total - tail0) g[tail0 + lane] = stage[sb + tail0 + lane];
    }
    __builtin_amdgcn_wave_barrier();  // the stage is reused by the next pass
    o += total;
    carry += span_tot;
    }
    }
}
#endif

// ---------------------------------------------------------------------------
// K3a: exclusive scan of unit sizes -> offsets[0..count], total.
// ---------------------------------------------------------------------------
// One workgroup walks the sizes in tiles of 8,192 staged through LDS
// (coalesced loads and stores); each thread scans 8 consecutive sizes, DPP
// scans combine threads within a wave and the 16 wave totals.  A unit is at
// most ~67.6 KB, so a tile's relative prefix fits 32 bits; the carry is 64-bit.
constexpr uint32_t kScanPer = 8;
[[maybe_unused]] constexpr uint32_t kScanTile = 1024 * kScanPer;

#if SNAPPY_TU_COMPRESS
__global__ __launch_bounds__(1024) void k3_scan(const uint32_t *__restrict__ sizes, uint64_t count,
                                                uint64_t *__restrict__ offsets, uint64_t *__restrict__ total)
{
    __shared__ uint32_t tile[kScanTile + kScanTile / 32];  // + one pad dword per 32 (bank spread)
    __shared__ uint32_t wtot[16];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
#define K3_AT(i) ((i) + ((i) >> 5))
    uint64_t carry = 0;
    for (uint64_t b = 0; b < count; b += kScanTile) {
        const uint32_t m = (uint32_t)(count - b < kScanTile ? count - b : kScanTile);
        for (uint32_t i = t; i < kScanTile; i += 1024) tile[K3_AT(i)] = i < m ? sizes[b + i] : 0u;
        __syncthreads();
        uint32_t v[kScanPer], s = 0;
#pragma unroll
        for (uint32_t k = 0; k < kScanPer; k++) {
            v[k] = tile[K3_AT(t * kScanPer + k)];
            s += v[k];
        }
        const uint32_t x = wave_incl_scan(s);
        if (lane == 63) wtot[w] = x;
        __syncthreads();
        if (w == 0) {
            const uint32_t y = lane < 16 ? wtot[lane] : 0u;
            const uint32_t z = wave_incl_scan(y);
            if (lane < 16) wtot[lane] = z - y;  // exclusive over waves
        }
        __syncthreads();
        uint32_t run = wtot[w] + x - s;
#pragma unroll
        for (uint32_t k = 0; k < kScanPer; k++) {
            tile[K3_AT(t * kScanPer + k)] = run;
            run += v[k];
        }
        __syncthreads();
        for (uint32_t i = t; i < m; i += 1024) offsets[b + i] = carry + tile[K3_AT(i)];
        if (t == 1023) wtot[0] = run;  // the tile's total
        __syncthreads();
        carry += wtot[0];
        __syncthreads();
    }
#undef K3_AT
    if (t == 0) {
        offsets[count] = carry;
        *total = carry;
    }
}

// The same scan in one wave (lane l scans sizes 8 l .. 8 l + 7 of each group of
// 512), for launches of few units: a 1,024-thread workgroup needs 16 free wave
// slots on one CU, which it does not get while another stream's match finder
// fills every SIMD (the host-buffer pipeline's chunk lanes: a K3 of 1,024
// blocks waited 1.06 ms for a CU, profiles/r04e_host_trace_*); one wave starts
// on the first free slot.
__global__ __launch_bounds__(64) void k3_scan_wave(const uint32_t *__restrict__ sizes, uint64_t count,
                                                  uint64_t *__restrict__ offsets, uint64_t *__restrict__ total)
{
    const uint32_t lane = threadIdx.x;
    uint64_t carry = 0;
    for (uint64_t b = 0; b < count; b += 64 * kScanPer) {
        uint32_t v[kScanPer], s = 0;
#pragma unroll
        for (uint32_t k = 0; k < kScanPer; k++) {
            const uint64_t i = b + kScanPer * lane + k;
            v[k] = i < count ? sizes[i] : 0u;
            s += v[k];
        }
        uint32_t tot;
        uint32_t run = wave_excl_scan(s, lane, &tot);
#pragma unroll
        for (uint32_t k = 0; k < kScanPer; k++) {
            const uint64_t i = b + kScanPer * lane + k;
            if (i < count) offsets[i] = carry + run;
            run += v[k];
        }
        carry += tot;
    }
    if (lane == 0) {
        offsets[count] = carry;
        *total = carry;
    }
}
#endif

// ---------------------------------------------------------------------------
// K4: one wave per unit.  The compressed unit streams through a 512-byte
// window in LDS (three 256-byte slots used round robin, the next segment
// prefetched into a register a slide ahead), so a lane reads its candidate
// element's bytes, or a literal byte, with one LDS read.  Each batch parses the elements
// starting in the next 64 window bytes lane-parallel (tag dispatch of
// src/snappy_decompression.c:290-333, element chain by pointer doubling),
// then executes them in 64-byte output passes into an LDS ring that is
// flushed to HBM in 1 KiB blocks; copies keep the byte-serial overlap
// semantics of :273-280 (out[op+j] = out[op-off + j mod off]).
//
// Block index entries (include/snappy_amd.h): bits [0,40) = compressed
// offset of the element holding the unit's first output byte, bits [40,64) =
// how many of that element's output bytes precede the unit (0 when the
// element starts the unit, always so for streams this codec writes).  A
// unit whose first element straddles in resumes it; a unit whose last
// element straddles out truncates it (the reference decodes one whole
// output buffer, :345-363, so elements may cross 65,536-byte boundaries and
// copies may reach into earlier blocks, :253-280).
//
// Pass 1 (k4_decompress_units, BACK = false) decodes every unit whose copies
// stay inside it; a unit needing bytes of earlier units stops with status
// DEFER.  Pass 2 (k4_decompress_back, BACK = true) runs only those: units
// take tickets in index order (so every unit a wave waits for is already
// resident or finished), publish their HBM progress with release stores and
// wait with acquire loads until the bytes their copies read are in HBM.
// ---------------------------------------------------------------------------
constexpr uint64_t kIdxOffMask = (1ull << 40) - 1;
constexpr uint32_t kIdxSkipShift = 40;
constexpr int32_t kK4Tail = 3;  // pass 1, in-batch: an element runs past the unit's end
// pass 2 keeps a deferred unit's progress in its status word: DEFER + bytes in
// HBM while it runs, its final status (<= 0) once done

__device__ __forceinline__ uint32_t load_dw_guarded(const uint8_t *comp, uint64_t a, uint64_t lim)
{
    // dword at 4-aligned absolute address a; bytes at or past lim read as 0
    if (a + 4 <= lim) return __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(comp + a));
    uint32_t w = 0;
    for (uint32_t k = 0; k < 4; k++)
        if (a + k < lim) w |= (uint32_t)comp[a + k] << (8 * k);
    return w;
}

// lane l <- dword l of the 256-byte segment at a0 (4-aligned): one uniform test
// instead of a per-lane 64-bit bound check unless the segment reaches lim
__device__ __forceinline__ uint32_t load_seg(const uint8_t *comp, uint64_t a0, uint64_t lim, uint32_t lane)
{
    if (a0 + 256 <= lim) return __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(comp + a0) + lane);
    return load_dw_guarded(comp, a0 + 4 * lane, lim);
}

// ring -> HBM for output bytes [F, T): 16-byte stores on a 16-aligned
// destination, bytes otherwise
__device__ __forceinline__ void k4_flush(const uint8_t *ob, uint32_t M, uint8_t *dst, uint32_t F, uint32_t T,
                                         uint32_t lane)
{
    if (T <= F) return;
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        uint32_t a = (F + 15) & ~15u;
        if (a > T) a = T;
        if (F + lane < a) dst[F + lane] = ob[(F + lane) & M];
        const uint32_t e = T & ~15u;
#pragma unroll 1
        for (uint32_t x = a + 16 * lane; x < e; x += 1024)
            *reinterpret_cast<u32x4 *>(dst + x) = *reinterpret_cast<const u32x4 *>(ob + (x & M));
        const uint32_t t0 = e > a ? e : a;
        if (t0 + lane < T) dst[t0 + lane] = ob[(t0 + lane) & M];
    } else {
#pragma unroll 1
        for (uint32_t x = F + lane; x < T; x += 64) dst[x] = ob[x & M];
    }
}

// literal bytes lsrc[0, kl) straight from HBM to output [kop, kop+kl): HBM to
// HBM in destination-aligned dwords (each funnel-shifted out of two aligned
// source dwords: an aligned dword holding a byte of the literal never crosses
// a page the literal does not touch), and its last min(kl, ring) bytes into the
// ring (later copies read only that far back from the ring; further back, HBM)
#define K4_LIT_ATTR __noinline__
__device__ K4_LIT_ATTR void k4_literal_hbm(const uint8_t *lsrc, uint32_t kl, uint32_t kop, uint8_t *ob, uint32_t M,
                                               uint8_t *dst, uint32_t lane)
{
    uint8_t *const d = dst + kop;
    const uint32_t h0 = (uint32_t)(-(uintptr_t)d & 3);
    const uint32_t h = h0 < kl ? h0 : kl;  // head bytes up to a 4-aligned destination
    if (lane < h) d[lane] = lsrc[lane];
    const uint32_t nd = (kl - h) >> 2;     // body dwords
    const uint8_t *const s = lsrc + h;
    const uint32_t sa = (uint32_t)((uintptr_t)s & 3);
    const uint32_t *const s4 = reinterpret_cast<const uint32_t *>(s - sa);
    uint32_t *const d4 = reinterpret_cast<uint32_t *>(d + h);
#pragma unroll 1
    for (uint32_t i = lane; i < nd; i += 256) {
        uint32_t w[4];
#pragma unroll
        for (int m = 0; m < 4; m++) {
            const uint32_t j = i + 64 * m;
            w[m] = 0;
            if (j < nd) {
                const uint32_t lo = __builtin_nontemporal_load(s4 + j);
                w[m] = sa ? __builtin_amdgcn_alignbit(__builtin_nontemporal_load(s4 + j + 1), lo, 8 * sa) : lo;
            }
        }
#pragma unroll
        for (int m = 0; m < 4; m++)
            if (i + 64 * m < nd) d4[i + 64 * m] = w[m];
    }
    const uint32_t t = h + 4 * nd;  // tail bytes
    if (t + lane < kl) d[t + lane] = lsrc[t + lane];
    // the ring: the literal's last min(kl, M + 1) bytes
    const uint32_t r0 = kl > M + 1 ? kl - (M + 1) : 0;
#pragma unroll 1
    for (uint32_t b = r0; b < kl; b += 256) {
        uint8_t v[4];
#pragma unroll
        for (int m = 0; m < 4; m++) {
            const uint32_t jj = b + 64 * m + lane;
            v[m] = jj < kl ? lsrc[jj] : 0;
        }
#pragma unroll
        for (int m = 0; m < 4; m++) {
            const uint32_t jj = b + 64 * m + lane;
            if (jj < kl) ob[(kop + jj) & M] = v[m];
        }
    }
}

// pass 2: this unit's output [0, F) is in HBM, or (val <= 0) it is done
// (release: the wave's stores first, then the status word)
__device__ __forceinline__ void k4_publish(int32_t *status, uint32_t u, int32_t val, uint32_t lane)
{
    if (lane == 0) __hip_atomic_store(status + u, val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// pass 2: wait until output bytes [g_lo, g_hi] (global positions below this
// unit) are in HBM.  Units [done_lo, u) are known complete.  Every unit waited
// for has a lower ticket than this one, so it is running or done; the time
// limit only guards against a corrupt progress array.
__device__ __noinline__ int32_t k4_wait(const int32_t *status, uint64_t g_lo, uint64_t g_hi, uint32_t unit,
                                        uint32_t lane, uint32_t *done_lo)
{
    const uint32_t vlo = (uint32_t)(g_lo / unit), vhi = (uint32_t)(g_hi / unit);
    for (uint32_t v = vhi + 1; v-- > vlo;) {
        if (v >= *done_lo) continue;
        const int32_t need = v == vhi ? (int32_t)(g_hi - (uint64_t)v * unit) + 1 : (int32_t)unit;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
            int32_t p = 0;
            if (lane == 0) p = __hip_atomic_load(status + v, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            p = __builtin_amdgcn_readfirstlane(p);
            if (p <= 0) {  // done (pass 1 or 2; an error status lets the caller fail on its own)
                if (v + 1 == *done_lo) *done_lo = v;
                break;
            }
            if (p - SNAPPY_ST_DEFER >= need) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > 30ull * 100000000ull) return SNAPPY_ST_TIMEOUT;  // 100 MHz clock
            __builtin_amdgcn_s_sleep(4);
        }
    }
    return SNAPPY_ST_OK;
}

#ifdef SNAPPY_K4_STATS
#if SNAPPY_TU_DECODE
__device__ uint64_t g_k4_stats[32768 * 16];
#else
static __device__ uint64_t g_k4_stats[16];  // (k4_body is parsed, never instantiated, here)
#endif
#define K4STAMP(var)                                                                        \
    do {                                                                                    \
        __builtin_amdgcn_sched_barrier(0);                                                  \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(var)::"memory");        \
        __builtin_amdgcn_sched_barrier(0);                                                  \
    } while (0)
#else
#define K4STAMP(var) do { } while (0)
#endif

// K4's LDS (static, so every base folds into a ds offset field): the
// compressed window at 0 (ds_read2 has only 8-bit dword offsets), the batch's
// element-start bitmap, two scalars, the output ring and one dummy byte
#ifndef SNAPPY_K4_RING
#define SNAPPY_K4_RING 4096
#endif
constexpr uint32_t kK4Ring = SNAPPY_K4_RING;  // output ring; copies reaching further back read HBM
// the ring is flushed to HBM when op - F reaches kK4FlushAt, up to a multiple of
// kK4FlushGran (a batch then starts with op - F < kK4FlushAt)
constexpr uint32_t kK4FlushAt = kK4Ring >= 4096 ? 2048 : 512;
constexpr uint32_t kK4FlushGran = kK4Ring >= 4096 ? 1024 : 512;
constexpr uint32_t kK4MapBits = 1024; // a batch's output span (bit j = an element starts at op + j)
constexpr uint32_t kK4MapAt = 784;    // after the window: 3 x 256 bytes + a 16-byte mirror
constexpr uint32_t kK4TailAt = kK4MapAt + kK4MapBits / 8;
constexpr uint32_t kK4RingAt = kK4TailAt + 16;
#ifndef SNAPPY_K4_LDS_PAD
#define SNAPPY_K4_LDS_PAD 0  // (measurement: pad the LDS to run fewer waves per CU)
#endif
constexpr uint32_t kK4Lds = kK4RingAt + kK4Ring + 4 + SNAPPY_K4_LDS_PAD;  // 5,028 B: 32 waves per CU fit 160 KiB

template <bool BACK>
__device__ __forceinline__ void k4_body(const uint8_t *__restrict__ comp, const uint64_t *__restrict__ offsets,
                                        uint64_t n, uint32_t unit, uint32_t hdr_mode, uint64_t header_value,
                                        uint32_t allow_back, uint32_t bias, uint8_t *__restrict__ out,
                                        int32_t *__restrict__ status, uint32_t u)
{
    // copy source positions: relative to the unit start, negative = an earlier unit (pass 2 only)
    using SrcT = typename std::conditional<BACK, int64_t, uint32_t>::type;
    __shared__ __attribute__((aligned(16))) uint32_t lds[kK4Lds / 4];
    uint8_t *ob = reinterpret_cast<uint8_t *>(lds + kK4RingAt / 4);  // output ring: position x -> ob[x & M]
    constexpr uint32_t ring = kK4Ring, M = ring - 1;
    uint32_t *const map32 = lds + kK4MapAt / 4;      // the batch's element starts, 32 dwords
    const uint32_t lane = threadIdx.x;
    const uint64_t ix0 = offsets[u], ix1 = offsets[u + 1];
    // comp is 4-byte aligned; the stream starts `bias` bytes into it
    const uint64_t c0 = (ix0 & kIdxOffMask) + bias, c1n = (ix1 & kIdxOffMask) + bias;
    const uint32_t skip0 = (uint32_t)(ix0 >> kIdxSkipShift), skip1 = (uint32_t)(ix1 >> kIdxSkipShift);
    const uint64_t base = (uint64_t)u * unit;
    const uint32_t want = (uint32_t)((n - base) < unit ? (n - base) : unit);
    int32_t st = SNAPPY_ST_OK;
    // the unit's compressed bytes: up to the next entry, or (its last element
    // straddling out) as far as the stream goes
    // (the last entry is the stream end: no read goes past it, whatever the
    // entries in between say -- a corrupt index fails as TRUNCATED, not a fault)
    const uint64_t c_end = (offsets[(n + unit - 1) / unit] & kIdxOffMask) + bias;
    uint64_t c1 = skip1 ? c_end : c1n;
    if (c1 > c_end) c1 = c_end;
    if (c1 > c0 + 0x7FFFFFFFull) c1 = c0 + 0x7FFFFFFFull;
    if (c1 < c0 || ((skip0 | skip1) && !allow_back)) st = SNAPPY_ST_TRUNCATED;
    const uint32_t clen = st == SNAPPY_ST_OK ? (uint32_t)(c1 - c0) : 0u;
    uint8_t *dst = out + base;
    uint32_t F = 0;  // output bytes [0, F) are in HBM; [F, op) only in the ring
    uint32_t done_lo = u;  // pass 2: units [done_lo, u) are complete
    // pass 2 checks every element in VALU; pass 1 keeps its loop state small and
    // resolves the rare cases (an element running past the unit, a copy into
    // an earlier unit) in scalar code after the batch ballot
    // the element the next unit resumes (skip1 > 0) starts here: it may run past the unit
    const uint32_t tail_ip = skip1 && c1n >= c0 && c1n - c0 < clen ? (uint32_t)(c1n - c0) : 0xFFFFFFFFu;
    // copies may reach this far before the unit start
    const uint32_t back_lim = (uint32_t)(base < 0xFFFFFFFFull ? base : 0xFFFFFFFFull);
    // pass 1 re-reads the tail element's position from LDS (past the ring) on its rare path
    volatile uint32_t *tail_lds = lds + kK4TailAt / 4;
    if (!BACK && lane == 0) {
        tail_lds[0] = tail_ip;
        tail_lds[1] = want - skip1;
    }

    // LDS window over the compressed unit: 3 slots of 256 bytes (after the ring
    // and the tail scalars) + a 16-byte mirror of slot 0's head, so an 8-byte
    // read crossing from slot 2 into slot 0 stays contiguous.  The window is the
    // 512 bytes from the absolute 4-aligned base B: its first 256 in slot ws, the
    // next in slot (ws + 1) % 3; the segment after that is prefetched into `pre`
    // (a register) and written to the free slot when the window slides.
    auto *const wb = (__attribute__((address_space(3))) uint8_t *)lds;
    auto *const w32 = reinterpret_cast<__attribute__((address_space(3))) uint32_t *>(wb);
    uint64_t B = c0 & ~3ull;
    c1 = c0 + clen;
    // a unit already failed by its index (an entry past the stream end) loads
    // nothing: its window bytes [B, c0) would lie outside the stream (the
    // guarded loads read below c1 = c0; at an entry 1 GiB past the stream end
    // that faulted whenever the address was unmapped)
    if (st != SNAPPY_ST_OK) B = c1 = 0;
    uint32_t ws = 0;
    // window byte x (< 512 + 8) -> LDS byte address in wb
#define WADR(x) ({ const uint32_t _a = 256 * ws + (x); _a >= 768 ? _a - 768 : _a; })
    auto put_seg = [&](uint32_t slot, uint32_t v) {
        w32[64 * slot + lane] = v;
        if (slot == 0 && lane < 4) w32[192 + lane] = v;  // the mirror
    };
    uint32_t pre;
    {
        const uint32_t w0 = load_seg(comp, B, c1, lane);
        const uint32_t w1 = load_seg(comp, B + 256, c1, lane);
        pre = load_seg(comp, B + 512, c1, lane);
        put_seg(0, w0);
        put_seg(1, w1);
        __builtin_amdgcn_wave_barrier();
    }
    // dword k (0..127) of the window at its start (ws = 0), k uniform
#define WDW(k) rfl(w32[k])

    uint32_t ip = 0, op = 0;  // ip relative to c0
    // varint preamble: every STREAMS unit, and block 0 of a SINGLE stream
    if (st == SNAPPY_ST_OK &&
        (hdr_mode == SNAPPY_HDR_EVERY_UNIT || (hdr_mode == SNAPPY_HDR_FIRST_UNIT && u == 0))) {
        const uint64_t expect = hdr_mode == SNAPPY_HDR_EVERY_UNIT ? want : header_value;
        const uint32_t o = (uint32_t)(c0 - B);
        uint64_t v = 0;
        uint32_t k = 0;
        bool done = false;
        for (; k < 10 && k < clen; k++) {
            const uint32_t q = o + k;
            const uint32_t byte = (WDW(q >> 2) >> (8 * (q & 3))) & 0xFF;
            v |= (uint64_t)(byte & 0x7F) << (7 * k);
            if (!(byte & 0x80)) { done = true; k++; break; }
        }
        if (!done || v != expect || skip0) st = SNAPPY_ST_HEADER;
        ip = k;
    }

    // ---- the unit starts inside the element at c0: resume it
    if (st == SNAPPY_ST_OK && skip0) {
        const uint32_t o = (uint32_t)(c0 - B);  // < 4
        const uint64_t v = (((uint64_t)WDW(1) << 32) | WDW(0)) >> (8 * o);  // tag + 4 bytes
        const uint32_t tag = (uint32_t)v & 0xFF, t = tag & 3, m = tag >> 2;
        uint32_t hl, off = 0;
        uint64_t len;
        if (t == 0) {
            const uint32_t k = m >= 60 ? m - 59 : 0;
            hl = 1 + k;
            len = (k ? ((v >> 8) & ((1ull << (8 * k)) - 1)) : m) + 1ull;
        } else if (t == 1) {
            hl = 2;
            len = (m & 7) + 4;
            off = ((tag >> 5) << 8) | ((uint32_t)(v >> 8) & 0xFF);
        } else {
            hl = t == 2 ? 3 : 5;
            len = m + 1;
            off = (uint32_t)(v >> 8) & (t == 2 ? 0xFFFFu : 0xFFFFFFFFu);
        }
        const uint64_t size = t == 0 ? hl + len : hl;
        if (skip0 >= len || size > clen) {
            st = SNAPPY_ST_TRUNCATED;
        } else {
            const uint64_t r = len - skip0;
            const uint32_t k = r < want ? (uint32_t)r : want;
            if (t == 0) {
                k4_literal_hbm(comp + c0 + hl + skip0, k, 0, ob, M, dst, lane);
                F = k;
            } else if (off == 0 || (uint64_t)off + skip0 > base) {
                st = SNAPPY_ST_OFFSET;
            } else if constexpr (!BACK) {
                st = SNAPPY_ST_DEFER;
            } else {
                // byte j of the unit is copy byte j + skip0: out[-skip0 - off + (j + skip0) mod off],
                // always before the unit
                const int64_t s0 = -(int64_t)skip0 - (int64_t)off;
                const int64_t s1 = s0 + (int64_t)(len < off ? len : off) - 1;
                st = k4_wait(status, base + s0, base + (s1 < -1 ? s1 : -1), unit, lane, &done_lo);
                if (st == SNAPPY_ST_OK && lane < k) ob[lane & M] = dst[s0 + (int64_t)((lane + skip0) % off)];
            }
            op = k;
            ip = (uint32_t)size;
        }
    }

#ifdef SNAPPY_K4_STATS
    const uint64_t t_loop = clock64();
    uint32_t n_el = 0, n_batch = 0, n_pass = 0, n_sub = 0, n_far = 0;
    uint64_t sg0 = 0, sg1 = 0, sg2 = 0, ta, tb, tc, td;
    // batch shape: halves parsed, parsed elements (E), and what ended the batch
    // before E: a bad element (tail / error), a literal leaving the window, the
    // output span; batches with E == 64; batches after a span cut (one half)
    uint32_t n_half = 0, n_E = 0, n_cut_bad = 0, n_cut_long = 0, n_cut_span = 0, n_full = 0, n_spanb = 0;
    uint32_t n_stop_win = 0;  // batches whose halves stopped at the window limit (E < 64)
#endif
#ifndef SNAPPY_K4_SPAN_ADAPT
#define SNAPPY_K4_SPAN_ADAPT 1
#endif
// SNAPPY_K4_JSIZE: the batch parse's jumps take a long literal (m >= 60) as
// leaving the 64 positions; only the last element's exact size is computed
#ifndef SNAPPY_K4_JSIZE
#define SNAPPY_K4_JSIZE 0
#endif
    // the last batch was cut by the 1,024-byte output span (long copies): parse one
    // half only -- more elements would be cut again (repeat-like data)
    bool span_cut = false;
    while (st == SNAPPY_ST_OK && op < want) {
        if (ip >= clen) { st = SNAPPY_ST_TRUNCATED; break; }
        K4STAMP(ta);
        uint32_t o = (uint32_t)(c0 + ip - B);
        if (o >= 256) {
            if (o < 512) {  // slide by 256 bytes: the prefetched segment fills the free slot
                B += 256;
                o -= 256;
                ws = ws == 2 ? 0 : ws + 1;
                put_seg(ws == 2 ? 0 : ws + 1, pre);
            } else {  // jumped past the window (long literal): restart it here
                B = (c0 + ip) & ~3ull;
                o = (uint32_t)(c0 + ip - B);
                ws = 0;
                put_seg(0, load_seg(comp, B, c1, lane));
                put_seg(1, load_seg(comp, B + 256, c1, lane));
            }
            __builtin_amdgcn_wave_barrier();
            pre = load_seg(comp, B + 512, c1, lane);
        }
        // ---- a batch parses up to two 64-position halves of the window: half A
        // at o, half B at o + xa, where A's element chain leaves its 64
        // positions.  The two chains' elements are merged into lanes 0 .. E - 1
        // (E <= 64) and decoded once: the per-element work (decode, scans,
        // validity, the passes' setup) runs on up to twice the elements, and the
        // byte passes over up to twice the output.
        K4STAMP(tb);
        uint32_t ex0, eb4, E;  // merged element k at lane k: its bytes 0..3 and 1..4
        {
            // lane l <- the bytes at window position ho + l (two aligned dwords: one
            // ds_read2_b32; unaligned LDS reads measured slower), its element size,
            // then the element chain from ho by pointer doubling (lane k <- element
            // k: bytes, count; the position after the last one in the 64, xa)
            auto parse_half = [&](uint32_t ho, uint32_t &hx0, uint32_t &hb4, uint32_t &hE, uint32_t &hexit) {
                const uint32_t qa = WADR(ho + lane);
                const uint32_t dA = w32[qa >> 2], dB = w32[(qa >> 2) + 1];
                const uint32_t sh = 8 * (qa & 3);
                const uint32_t x0 = __builtin_amdgcn_alignbit(dB, dA, sh);      // tag, t1, t2, t3
                const uint32_t b4 = __builtin_amdgcn_alignbit(dB >> sh, x0, 8);  // t1 .. t4
                // element size: literal 1 + k + (length - 1) + 1, copies 2 / 3 / 5
                // (src/snappy_decompression.c:290-333)
                const uint32_t tag = x0 & 0xFF, m = tag >> 2, t = tag & 3;
#if SNAPPY_K4_JSIZE == 2
                const uint32_t k = __builtin_elementwise_sub_sat(m, 59u);
                const uint32_t lv = k ? b4 & (0xFFFFFFFFu >> ((32 - 8 * k) & 31)) : m;
                const uint32_t xsize = t == 0 ? lv + k + 2 : (0x5320u >> (4 * t)) & 0xF;
                const uint32_t size = t == 0 ? (m < 60 ? m + 2 : 64u) : (0x5320u >> (4 * t)) & 0xF;
#elif SNAPPY_K4_JSIZE
                // for the jumps only: a literal with m >= 60 is >= 63 bytes, taken as
                // leaving the 64 (at lane 0 it may end at 63: the half then ends one
                // element early, and the next starts at its exact end, hexit below)
                const uint32_t size = t == 0 ? (m < 60 ? m + 2 : 64u) : (0x5320u >> (4 * t)) & 0xF;
#else
                const uint32_t k = __builtin_elementwise_sub_sat(m, 59u);
                const uint32_t lv = k ? b4 & (0xFFFFFFFFu >> ((32 - 8 * k) & 31)) : m;
                const uint32_t size = t == 0 ? lv + k + 2 : (0x5320u >> (4 * t)) & 0xF;
#endif
                // positions as ds_bpermute addresses (4 x position); one >= 256 has
                // left the 64 and must stay >= 256 (its exact value is never used).
                // Every jump goes forward (an element is >= 2 bytes: T[a / 4] > a for
                // a < 256), so max(bpermute, a) is the jump inside the 64 and keeps an
                // exited position >= 256 (bpermute wraps addr[7:2]): one v_max per
                // step instead of a compare and a select
                const uint32_t J1 = 4 * lane + 4 * (size < 64 ? size : 64);
#define JUMP(T, a) ({ const uint32_t _a = (a);                                            \
        const uint32_t _g = (uint32_t)__builtin_amdgcn_ds_bpermute((int)_a, (int)(T));     \
        _g > _a ? _g : _a; })
                const uint32_t J2 = JUMP(J1, J1);
                const uint32_t J4 = JUMP(J2, J2);
                const uint32_t J8 = JUMP(J4, J4);
                const uint32_t J16 = JUMP(J8, J8);
                // (bpermute must run with every lane active: select afterwards).  An
                // element is at least 2 bytes, so 64 positions hold at most 32
                // elements: lanes >= 32 (copies of lanes 0-31) are out of the half
                uint32_t pos4 = 0;
                { const uint32_t g = JUMP(J1, pos4); pos4 = (lane & 1) ? g : pos4; }
                { const uint32_t g = JUMP(J2, pos4); pos4 = (lane & 2) ? g : pos4; }
                { const uint32_t g = JUMP(J4, pos4); pos4 = (lane & 4) ? g : pos4; }
                { const uint32_t g = JUMP(J8, pos4); pos4 = (lane & 8) ? g : pos4; }
                { const uint32_t g = JUMP(J16, pos4); pos4 = (lane & 16) ? g : pos4; }
#undef JUMP
                hE = (uint32_t)__builtin_popcountll(__ballot(pos4 < 256) & 0xFFFFFFFFull);  // >= 1
                hx0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)pos4, (int)x0);
                hb4 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)pos4, (int)b4);
                const uint32_t last = (uint32_t)__builtin_amdgcn_readlane(pos4, hE - 1) >> 2;
#if SNAPPY_K4_JSIZE == 2
                hexit = last + (uint32_t)__builtin_amdgcn_readlane(xsize, last);
#elif SNAPPY_K4_JSIZE
                {  // the last element's exact size, in scalar registers
                    const uint32_t lx = (uint32_t)__builtin_amdgcn_readlane(x0, last);
                    const uint32_t lb = (uint32_t)__builtin_amdgcn_readlane(b4, last);
                    const uint32_t ltag = lx & 0xFF, lm = ltag >> 2, lt = ltag & 3;
                    uint32_t lk;  // max(m, 59) - 59 in scalar code (the compiler's saturating form is VALU)
                    asm("s_max_u32 %0, %1, 59" : "=s"(lk) : "s"(lm) : "scc");
                    lk -= 59;
                    const uint32_t llv = lk ? lb & (0xFFFFFFFFu >> ((32 - 8 * lk) & 31)) : lm;
                    hexit = last + (lt == 0 ? llv + lk + 2 : (0x5320u >> (4 * lt)) & 0xF);
                }
#else
                hexit = last + (uint32_t)__builtin_amdgcn_readlane(size, last);
#endif
            };
            uint32_t ax0, ab4, ea, xa;
            parse_half(o, ax0, ab4, ea, xa);
            ex0 = ax0;
            eb4 = ab4;
            E = ea;
            // more halves where the previous half's chain exits, while its 64
            // positions and their 5 bytes stay in the valid window (bytes [0, 512)
            // from B: hpos + 63 + 5 < 512) and lanes are free; elements past lane 63
            // are dropped (the batch is a prefix of the element sequence, and the
            // next batch starts after its last element).  Lanes >= E take the new
            // half's element lane - E.  A/B on 1 GiB, outputs identical
            // (profiles/r04a_ab_k4_*, r04k_ab_k4_*): K4 per GiB of 32 KiB text
            // streams 3.11 / 2.65-2.69 / 2.51 ms with 1 / 2 / 3 halves, 64 KiB
            // blocks 3.36 / 2.85-2.90 / 2.69-2.74
#ifndef SNAPPY_K4_HALVES
#define SNAPPY_K4_HALVES 3
#endif
            uint32_t hpos = o + xa;
#ifdef SNAPPY_K4_STATS
            n_half++;
            n_spanb += span_cut;
#endif
#pragma unroll
            for (int hh = 1; hh < SNAPPY_K4_HALVES; hh++) {
#ifdef SNAPPY_K4_STATS
                n_stop_win += (E < 64 && hpos > 440 && !span_cut) ? 1u : 0u;
#endif
                if (!(E < 64 && hpos <= 440) || (SNAPPY_K4_SPAN_ADAPT && span_cut)) break;
#ifdef SNAPPY_K4_STATS
                n_half++;
#endif
                uint32_t bx0, bb4, eb, xb;
                parse_half(hpos, bx0, bb4, eb, xb);
                const int sa = (int)(4 * (lane - E));
                const uint32_t sx0 = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)bx0);
                const uint32_t sb4 = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, (int)bb4);
                const bool fa = lane < E;
                ex0 = fa ? ex0 : sx0;
                eb4 = fa ? eb4 : sb4;
                E = E + eb < 64 ? E + eb : 64;
                hpos += xb;
            }
        }
        // lane k < E holds element k of the batch; lanes >= E hold garbage,
        // masked by `live` / nexec below.  Decode: tag dispatch as selects of
        // precomputed values (no exec-mask branches; src/snappy_decompression.c:290-333)
        uint32_t e_t, e_size, e_len, e_info;  // e_info: copy offset, or literal header length
        {
            const uint32_t tag = ex0 & 0xFF, m = tag >> 2;
            e_t = tag & 3;
            const uint32_t k = __builtin_elementwise_sub_sat(m, 59u);  // literal: extra length bytes
            const uint32_t lx = eb4 & (0xFFFFFFFFu >> ((32 - 8 * k) & 31));
            const uint32_t lv = k ? lx : m;
            const uint32_t l_olen = lv + 1, c1_olen = (m & 7) + 4, c_olen = m + 1;
            const uint32_t c1b = ((tag >> 5) << 8) | (eb4 & 0xFF), c2b = eb4 & 0xFFFF, l_info = 1 + k;
            const uint32_t l_size = lv + k + 2, c_size = (0x5320u >> (4 * e_t)) & 0xF;  // copies: 2, 3, 5 bytes
            const bool is_l = e_t == 0, is_c1 = e_t == 1, is_c2 = e_t == 2;
            const uint32_t cx_olen = is_c1 ? c1_olen : c_olen;
            e_len = is_l ? l_olen : cx_olen;  // garbage lengths are clamped below
            const uint32_t c24 = is_c2 ? c2b : eb4;
            const uint32_t cx_info = is_c1 ? c1b : c24;
            e_info = is_l ? l_info : cx_info;
            e_size = is_l ? l_size : c_size;
        }
        // exclusive prefix sums of compressed sizes and output lengths over
        // the batch (64-bit safe: garbage past E is zeroed)
        const bool live = lane < E;
        // both scans as one over size | len << 16, each clamped to 1,023: exact for
        // every lane, because only the batch's last element can exceed 440 in either
        // (an element followed by another of its half is < 64 bytes; one that ends a
        // half is followed by another half only when that starts <= 440 bytes into
        // the window), so a clamped value never enters another lane's prefix, and 64
        // clamped values sum below 2^16 (no carry between the halves)
        uint32_t in_off, out_off;
        {
            const uint32_t pk = live ? (__builtin_elementwise_min(e_size, 1023u) |
                                        (__builtin_elementwise_min(e_len, 1023u) << 16)) : 0u;
            const uint32_t ex = wave_incl_scan(pk) - pk;
            in_off = ex & 0xFFFF;
            out_off = ex >> 16;
        }
        // validity in stream order: stop at the first element that runs past the
        // unit (truncated / overrun), reaches before the stream start, or needs
        // an earlier unit's bytes (pass 1: DEFER); an element running past the
        // unit's end is cut there when the index says the next unit resumes it
        const uint32_t e_ip = ip + in_off, e_op = op + out_off;
        int32_t e_err = SNAPPY_ST_OK;
        bool e_back = false;
        if constexpr (BACK) {
            if (e_op >= want) {
                e_err = 1;  // done before this element: not an error
            } else if (e_size > clen - e_ip) {
                e_err = SNAPPY_ST_TRUNCATED;
            } else {
                if (e_len > want - e_op) {
                    if (e_ip != tail_ip) e_err = SNAPPY_ST_OVERRUN;
                    e_len = want - e_op;
                }
                if (e_err == SNAPPY_ST_OK && e_t != 0 && (e_info == 0 || e_info > e_op)) {
                    if (e_info == 0 || e_info - e_op > back_lim) e_err = SNAPPY_ST_OFFSET;
                    else e_back = true;
                }
            }
        } else {
            // (selects of precomputed conditions, not exec-mask branches)
            const bool done = e_op >= want;  // done before this element: not an error
            const bool trunc = e_size > clen - e_ip;
            const bool back = e_t != 0 && e_info - 1 >= e_op;  // offset 0, or reaching before the unit
            const int32_t back_err = e_info ? SNAPPY_ST_DEFER : SNAPPY_ST_OFFSET;
            const int32_t tail_err = e_len > want - e_op ? kK4Tail : SNAPPY_ST_OK;
            const int32_t e3 = back ? back_err : tail_err;
            const int32_t e2 = trunc ? SNAPPY_ST_TRUNCATED : e3;
            e_err = done ? 1 : e2;
        }
        const uint64_t badm = __ballot(live && e_err != SNAPPY_ST_OK);
        uint32_t nexec = E;
#ifdef SNAPPY_K4_STATS
        n_E += E;
        n_full += E == 64;
        const uint32_t nexec_e = E;
#endif
        if (badm) {
            nexec = (uint32_t)__builtin_ctzll(badm);
            int32_t er = __builtin_amdgcn_readlane(e_err, nexec);
            if (!BACK && er == kK4Tail) {
                // the element runs past the unit's end: legal when the index says
                // the next unit resumes it (entry u+1 re-read here, off the loop state)
                const uint32_t t_ip = rfl(tail_lds[0]), t_op = rfl(tail_lds[1]);
                const uint32_t kip = __builtin_amdgcn_readlane(e_ip, nexec);
                const uint32_t kop = __builtin_amdgcn_readlane(e_op, nexec);
                er = SNAPPY_ST_OVERRUN;
                if (kip == t_ip && kop == t_op) {  // run it: op_end / op / the literal length are cut at want below
                    er = 1;
                    nexec++;
                }
            }
            // pass 1: DEFER (a copy into an earlier unit) is final for a STREAMS
            // unit (its own stream): the host reports it as SNAPPY_AMD_ERR_OFFSET
            if (er != 1) st = er;
        }
        K4STAMP(tc);
        // ---- a literal whose bytes leave the register window ends the batch;
        // as the batch's first element it is copied straight from HBM
        const uint32_t e_lsrc = (uint32_t)(c0 + e_ip - B) + e_info;  // literal data, window byte offset
        const uint64_t longm = __ballot(lane < nexec && e_t == 0 && e_lsrc + e_len > 508);
        if (longm) {
            const uint32_t k = (uint32_t)__builtin_ctzll(longm);
            if (k == 0) {
                nexec = 1;
                const uint32_t kop = __builtin_amdgcn_readlane(e_op, 0);
                const uint32_t kl0 = __builtin_amdgcn_readlane(e_len, 0);
                const uint32_t kl = kl0 < want - kop ? kl0 : want - kop;  // a tail element ends at want
                const uint32_t kip = __builtin_amdgcn_readlane(e_ip, 0);
                const uint32_t ki = __builtin_amdgcn_readlane(e_info, 0);
                // everything before the literal goes out first
                k4_flush(ob, M, dst, F, kop, lane);
                k4_literal_hbm(comp + c0 + kip + ki, kl, kop, ob, M, dst, lane);
                F = kop + kl;
            } else {
                nexec = k;
            }
        }
        // ---- byte passes over the batch output [op, op_end), 64 bytes each:
        // byte lane l finds its element from the bitmap of element starts,
        // literals read the window, copies the LDS ring (or HBM beyond it); a
        // copy byte whose source lies in the same pass takes it from that lane
        // by pointer jumping (out[op+j] = out[op-off + j mod off], :273-280).
        if (nexec && !(longm && (longm & 1))) {
            // the bitmap must hold the batch's output: cut the batch (never below
            // one element: the first is <= 508 bytes).  The ring then holds [F,
            // op_end) too: a batch starts with op - F < kK4FlushAt (the flush below),
            // and kK4FlushAt + kK4MapBits <= ring - 64
            static_assert(kK4FlushAt + kK4MapBits <= kK4Ring - 64, "K4: the ring must hold [F, op_end)");
            const uint64_t over = __ballot(lane < nexec && lane > 0 &&
                                           out_off + e_len > kK4MapBits);
#ifdef SNAPPY_K4_STATS
            const uint32_t nexec_l = nexec;
#endif
            if (over) nexec = (uint32_t)__builtin_ctzll(over);
            span_cut = over != 0;
#ifdef SNAPPY_K4_STATS
            n_cut_span += nexec < nexec_l;
            n_cut_long += (longm != 0) && nexec_l < E;
            n_cut_bad += (badm != 0) && (uint32_t)__builtin_ctzll(badm) < nexec_e;
#endif
            if constexpr (BACK) {
                // copies reading earlier units: wait until those bytes are in HBM
                uint64_t bm = __ballot(e_back && lane < nexec);
                if (bm) {
                    int64_t lo_s = INT64_MAX, hi_s = INT64_MIN;
                    while (bm) {
                        const uint32_t k = (uint32_t)__builtin_ctzll(bm);
                        bm &= bm - 1;
                        const int64_t s = (int64_t)(uint32_t)__builtin_amdgcn_readlane(e_op, k) -
                                          (int64_t)(uint32_t)__builtin_amdgcn_readlane(e_info, k);
                        const uint32_t kl = __builtin_amdgcn_readlane(e_len, k);
                        const uint32_t ki = __builtin_amdgcn_readlane(e_info, k);
                        const int64_t h = s + (int64_t)(kl < ki ? kl : ki) - 1;
                        lo_s = s < lo_s ? s : lo_s;
                        hi_s = h > hi_s ? h : hi_s;
                    }
                    if (hi_s > -1) hi_s = -1;
                    st = k4_wait(status, base + lo_s, base + hi_s, unit, lane, &done_lo);
                    if (st != SNAPPY_ST_OK) nexec = 0;
                }
            }
        }
        if (nexec && !(longm && (longm & 1))) {
            uint32_t op_end = op + __builtin_amdgcn_readlane(out_off, nexec - 1) +
                              __builtin_amdgcn_readlane(e_len, nexec - 1);
            op_end = op_end < want ? op_end : want;  // a tail element ends at want
            // ring slots below lo were overwritten (or are being): read those from HBM
            const uint32_t lo = op_end > ring ? op_end - ring : 0;
            const bool ex = lane < nexec;
            // the batch's element starts as a bitmap over [op, op_end): bit j of
            // dword j / 32 = an element starts at op + j (out_off < kK4MapBits, see
            // `over`); lane w < 32 keeps dword w, pass i reads dwords 2i, 2i + 1
            // (all three as u32 accesses, each behind a compiler barrier: one wave's
            // LDS operations complete in issue order, so only the compiler could
            // reorder the clear, the or and the read; lanes w and w + 32 store
            // the same zero into dword w)
            map32[lane & 31] = 0;
            asm volatile("" ::: "memory");
            if (ex) __hip_atomic_fetch_or(map32 + (out_off >> 5), 1u << (out_off & 31), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
            asm volatile("" ::: "memory");
            const uint32_t bm = map32[lane & 31];
            // element k: kop = output start | literal flag (bit 31); kinfo = the
            // copy offset, or for a literal its window address (slot base + data
            // start) + 2^31, so that kinfo + (o - kop) is byte o's window address
            // (a pass with one per-element base, x = o + kd, measured 0.7 % slower on
            // 32 KiB streams and 1.3 % on 64 KiB blocks: profiles/r04a_ab_k4_*, r04b_ab_k4_*)
            const uint32_t kop = e_op | (e_t == 0 ? 0x80000000u : 0u);
            const uint32_t kinfo = e_t == 0 ? (256 * ws + e_lsrc) ^ 0x80000000u : e_info;
            uint32_t cb = 0;  // elements starting before the pass
            if constexpr (!BACK) {
            // pass 1: a byte's address from one per-element value, kx = the literal's
            // window address - its output start, or - the copy offset: t = o + kx is the
            // window address (literal) or the source (copy); a copy overlaps its own
            // output iff t >= its start (d >= off), far iff t < lo.  (A software-
            // pipelined asm form of this loop, with every wait written out and four
            // VALU fewer per pass, measured the same: DESIGN.md 4.3.)
            const uint32_t kx = e_t == 0 ? 256 * ws + e_lsrc - e_op : 0u - e_info;
            for (uint32_t P = op, i = 0; P < op_end; P += 64, i++) {
                const uint64_t sm = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(bm, 2 * i + 1) << 32) |
                                    (uint32_t)__builtin_amdgcn_readlane(bm, 2 * i);
                const uint64_t sm1 = sm >> 1;
                const uint32_t id = __builtin_amdgcn_mbcnt_hi(
                    (uint32_t)(sm1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sm1, cb - 1 + (uint32_t)(sm & 1)));
                cb += (uint32_t)__builtin_popcountll(sm);
                const uint32_t f_op = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(id << 2), (int)kop);
                const uint32_t f_x = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(id << 2), (int)kx);
                const uint32_t o = P + lane;
                const bool lit = (int32_t)f_op < 0;
                const bool pend = o < op_end;
                uint32_t t = o + f_x;
                const bool far = pend && !lit && t < lo;
                uint32_t fv;
                asm volatile("" : "=v"(fv));  // (no initial value: read only where far)
#ifndef SNAPPY_K4_NOFAR
                if (far) fv = dst[t];
#endif
                const uint32_t a2 = t - 768;
                const uint32_t lb = wb[__builtin_elementwise_min(__builtin_elementwise_min(t, a2), 783u)];
                if (pend && !lit && !far && t >= f_op) {
                    // overlapping copy (off < len <= 64): source byte d mod off
                    const uint32_t off = 0u - f_x, d = o - f_op;
                    const float r = __builtin_amdgcn_rcpf((float)off);
                    const uint32_t qd = (uint32_t)((float)d * r + 0.0001f);
                    t = f_op - off + (d - qd * off);
                }
#ifdef SNAPPY_K4_STATS
                n_far += __ballot(far) != 0;
                n_pass++;
#endif
                // a source in this pass: copy lanes' t (< 2^31), -1 elsewhere (one compare
                // for the ballot: a ballot of the and of the conditions went through a
                // 0 / 1 VGPR and a second compare)
                const int32_t tin = (pend && !lit && !far) ? (int32_t)t : -1;
                const uint8_t rv = ob[t & M];
                const uint8_t lr = lit ? (uint8_t)lb : rv;
                uint32_t val = far ? fv : (uint32_t)lr;
                if (__builtin_expect(__ballot(tin >= (int32_t)P) != 0, 0)) {
                    uint32_t rt = tin >= (int32_t)P ? t - P : lane;
                    for (;;) {
#ifdef SNAPPY_K4_STATS
                        n_sub++;
#endif
                        const uint32_t r2 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(rt << 2), (int)rt);
                        if (!__ballot(r2 != rt)) break;
                        rt = r2;
                    }
                    val = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(rt << 2), (int)val);
                }
                ob[pend ? (o & M) : kK4Ring] = (uint8_t)val;
#ifdef SNAPPY_K4_STATS
                n_sub++;
#endif
            }
            } else
            // pass P: byte lane l writes output byte o = P + l
            for (uint32_t P = op, i = 0; P < op_end; P += 64, i++) {
                const uint64_t sm = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(bm, 2 * i + 1) << 32) |
                                    (uint32_t)__builtin_amdgcn_readlane(bm, 2 * i);
                // the byte's element: cb - 1 + the starts in [P, P + l] (the first
                // pass starts with one, so it is never -1)
                const uint64_t sm1 = sm >> 1;
                const uint32_t id = __builtin_amdgcn_mbcnt_hi(
                    (uint32_t)(sm1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sm1, cb - 1 + (uint32_t)(sm & 1)));
                cb += (uint32_t)__builtin_popcountll(sm);
                const uint32_t f_op = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(id << 2), (int)kop);
                const uint32_t f_in = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(id << 2), (int)kinfo);
                const uint32_t o = P + lane;
                const uint32_t d = o - f_op;  // a literal's carries 2^31, cancelled by its kinfo
                const bool lit = (int32_t)f_op < 0;
                const bool pend = o < op_end;
                // copy source (pass 2: negative = an earlier unit).  Below lo only
                // HBM holds the byte: a far copy never overlaps (off > ring - 64 >
                // len), so its load goes out first, into a register of its own
                SrcT src = (SrcT)o - (SrcT)f_in;
                bool far = pend && !lit && src < (SrcT)lo;
                uint32_t fv = 0;
#ifndef SNAPPY_K4_NOFAR  // (experiment only: wrong output, measures what the far loads cost)
                if (far) fv = dst[src];
#endif
                // literal byte: the window's LDS copy (3 slots of 256 bytes), read
                // by every lane (no exec change): a copy lane's address is clamped
                uint32_t a = f_in + d;
                const uint32_t a2 = a - 768;
                a = a < a2 ? a : a2;
                const uint32_t lb = wb[a < 783 ? a : 783];
                if (pend && !lit && !far && d >= f_in) {
                    // overlapping copy (off < len <= 64): source byte d mod off
                    const float r = __builtin_amdgcn_rcpf((float)f_in);
                    const uint32_t qd = (uint32_t)((float)d * r + 0.0001f);
                    src = (SrcT)f_op - (SrcT)f_in + (SrcT)(d - qd * f_in);
                    if constexpr (BACK) {
                        // near the unit start it may repeat bytes of an earlier unit
                        if (src < (SrcT)lo) {
                            fv = dst[src];
                            far = true;
                        }
                    }
                }
                const bool direct = lit || far;
#ifdef SNAPPY_K4_STATS
                n_far += __ballot(pend && !lit && direct) != 0;
                n_pass++;
#endif
                // every lane reads the ring (a byte whose source lies in this pass
                // reads garbage, replaced below) and writes (a lane past op_end to the
                // dummy byte after the ring): no exec changes
                const bool inpass = pend && !direct && src >= (SrcT)P;
                // two selects, each over values every lane loaded, kept as bytes: with
                // val = lit ? lb : (far ? fv : rv) the compiler sank the ring read into an
                // exec-masked region for the copy lanes and zero-extended (and waited for)
                // the window byte where it was read (K4 text32k 3.18 -> 3.10 ms per GiB,
                // 64 KiB blocks 3.45 -> 3.36; profiles/r03s2r_*)
                const uint8_t rv = ob[(uint32_t)src & M];
                const uint8_t lr = lit ? (uint8_t)lb : rv;
                uint32_t val = far ? fv : (uint32_t)lr;
                if (__builtin_expect(__ballot(inpass) != 0, 0)) {
                    // out[op+j] = out[op-off + j mod off] (:273-280) with the source in
                    // this pass: lane src - P (a lower lane) holds it.  Follow those
                    // links by pointer jumping to a lane whose value is known (direct,
                    // or read from the ring), then take its value
                    uint32_t rt = inpass ? (uint32_t)(src - (SrcT)P) : lane;
                    for (;;) {
#ifdef SNAPPY_K4_STATS
                        n_sub++;
#endif
                        const uint32_t r2 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(rt << 2), (int)rt);
                        if (!__ballot(r2 != rt)) break;
                        rt = r2;
                    }
                    val = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(rt << 2), (int)val);
                }
                ob[pend ? (o & M) : kK4Ring] = (uint8_t)val;
#ifdef SNAPPY_K4_STATS
                n_sub++;
#endif
            }
        }
        K4STAMP(td);
#ifdef SNAPPY_K4_STATS
        sg0 += tb - ta;
        sg1 += tc - tb;
        sg2 += td - tc;
        n_batch++;
        n_el += nexec;
#endif
        if (nexec) {
            ip += __builtin_amdgcn_readlane(in_off, nexec - 1) + __builtin_amdgcn_readlane(e_size, nexec - 1);
            op += __builtin_amdgcn_readlane(out_off, nexec - 1) + __builtin_amdgcn_readlane(e_len, nexec - 1);
            op = op < want ? op : want;
            if (op - F >= kK4FlushAt) {
                const uint32_t T = op & ~(kK4FlushGran - 1);
                k4_flush(ob, M, dst, F, T, lane);
                F = T;
                if constexpr (BACK) k4_publish(status, u, SNAPPY_ST_DEFER + (int32_t)F, lane);
            }
        } else if (st == SNAPPY_ST_OK && op < want) {
            st = SNAPPY_ST_TRUNCATED;  // no progress possible
        }
    }
#undef WADR
#undef WDW
    // SINGLE: a unit whose last element ends inside it (skip1 == 0) must end
    // exactly at the next entry.  Block 0 starts after the checked preamble,
    // so by induction every entry of an index that passes is a true element
    // boundary (and a straddle entry is tied to the chain by the tail check
    // above): a sidecar entry moved inside an element is refused here instead
    // of decoding a shifted block.  The last unit may leave bytes unread, as
    // the reference does (src/snappy_decompression.c:356-359 stops at N).
    if (st == SNAPPY_ST_OK && allow_back && !skip1 && base + unit < n && ip != clen) st = SNAPPY_ST_INDEX;
#ifdef SNAPPY_K4_STATS
    if (lane == 0 && u < 32768) {
        uint64_t *g = g_k4_stats + 16 * u;
        g[8] = n_half;
        g[9] = n_E;
        g[10] = n_cut_bad;
        g[11] = n_cut_long;
        g[12] = n_cut_span;
        g[13] = n_full;
        g[14] = n_spanb;
        g[15] = n_stop_win;
        g[0] = clock64() - t_loop;
        g[1] = n_el | ((uint64_t)n_far << 32);
        g[2] = n_batch;
        g[3] = n_pass;
        g[4] = n_sub;
        g[5] = sg0;
        g[6] = sg1;
        g[7] = sg2;
    }
#endif
    __syncthreads();

    k4_flush(ob, M, dst, F, op < want ? op : want, lane);
    if constexpr (BACK) {
        k4_publish(status, u, st, lane);
    } else {
        if (lane == 0) status[u] = st;
        // status[units + 1] = pass 2 has work (status[units] is pass 2's ticket counter)
        if (st == SNAPPY_ST_DEFER && lane == 0) status[gridDim.x + 1] = 1;
    }
}

#if SNAPPY_TU_DECODE
#ifndef SNAPPY_K4_WAVES
#define SNAPPY_K4_WAVES 8  // waves per SIMD: <= 64 VGPRs, <= 80 SGPRs (5,028 B of LDS: 32 per CU fit)
#endif
__global__ __launch_bounds__(64, SNAPPY_K4_WAVES) void k4_decompress_units(
    const uint8_t *__restrict__ comp, const uint64_t *__restrict__ offsets, uint64_t n, uint32_t unit,
    uint32_t hdr_mode, uint64_t header_value, uint32_t allow_back, uint32_t bias, uint8_t *__restrict__ out,
    int32_t *__restrict__ status)
{
    k4_body<false>(comp, offsets, n, unit, hdr_mode, header_value, allow_back, bias, out, status, blockIdx.x);
}
#endif

#if SNAPPY_TU_DECODE
__global__ __launch_bounds__(64) void k4_decompress_back(const uint8_t *__restrict__ comp,
                                                         const uint64_t *__restrict__ offsets, uint64_t n,
                                                         uint32_t unit, uint32_t hdr_mode, uint64_t header_value,
                                                         uint32_t bias, uint8_t *__restrict__ out,
                                                         int32_t *__restrict__ status)
{
    // status[units + 1] == 0: pass 1 deferred nothing (the common case: every wave leaves at once)
    if (*reinterpret_cast<const volatile int32_t *>(status + gridDim.x + 1) == 0) return;
    // tickets in dispatch order: a unit only ever waits for lower tickets
    uint32_t tk = 0;
    if (threadIdx.x == 0) tk = atomicAdd(reinterpret_cast<uint32_t *>(status + gridDim.x), 1u);
    const uint32_t u = __builtin_amdgcn_readfirstlane(tk);
    if (status[u] != SNAPPY_ST_DEFER) return;
    k4_body<true>(comp, offsets, n, unit, hdr_mode, header_value, 1u, bias, out, status, u);
}
#endif
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

#if SNAPPY_TU_DECODE
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
    if (st == SNAPPY_ST_OK && units >= max_units) st = SNAPPY_ST_CAPACITY;  // units + 1 entries needed
    uint64_t op = 0, unit = 0;
    if (st == SNAPPY_ST_OK && lane == 0 && units) offsets[0] = 0;
    unit = 1;
    while (st == SNAPPY_ST_OK && op < N) {
        if (ip >= clen) { st = SNAPPY_ST_TRUNCATED; break; }
        const uint64_t x = ip;  // element start
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
        // boundaries strictly inside [op, op+len): straddle entries (element
        // start | bytes of it before the boundary << 40)
        while (unit * SNAPPY_BLOCK < op + len && unit * SNAPPY_BLOCK < N) {
            const uint64_t skip = unit * SNAPPY_BLOCK - op;
            if ((skip >> 24) || (x >> 40)) { st = SNAPPY_ST_UNSUPPORTED; break; }
            if (lane == 0) offsets[unit] = x | (skip << 40);
            unit++;
        }
        if (st != SNAPPY_ST_OK) break;
        const uint64_t next_boundary = unit * SNAPPY_BLOCK;
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
#endif


// ---------------------------------------------------------------------------
// K5p: block index of a foreign SINGLE stream, chunk-parallel.  A stream has
// no block markers (the decoder of src/snappy_decompression.c:345-363 just
// walks elements until 65,536 bytes came out), so the walk is split into
// K5_S-byte chunks of compressed stream, each staged in LDS (chunk + halo):
//   K5a  lane l walks the element chain entered at byte l of its chunk to the
//        chunk end: its exit (first start at or past the end) and output.
//        The 64 chains walk element by element, checked at every 192-byte
//        checkpoint; chains through a common start coincide from there on, so
//        once every unfinished lane stands on one start (text: at once) the
//        rest is ONE chain, walked by batch parse (every byte of a 64-byte
//        window parsed as a candidate element, the chain found by pointer
//        doubling over ds_bpermute, sizes and outputs by DPP scans).  K5a also
//        writes the chunk's entry map (entry byte -> next chunk's entry byte |
//        output << 8) for K5b1;
//   K5b1 composes the maps of 64 consecutive chunks (one ds_bpermute per chunk);
//   K5b2 (k5b_carry) one wave carries the true entry and output base over the
//        blocks of 64 chunks (one readlane per composed block; chunk by chunk
//        where a map escapes: an entry < 64 bytes in is a K5a lookup, a later
//        one walks);
//   K5b3 fills in the entry and base of every chunk of a composed block;
//   K5c  every chunk re-walks its true chain from the true entry with the true
//        output base by batch parse and records the element holding each
//        multiple of 65,536 (with the checks of K5);
//   K5d  first error in stream order, final offset.
// Chunks entirely inside one element (long literals) are skipped.
// ---------------------------------------------------------------------------
[[maybe_unused]] constexpr uint32_t K5_S = SNAPPY_K5_CHUNK;
[[maybe_unused]] constexpr uint64_t K5_SKIP = ~0ull;

struct K5Hdr {
    uint64_t N;
    uint32_t len;
    int32_t st;
};

__device__ __forceinline__ K5Hdr k5_header(const uint8_t *comp, uint64_t clen)
{
    K5Hdr h{0, 0, SNAPPY_ST_HEADER};
    for (uint32_t k = 0; k < 10 && k < clen; k++) {
        const uint32_t b = comp[k];
        h.N |= (uint64_t)(b & 0x7F) << (7 * k);
        if (!(b & 0x80)) {
            h.len = k + 1;
            h.st = SNAPPY_ST_OK;
            break;
        }
    }
    return h;
}

// element at x: compressed size and output length; false if its header
// bytes run past clen (uniform across the wave: scalar loads)
__device__ __forceinline__ bool k5_parse(const uint8_t *__restrict__ comp, uint64_t clen, uint64_t x, uint64_t &size,
                                         uint64_t &len)
{
    uint64_t v;  // bytes x .. x+4 (little-endian), zero past clen
    if (x + 8 <= clen) {
        const uint64_t a = x & ~3ull;
        const uint32_t *w = reinterpret_cast<const uint32_t *>(comp + a);
        const uint64_t d = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
        const uint32_t sh = 8 * (uint32_t)(x & 3);
        v = d >> sh;
        if (sh > 24) v |= (uint64_t)comp[x + 4] << 32;
        else v &= 0xFFFFFFFFFFull;
    } else {
        if (x >= clen) return false;
        v = 0;
        for (uint32_t k = 0; k < 5; k++)
            if (x + k < clen) v |= (uint64_t)comp[x + k] << (8 * k);
    }
    const uint32_t tag = (uint32_t)v & 0xFF;
    uint32_t hb;  // header bytes
    switch (tag & 3) {
    case 0: {
        const uint32_t m = tag >> 2;
        if (m < 60) {
            len = m + 1;
            hb = 1;
        } else {
            const uint32_t k = m - 59;
            len = ((v >> 8) & (k == 4 ? 0xFFFFFFFFull : ((1ull << (8 * k)) - 1))) + 1;
            hb = 1 + k;
        }
        size = hb + len;
        break;
    }
    case 1: len = ((tag >> 2) & 7) + 4; hb = 2; size = 2; break;
    case 2: len = (tag >> 2) + 1; hb = 3; size = 3; break;
    default: len = (tag >> 2) + 1; hb = 5; size = 5; break;
    }
    return x + hb <= clen;
}

// 64-bit readlane
__device__ __forceinline__ uint64_t rl64(uint64_t v, uint32_t l)
{
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}

// LDS image of a chunk: the dwords from c0 & ~3 on, K5_S + 128 bytes (a batch
// window starting before the chunk end reads at most 76 bytes past it), zero
// at and past clen.  Byte r of the chunk (r relative to c0) is image byte r + o0.
constexpr uint32_t K5_IMG = K5_S + 128;
[[maybe_unused]] constexpr uint32_t kK5Esc = 0xFFFFFFFFu;  // K5a entry map: no fast successor
[[maybe_unused]] constexpr uint64_t kK5Esc64 = ~0ull;      // K5b1 block map: no fast successor

// BYTES of stream from the 4-aligned absolute a0 into img (zero at and past clen)
template <uint32_t BYTES>
__device__ __forceinline__ void k5_stage_at(const uint8_t *__restrict__ comp, uint64_t clen, uint64_t a0, uint32_t *img,
                                            uint32_t lane)
{
    uint32_t v[8];
    for (uint32_t i0 = 0; i0 < BYTES / 4; i0 += 8 * 64) {
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) {  // 8 loads per lane in flight
            const uint32_t i = i0 + 64 * j + lane;
            v[j] = i < BYTES / 4 ? load_dw_guarded(comp, a0 + 4ull * i, clen) : 0u;
        }
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) {
            const uint32_t i = i0 + 64 * j + lane;
            if (i < BYTES / 4) img[i] = v[j];
        }
    }
    __syncthreads();
}

__device__ __forceinline__ void k5_stage(const uint8_t *__restrict__ comp, uint64_t clen, uint64_t c0, uint32_t *img,
                                         uint32_t lane)
{
    k5_stage_at<K5_IMG>(comp, clen, c0 & ~3ull, img, lane);
}

// K5c's image: a WIN-byte window (+ 128) re-staged as its chain moves on, so
// K5c holds 4.2 KiB of LDS (32 waves per CU) instead of the whole chunk
#ifndef SNAPPY_K5_WIN
#define SNAPPY_K5_WIN 4096
#endif
[[maybe_unused]] constexpr uint32_t K5_WIN = SNAPPY_K5_WIN;  // (K5c, decode TU)

// the element at image byte q (rem = stream bytes from it to clen): as k5_parse
__device__ __forceinline__ bool k5_parse_img(const uint32_t *img, uint32_t q, uint64_t rem, uint64_t &size,
                                             uint64_t &len)
{
    const uint32_t a = q >> 2, sh = 8 * (q & 3);
    const uint32_t d0 = img[a], d1 = img[a + 1];
    const uint32_t x0 = sh ? (d0 >> sh) | (d1 << (32 - sh)) : d0;  // bytes 0..3
    const uint32_t b4 = (d1 >> sh) & 0xFF;                        // byte 4
    const uint32_t tag = x0 & 0xFF, t = tag & 3, m = tag >> 2;
    uint32_t hb;
    if (t == 0) {
        const uint32_t k = m >= 60 ? m - 59 : 0;
        const uint32_t lv = k == 0 ? m : (k == 4 ? (x0 >> 8) | (b4 << 24) : (x0 >> 8) & ((1u << (8 * k)) - 1));
        len = (uint64_t)lv + 1;
        hb = 1 + k;
        size = hb + len;
    } else {
        len = t == 1 ? (m & 7) + 4 : m + 1;
        hb = t == 1 ? 2 : (t == 2 ? 3 : 5);
        size = hb;
    }
    return rem > 0 && hb <= rem;
}

// Walk ONE element chain (x uniform, relative to c0) while x < end_rel (and,
// MARK, op < N) by batch parse.  Not MARK (K5a): op accumulates the output, a
// header past clen ends the walk with x = clen + 1 - c0.  MARK (K5c): op is
// the absolute output position; the checks and index entries of the serial
// walk (an element holding a multiple of 65,536 strictly inside it gets a
// straddle entry, one ending on it the entry of its successor); any error
// leaves st set (the index is then discarded, so extra entries are harmless).
// The image holds the stream from the absolute 4-aligned ia on; WIN > 0: it
// is a WIN + 128-byte window, re-staged at the chain when the chain leaves it.
template <bool MARK, uint32_t WIN>
__device__ __forceinline__ void k5_chain(const uint8_t *__restrict__ comp, uint32_t *img, uint64_t &ia, uint64_t c0,
                                         uint64_t clen, uint32_t end_rel, uint64_t &x, uint64_t &op, uint64_t N,
                                         uint64_t *__restrict__ offsets, uint64_t max_units, int32_t &st, uint32_t lane)
{
    while (x < end_rel && (!MARK || op < N) && st == SNAPPY_ST_OK) {
        if constexpr (WIN > 0) {
            if (c0 + x >= ia + WIN) {  // a window's reads end before ia + WIN + 72
                ia = (c0 + x) & ~3ull;
                k5_stage_at<WIN + 128>(comp, clen, ia, img, lane);
            }
        }
        const uint32_t r = (uint32_t)x + lane;
        uint64_t size, len;
        const bool ok = k5_parse_img(img, (uint32_t)(c0 + r - ia), c0 + r < clen ? clen - (c0 + r) : 0, size, len);
        // element chain from lane 0 by pointer doubling: lane k <- start of element k
        const uint32_t nx = lane + (size < 64 ? (uint32_t)size : 64u);
#define K5JUMP(T, idx) ({ const uint32_t _i = (idx);                                                  \
        const uint32_t _g = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((_i & 63) << 2), (int)(T));    \
        _i < 64 ? _g : _i; })
        const uint32_t J1 = nx, J2 = K5JUMP(J1, J1), J4 = K5JUMP(J2, J2), J8 = K5JUMP(J4, J4), J16 = K5JUMP(J8, J8);
        uint32_t pos = 0;
        { const uint32_t g = K5JUMP(J1, pos); pos = (lane & 1) ? g : pos; }
        { const uint32_t g = K5JUMP(J2, pos); pos = (lane & 2) ? g : pos; }
        { const uint32_t g = K5JUMP(J4, pos); pos = (lane & 4) ? g : pos; }
        { const uint32_t g = K5JUMP(J8, pos); pos = (lane & 8) ? g : pos; }
        { const uint32_t g = K5JUMP(J16, pos); pos = (lane & 16) ? g : pos; }
#undef K5JUMP
        // elements of at least 2 bytes: <= 32 start in the window; only starts before the chunk end count
        const bool in = lane < 32 && pos < 64 && (uint32_t)x + pos < end_rel;
        const uint32_t E = (uint32_t)__builtin_popcountll(__ballot(in));  // lanes 0..E-1 (>= 1: lane 0 is x)
        const uint32_t pg = (in ? pos : 0u) << 2;
        const uint32_t s_lo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)pg, (int)(uint32_t)size);
        const uint32_t s_hi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)pg, (int)((uint32_t)(size >> 32) | (ok ? 0u : 0x80000000u)));
        const uint32_t l_lo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)pg, (int)(uint32_t)len);
        const uint32_t l_hi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)pg, (int)(uint32_t)(len >> 32));
        const bool live = lane < E;
        const bool e_ok = (s_hi >> 31) == 0;
        const uint64_t e_size = ((uint64_t)(s_hi & 0x7FFFFFFFu) << 32) | s_lo;
        const uint64_t e_len = ((uint64_t)l_hi << 32) | l_lo;
        // element k's relative start is x + pos: the exclusive sum of the live
        // sizes before it, every one of which ended inside the window (< 64);
        // output offsets: exclusive prefix sums of the lengths (64-bit values
        // < 2^33, as 16-bit low parts + the rest)
        uint32_t t2, t3;
        const uint32_t ll = wave_excl_scan32(live ? (uint32_t)e_len & 0xFFFF : 0u, &t2);
        const uint32_t lh = wave_excl_scan32(live ? (uint32_t)(e_len >> 16) : 0u, &t3);
        const uint64_t e_x = x + pos;  // relative start
        const uint64_t e_op = op + ((uint64_t)lh << 16) + ll;
        // the first element that ends the walk: a bad header (both), a truncated
        // element (MARK), or (MARK) one at or past N (not run) / past N (run, then OVERRUN)
        bool bad = !e_ok, skipn = false, over = false;
        if constexpr (MARK) {
            bad = bad || c0 + e_x + e_size > clen;
            skipn = e_op >= N;
            over = e_op + e_len > N;
        }
        const uint64_t stopm = __ballot(live && (bad || skipn || over));
        uint32_t nexec = E;
        int32_t er = SNAPPY_ST_OK;
        if (stopm) {
            const uint32_t k = (uint32_t)__builtin_ctzll(stopm);
            const uint32_t kb = __builtin_amdgcn_readlane((uint32_t)bad, k), ks = __builtin_amdgcn_readlane((uint32_t)skipn, k);
            if (kb) {
                nexec = k;
                er = SNAPPY_ST_TRUNCATED;
            } else if (ks) {
                nexec = k;
            } else {
                nexec = k + 1;
                er = SNAPPY_ST_OVERRUN;
            }
        }
        if constexpr (MARK) {
            const bool run = lane < nexec;
            const uint64_t e_end = e_op + e_len;
            // an element ending on a block boundary: the next entry is its successor
            if (run && (e_end & (SNAPPY_BLOCK - 1)) == 0 && e_end < N) {
                const uint64_t uu = e_end / SNAPPY_BLOCK;
                if (uu < max_units) offsets[uu] = c0 + e_x + e_size;
            }
            // boundaries strictly inside an element (rare: serial over those lanes)
            const uint64_t nb1 = (e_op / SNAPPY_BLOCK + 1) * SNAPPY_BLOCK;
            uint64_t sm = __ballot(run && nb1 < e_end && nb1 < N);
            while (sm) {
                const uint32_t k = (uint32_t)__builtin_ctzll(sm);
                sm &= sm - 1;
                const uint64_t kop = rl64(e_op, k), kend = rl64(e_end, k), kx = c0 + rl64(e_x, k);
                for (uint64_t nb = (kop / SNAPPY_BLOCK + 1) * SNAPPY_BLOCK; nb < kend && nb < N; nb += SNAPPY_BLOCK) {
                    const uint64_t skip = nb - kop;
                    if ((skip >> 24) || (kx >> 40)) {
                        er = SNAPPY_ST_UNSUPPORTED;
                        break;
                    }
                    const uint64_t uu = nb / SNAPPY_BLOCK;
                    if (lane == 0 && uu < max_units) offsets[uu] = kx | (skip << 40);
                }
            }
        }
        if (nexec) {
            x = rl64(e_x, nexec - 1) + rl64(e_size, nexec - 1);
            op = rl64(e_op, nexec - 1) + rl64(e_len, nexec - 1);
        }
        if (er != SNAPPY_ST_OK) {
            if constexpr (MARK) st = er;
            else x = clen + 1 - c0;  // a header past clen (the only error without MARK)
        }
    }
}

#if SNAPPY_TU_DECODE
__global__ __launch_bounds__(64) void k5a_chunk_walk(const uint8_t *__restrict__ comp, uint64_t clen,
                                                     uint64_t *__restrict__ X, uint64_t *__restrict__ O,
                                                     uint32_t *__restrict__ P)
{
    // lane l: the chain entered at byte l of the chunk (every entry offset < 64
    // covered exactly; chains need not converge -- a periodic stream never
    // re-synchronises, and then every lane walks alone)
    __shared__ uint32_t img[K5_IMG / 4 + 4];
    const uint32_t lane = threadIdx.x;
    const uint32_t c = blockIdx.x;
    const K5Hdr h = k5_header(comp, clen);
    const uint64_t c0 = h.len + (uint64_t)c * K5_S;
    const uint32_t end_rel = (uint32_t)(c0 + K5_S < clen ? K5_S : clen - c0);
    const uint32_t o0 = (uint32_t)(c0 & 3);
    k5_stage(comp, clen, c0, img, lane);
    uint64_t x = lane, cum = 0;
    // element by element to the checkpoint (or the end), then alone if the chains differ
    auto walk_to = [&](uint32_t lim) {
        while (__ballot(x < lim)) {
            if (x < lim) {
                uint64_t size, len;
                const uint32_t r = (uint32_t)x;
                if (!k5_parse_img(img, r + o0, c0 + r < clen ? clen - (c0 + r) : 0, size, len)) {
                    x = clen + 1 - c0;
                } else {
                    cum += len;
                    x += size;
                }
            }
        }
    };
    // checkpoints every kCheck bytes: as soon as the unfinished lanes stand on
    // one start, the rest is one batch-parsed chain
#ifndef SNAPPY_K5_CHECK
#define SNAPPY_K5_CHECK 192
#endif
    constexpr uint32_t kCheck = SNAPPY_K5_CHECK;
    for (uint32_t lim = kCheck;; lim += kCheck) {
        walk_to(end_rel < lim ? end_rel : lim);
        const uint64_t open = __ballot(x < end_rel);
        if (!open) break;
        const uint32_t x1 = __builtin_amdgcn_readlane((uint32_t)x, (uint32_t)__builtin_ctzll(open));
        if (!__ballot(x < end_rel && (uint32_t)x != x1)) {
            uint64_t xe = x1, oe = 0;
            int32_t st = SNAPPY_ST_OK;
            uint64_t ia = c0 & ~3ull;
            k5_chain<false, 0>(comp, img, ia, c0, clen, end_rel, xe, oe, 0, nullptr, 0, st, lane);
            if (x < end_rel) {
                x = xe;
                cum += oe;
            }
            break;
        }
    }
    X[(uint64_t)c * 64 + lane] = c0 + x;
    O[(uint64_t)c * 64 + lane] = cum;
    // the chunk's entry map for K5b1: the entry byte of the next chunk (< 64) |
    // output << 8, or kK5Esc when either does not fit
    const uint64_t nx = x - K5_S;
    // (only into a full next chunk: an exit past clen, or a parse error, never composes)
    P[(uint64_t)c * 64 + lane] = c0 + 2 * K5_S <= clen && x >= K5_S && nx < 64 && cum < (1u << 24)
                                     ? (uint32_t)nx | ((uint32_t)cum << 8) : kK5Esc;
}
#endif

#ifndef SNAPPY_K5_G
#define SNAPPY_K5_G 8
#endif
[[maybe_unused]] constexpr uint32_t K5_G = SNAPPY_K5_G;  // chunks per prefetch group

#if SNAPPY_TU_DECODE
// K5b1: the entry maps of 64 consecutive chunks composed (block B = chunks
// 64 B .. 64 B + 63): lane e follows the chain entered at byte e of the block's
// first chunk through the block by one ds_bpermute per chunk (the row of chunk
// c holds, per entry byte, the next chunk's entry byte | output << 8);
// F[64 B + e] = exit entry byte into the next block | output << 8, or kK5Esc64.
// A block with a short chunk (the stream's last) is never composed.
__global__ __launch_bounds__(64) void k5b1_compose(const uint32_t *__restrict__ P, uint32_t nchunks,
                                                   uint64_t *__restrict__ F)
{
    const uint32_t lane = threadIdx.x;
    const uint32_t B = blockIdx.x;
    uint32_t row[64];
#pragma unroll
    for (uint32_t j = 0; j < 64; j++)
        row[j] = P[(uint64_t)__builtin_elementwise_min(64 * B + j, nchunks - 1) * 64 + lane];
    uint32_t cur = lane;
    uint64_t out = 0;
    bool esc = 64 * B + 64 > nchunks;
#pragma unroll
    for (uint32_t j = 0; j < 64; j++) {
        const uint32_t w = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((cur & 63) << 2), (int)row[j]);
        esc = esc || w == kK5Esc;
        out += w >> 8;
        cur = w & 0xFF;
    }
    F[64 * (uint64_t)B + lane] = esc ? kK5Esc64 : (uint64_t)cur | (out << 8);
}

// K5b2: one wave carries the true entry and output base through the stream:
// a block whose entry byte is < 64, whose composed map has a fast successor
// and that ends before N costs one readlane (its first chunk's entry and base
// go to BE / BB for K5b3); any other block runs chunk by chunk (K5_G chunks per
// prefetch group, entries < 64 by K5a's X / O, later ones walked, skipped
// chunks marked) and writes its chunks' Ent / Base itself (BE = K5_SKIP).
__global__ __launch_bounds__(64) void k5b_carry(const uint8_t *__restrict__ comp, uint64_t clen, uint32_t nchunks,
                                                const uint64_t *__restrict__ X, const uint64_t *__restrict__ O,
                                                const uint64_t *__restrict__ F, uint64_t *__restrict__ BE,
                                                uint64_t *__restrict__ BB, uint64_t *__restrict__ Ent,
                                                uint64_t *__restrict__ Base, int64_t *__restrict__ result)
{
    const uint32_t lane = threadIdx.x;
    const K5Hdr h = k5_header(comp, clen);
    const uint64_t N = h.N;
    uint64_t E = h.len, base = 0;
    uint64_t xa[K5_G], oa[K5_G], xb[K5_G], ob_[K5_G];
    // walk lookahead: a run of long elements (incompressible data: one literal
    // per block, so a walk per block, each step a dependent global load) is
    // parsed 64 elements per load round trip -- after a miss parses the element
    // at x, lane k parses the one at x + k * size (the next ones, if they repeat
    // its size); later walks look their start up first.  A parse depends only on
    // its position, so a hit equals the load it replaces.
    uint64_t la_x = ~0ull, la_size = 0, la_len = 0;
    bool la_ok = false;
    auto parse_la = [&](uint64_t x, uint64_t &size, uint64_t &len) -> bool {
        const uint64_t m = __ballot(la_x == x);
        if (m) {
            const uint32_t k = (uint32_t)__builtin_ctzll(m);
            size = rl64(la_size, k);
            len = rl64(la_len, k);
            return __builtin_amdgcn_readlane((uint32_t)la_ok, k) != 0;
        }
        const bool ok = k5_parse(comp, clen, x, size, len);
        if (ok && size >= 64) {
            la_x = x + (uint64_t)lane * size;
            la_ok = k5_parse(comp, clen, la_x, la_size, la_len);
        }
        return ok;
    };
    auto load = [&](uint32_t g, uint64_t *xs, uint64_t *os) {
#pragma unroll
        for (uint32_t j = 0; j < K5_G; j++) {
            const uint64_t c = (uint64_t)g * K5_G + j;
            xs[j] = c < nchunks ? X[c * 64 + lane] : 0;
            os[j] = c < nchunks ? O[c * 64 + lane] : 0;
        }
    };
    uint32_t lookups = 0;  // K5a lookups in the current chunk-by-chunk block
    // chunk c: its entry and base, then the chain through it (a K5a lookup by
    // `look`, or a walk)
    auto step = [&](uint32_t c, auto look) {
        const uint64_t c0 = h.len + (uint64_t)c * K5_S;
        const uint64_t end = c0 + K5_S < clen ? c0 + K5_S : clen;
        if (h.st != SNAPPY_ST_OK || base >= N || E >= end) {
            if (lane == 0) Ent[c] = K5_SKIP;
            return;
        }
        if (lane == 0) {
            Ent[c] = E;
            Base[c] = base;
        }
        if (E - c0 < 64) {
            uint64_t xo, oo;
            look((uint32_t)(E - c0), xo, oo);
            base += oo;
            E = xo;
            lookups++;
        } else {  // entered past byte 63 (after a long literal): walk the chunk
            uint64_t x = E;
            while (x < end && base < N) {
                uint64_t size, len;
                if (!parse_la(x, size, len)) {
                    x = clen + 1;
                    break;
                }
                base += len;
                x += size;
            }
            E = x;
        }
    };
    auto run = [&](uint32_t g, const uint64_t *xs, const uint64_t *os) {
#pragma unroll
        for (uint32_t j = 0; j < K5_G; j++) {
            const uint32_t c = g * K5_G + j;
            if (c >= nchunks) break;
            step(c, [&](uint32_t l, uint64_t &xo, uint64_t &oo) {
                xo = rl64(xs[j], l);
                oo = rl64(os[j], l);
            });
        }
    };
    static_assert(64 % K5_G == 0, "K5_G divides a 64-chunk block");
    constexpr uint32_t kGB = 64 / K5_G;  // prefetch groups per block
    const uint32_t nblk = (nchunks + 63) / 64;
    // a chunk-by-chunk block whose predecessor of that kind needed fewer than
    // kDemand lookups (runs of long literals: incompressible data) loads its
    // lookups on demand and skips the chunks its chain jumps over, instead of
    // prefetching every chunk's 64-entry rows (a load round trip per 8 chunks)
    constexpr uint32_t kDemand = 8;
    bool demand = false;
    uint64_t fr = F[lane];  // block 0's composed map, then each next one a block ahead
    for (uint32_t B = 0; B < nblk; B++) {
        const uint64_t fn = B + 1 < nblk ? F[64 * (uint64_t)(B + 1) + lane] : kK5Esc64;
        const uint64_t c0 = h.len + (uint64_t)B * 64 * K5_S;
        const uint64_t el = E - c0;
        bool fast = false;
        if (h.st == SNAPPY_ST_OK && base < N && el < 64) {
            const uint64_t f = rl64(fr, (uint32_t)el);
            if (f != kK5Esc64 && base + (f >> 8) < N) {
                fast = true;
                if (lane == 0) {
                    BE[B] = E;
                    BB[B] = base;
                }
                base += f >> 8;
                E = c0 + 64 * (uint64_t)K5_S + (f & 0xFF);
            }
        }
        if (!fast) {
            if (lane == 0) BE[B] = K5_SKIP;
            lookups = 0;
            const uint32_t cb = 64 * B, ce = cb + 64 < nchunks ? cb + 64 : nchunks;
            if (demand) {
                for (uint32_t c = cb; c < ce;) {
                    // chunks the chain jumps over (entry past their end) are skipped at once
                    const uint64_t cc0 = h.len + (uint64_t)c * K5_S;
                    if (h.st == SNAPPY_ST_OK && base < N && E >= cc0 + K5_S && E < clen) {
                        const uint64_t cj = (E - h.len) / K5_S;
                        const uint32_t cn = cj < ce ? (uint32_t)cj : ce;
                        if (c + lane < cn) Ent[c + lane] = K5_SKIP;  // (cn - c <= 64)
                        c = cn;
                        continue;
                    }
                    step(c, [&](uint32_t l, uint64_t &xo, uint64_t &oo) {
                        xo = X[(uint64_t)c * 64 + l];
                        oo = O[(uint64_t)c * 64 + l];
                    });
                    c++;
                }
            } else {
                const uint32_t g0 = B * kGB;
                load(g0, xa, oa);
                for (uint32_t g = g0; g < g0 + kGB; g += 2) {
                    load(g + 1, xb, ob_);
                    run(g, xa, oa);
                    if (g + 2 < g0 + kGB) load(g + 2, xa, oa);
                    run(g + 1, xb, ob_);
                }
            }
            demand = lookups < kDemand;
        }
        fr = fn;
    }
    if (lane == 0) {
        result[0] = h.st;
        result[1] = (int64_t)N;
        result[2] = (int64_t)base;  // output the chain accounts for (== N for a whole stream)
    }
}

// K5b3: the chunks of every composed block get their entry and base by
// following the block's entry through the 64 entry maps (one readlane each)
__global__ __launch_bounds__(64) void k5b3_fill(const uint8_t *__restrict__ comp, uint64_t clen,
                                                const uint32_t *__restrict__ P, uint32_t nchunks,
                                                const uint64_t *__restrict__ BE, const uint64_t *__restrict__ BB,
                                                uint64_t *__restrict__ Ent, uint64_t *__restrict__ Base)
{
    const uint32_t lane = threadIdx.x;
    const uint32_t B = blockIdx.x;
    const uint64_t e0 = BE[B];
    if (e0 == K5_SKIP) return;  // K5b2 wrote this block chunk by chunk
    const K5Hdr h = k5_header(comp, clen);
    uint32_t row[64];
#pragma unroll
    for (uint32_t j = 0; j < 64; j++) row[j] = P[(uint64_t)(64 * B + j) * 64 + lane];  // composed: 64 full chunks
    const uint64_t c0 = h.len + (uint64_t)B * 64 * K5_S;
    uint32_t el = (uint32_t)(e0 - c0);
    uint64_t base = BB[B], my_e = 0, my_b = 0;
#pragma unroll
    for (uint32_t j = 0; j < 64; j++) {
        if (lane == j) {
            my_e = c0 + (uint64_t)j * K5_S + el;
            my_b = base;
        }
        const uint32_t w = __builtin_amdgcn_readlane(row[j], el);
        base += w >> 8;
        el = w & 0xFF;
    }
    Ent[64 * (uint64_t)B + lane] = my_e;
    Base[64 * (uint64_t)B + lane] = my_b;
}
#endif

#if SNAPPY_TU_DECODE
__global__ __launch_bounds__(64) void k5c_mark(const uint8_t *__restrict__ comp, uint64_t clen,
                                               const uint64_t *__restrict__ Ent, const uint64_t *__restrict__ Base,
                                               uint64_t *__restrict__ offsets, uint64_t max_units,
                                               int32_t *__restrict__ cst, uint64_t *__restrict__ fin)
{
    __shared__ uint32_t img[(K5_WIN ? K5_WIN + 128 : K5_IMG) / 4 + 4];
    const uint32_t lane = threadIdx.x;
    const uint32_t c = blockIdx.x;
    const K5Hdr h = k5_header(comp, clen);
    int32_t st = SNAPPY_ST_OK;
    uint64_t x = Ent[c];
    if (x != K5_SKIP) {
        const uint64_t N = h.N;
        const uint64_t units = (N + SNAPPY_BLOCK - 1) / SNAPPY_BLOCK;
        const uint64_t c0 = h.len + (uint64_t)c * K5_S;
        const uint32_t end_rel = (uint32_t)(c0 + K5_S < clen ? K5_S : clen - c0);
        uint64_t op = Base[c], xr = x - c0, ia;
        if constexpr (K5_WIN > 0) {
            ia = x & ~3ull;  // from the true entry on
            k5_stage_at<K5_WIN + 128>(comp, clen, ia, img, lane);
        } else {
            ia = c0 & ~3ull;
            k5_stage(comp, clen, c0, img, lane);
        }
        k5_chain<true, K5_WIN>(comp, img, ia, c0, clen, end_rel, xr, op, N, offsets, max_units, st, lane);
        x = c0 + xr;
        if (st == SNAPPY_ST_OK && op == N && lane == 0) {
            if (units < max_units) offsets[units] = x;
            *fin = x;
        }
        if (st == SNAPPY_ST_OK && op < N && x >= clen) st = SNAPPY_ST_TRUNCATED;
    }
    if (lane == 0) cst[c] = st;
}
#endif

#if SNAPPY_TU_DECODE
__global__ __launch_bounds__(64) void k5d_result(uint32_t nchunks, const int32_t *__restrict__ cst,
                                                 int64_t *__restrict__ result, uint64_t *__restrict__ offsets,
                                                 uint64_t max_units)
{
    const uint32_t lane = threadIdx.x;
    int64_t st = result[0];
    const uint64_t N = (uint64_t)result[1];
    const uint64_t units = (N + SNAPPY_BLOCK - 1) / SNAPPY_BLOCK;
    if (st == SNAPPY_ST_OK && units >= max_units) st = SNAPPY_ST_CAPACITY;  // units + 1 entries needed
    for (uint32_t cb = 0; st == SNAPPY_ST_OK && cb < nchunks; cb += 64) {
        const int32_t v = cb + lane < nchunks ? cst[cb + lane] : 0;
        const uint64_t m = __ballot(v != SNAPPY_ST_OK);
        if (m) st = __builtin_amdgcn_readlane(v, (uint32_t)__builtin_ctzll(m));
    }
    if (st == SNAPPY_ST_OK && (uint64_t)result[2] < N) st = SNAPPY_ST_TRUNCATED;
    if (lane == 0) {
        if (st == SNAPPY_ST_OK && units) offsets[0] = 0;
        result[0] = st;
        result[2] = (int64_t)units;
    }
}
#endif

}  // namespace snappy_amd

// The knobs this object was built with (snappy_amd_build_config in
// snappy_device.hip joins the two halves): measurement = a build that may write
// wrong output or carries statistics / timestamp code, 0 for the product.
#define CFG_STR2(x) #x
#define CFG_STR(x) CFG_STR2(x)
#if defined(SNAPPY_MEASUREMENT_BUILD) || defined(SNAPPY_K4_NOFAR) || (defined(SNAPPY_K2_NOLIT) && SNAPPY_K2_NOLIT) || \
    defined(SNAPPY_K1R_STATS) || defined(SNAPPY_K1R_LSTAMPS) || defined(SNAPPY_K1R_RSTAMPS) || defined(SNAPPY_K4_STATS)
#define CFG_MEASURE "1"
#else
#define CFG_MEASURE "0"
#endif
#if SNAPPY_TU_COMPRESS
extern "C" __attribute__((visibility("hidden"))) const char *snappy_amd_config_compress(void)
{
    return "compress{measurement=" CFG_MEASURE " k1r_dmax=" CFG_STR(SNAPPY_K1R_DMAX) " k1r_dmax64=" CFG_STR(
        SNAPPY_K1R_DMAX64) " k1r_rmin=" CFG_STR(SNAPPY_K1R_RMIN) " k1r_pad32=" CFG_STR(SNAPPY_K1R_PAD32) " k1r_pad64=" CFG_STR(SNAPPY_K1R_PAD64)
#if K1R_ASM_ROUNDS
           " k1r_asm=1"
#else
           " k1r_asm=0"
#endif
           " k2_nolit=" CFG_STR(SNAPPY_K2_NOLIT) " k2_pass=" CFG_STR(SNAPPY_K2_PASS) "}";
}
#endif
#if SNAPPY_TU_DECODE
extern "C" __attribute__((visibility("hidden"))) const char *snappy_amd_config_decode(void)
{
    return "decode{measurement=" CFG_MEASURE
#ifdef SNAPPY_K4_NOFAR
           " k4_nofar=1"
#else
           " k4_nofar=0"
#endif
           "}";
}
#endif

#if defined(SNAPPY_K4_STATS) && SNAPPY_TU_DECODE
extern "C" int snappy_amd_debug_k4_stats(uint64_t *host, size_t count)
{
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(snappy_amd::g_k4_stats), count * sizeof(uint64_t), 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -7;
}
#endif
