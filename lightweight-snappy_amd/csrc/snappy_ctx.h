// snappy_ctx.h -- the device context shared by the HIP shim
// (snappy_device.hip: contexts, kernel launches, copies, status) and the host
// pipelines built on it (snappy_pipeline.cpp: pooled host contexts, the FILE*
// and host-buffer pipelines, several devices).  Private: not part of the C ABI.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

#include "snappy_amd.h"

struct snappy_amd_ctx {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    uint32_t *sizes = nullptr;
    size_t sizes_cap = 0;
    void *tokens = nullptr;         // K1r tokens (uint2 words) + escapes
    size_t tokens_cap = 0;
    uint32_t *ntok = nullptr;
    size_t ntok_cap = 0;
    uint32_t *seg_off = nullptr;    // K2 segments: (output offset in the unit, input position) pairs
    size_t seg_off_cap = 0;
    int32_t *status = nullptr;
    size_t status_cap = 0;
    uint64_t *total = nullptr;      // device u64
    int64_t *k5res = nullptr;       // device i64[3]
    uint64_t *h_total = nullptr;    // pinned
    int32_t *h_status = nullptr;    // pinned, grows with status_cap
    size_t h_status_cap = 0;
    size_t last_units = 0;
    bool status_pending = false;    // the last decode's status words not read back yet
    int last_status = 0;            // its result once read (decompress_status returns it again)
    int last_layout = SNAPPY_AMD_SINGLE;  // of the last decode launch (status mapping)
    // host-buffer path staging
    uint8_t *d_a = nullptr; size_t d_a_cap = 0;
    uint8_t *d_b = nullptr; size_t d_b_cap = 0;
    uint64_t *d_idx = nullptr; size_t d_idx_cap = 0;
    uint8_t *k5buf = nullptr; size_t k5buf_cap = 0;  // chunk-parallel index scratch
    uint8_t *k5copy = nullptr; size_t k5copy_cap = 0;  // aligned copy of a misaligned stream
    bool timing = false;
    bool serial_index = false;  // SNAPPY_AMD_OPT_SERIAL_INDEX
    uint32_t k1r_extra_lds = 0; // SNAPPY_AMD_OPT_K1R_EXTRA_LDS
    hipEvent_t ev[5] = {};
    bool ev_compress = false, ev_decode = false;  // ev[0..2] / ev[3..4] recorded by a launch
    float k1_ms = 0, k3_ms = 0, k4_ms = 0;
};

#define HIP_OK(expr) do { if ((expr) != hipSuccess) return SNAPPY_AMD_ERR_DEVICE; } while (0)

#define SNAPPY_PRIVATE __attribute__((visibility("hidden")))

// grow a device buffer to at least `need` bytes (contents not kept); the slack
// is capped (dist.py's _grown mirrors it for bench.py's memory plan)
SNAPPY_PRIVATE int grow(void **ptr, size_t *cap, size_t need);
// c->stream, creating the context's own stream if none is bound and none was
// made yet (contexts create it lazily: a caller-bound stream leaves no idle one)
SNAPPY_PRIVATE int ctx_stream(snappy_amd_ctx *c);
// K1r (or K1r64) -> K3 -> K2 on c->stream; *out_len (when non-null) after a
// sync of that stream, otherwise the size stays in c->total (device)
extern "C" SNAPPY_PRIVATE int compress_impl(snappy_amd_ctx *c, const void *d_in, size_t n, uint32_t chunk, int layout,
                                 uint32_t flags, uint64_t header_value, void *d_out, uint64_t *d_offsets,
                                 size_t *out_len);
