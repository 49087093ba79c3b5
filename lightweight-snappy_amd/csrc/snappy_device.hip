// snappy_device.hip -- the thin extern "C" shim between the host code and
// the gfx950 kernels: device contexts and their scratch, the launch stream,
// HIP events, the launch geometry and the status read-back.  Declared in
// include/snappy_amd.h (device batch API).  The host pipelines (host-buffer,
// FILE*, several devices) are host C++ in snappy_pipeline.cpp; the reference's
// FILE* API is the C layer in snappy_host.c.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "snappy_amd.h"
#include "snappy_ctx.h"
#include "snappy_kernels.h"

using namespace snappy_amd;

int grow(void **ptr, size_t *cap, size_t need)
{
    if (need <= *cap) return SNAPPY_AMD_OK;
    if (*ptr) (void)hipFree(*ptr);
    *ptr = nullptr;
    *cap = 0;
    // slack for slowly growing calls, capped: a 16 GiB piece's token scratch
    // must not carry 4 GB of slack (bench.py's per-rank memory plan counts it)
    const size_t slack = need / 8 < ((size_t)64 << 20) ? need / 8 : ((size_t)64 << 20);
    size_t want = need + slack + 4096;
    if (hipMalloc(ptr, want) != hipSuccess) { *ptr = nullptr; return SNAPPY_AMD_ERR_DEVICE; }
    *cap = want;
    return SNAPPY_AMD_OK;
}

int ctx_stream(snappy_amd_ctx *c)
{
    if (c->stream) return SNAPPY_AMD_OK;
    // a blocking stream: work a caller queued on the legacy default stream (torch's
    // default stream, cuda_stream == 0, which set_stream(NULL) maps here) is
    // ordered before the context's launches (a non-blocking own stream raced it)
    if (!c->own) {
        HIP_OK(hipSetDevice(c->device));
        HIP_OK(hipStreamCreateWithFlags(&c->own, hipStreamDefault));
    }
    c->stream = c->own;
    return SNAPPY_AMD_OK;
}

extern "C" {

const char *snappy_amd_config_compress(void);
const char *snappy_amd_config_decode(void);

const char *snappy_amd_build_config(void)
{
    static char cfg[512];
    static int made = 0;
    if (!made) {  // (the same bytes from every thread that races here)
        snprintf(cfg, sizeof cfg, "%s %s", snappy_amd_config_compress(), snappy_amd_config_decode());
        made = 1;
    }
    return cfg;
}

int snappy_amd_create(int device, snappy_amd_ctx **out)
{
    if (!out) return SNAPPY_AMD_ERR_ARG;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0 || device < 0 || device >= count)
        return SNAPPY_AMD_ERR_DEVICE;
    HIP_OK(hipSetDevice(device));
    snappy_amd_ctx *c = new snappy_amd_ctx();
    c->device = device;
    // the context's own stream is created on first use (ctx_stream), so a context
    // whose caller binds a stream of its own never holds an idle one (DESIGN.md 6:
    // the streams of a rank at N > 1 against GPU_MAX_HW_QUEUES)
    if (hipMalloc(&c->total, 64) != hipSuccess || hipMalloc(&c->k5res, 64) != hipSuccess ||
        hipHostMalloc(&c->h_total, 64, hipHostMallocDefault) != hipSuccess) {
        snappy_amd_destroy(c);
        return SNAPPY_AMD_ERR_DEVICE;
    }
    for (int i = 0; i < 5; i++) (void)hipEventCreate(&c->ev[i]);
    *out = c;
    return SNAPPY_AMD_OK;
}

void snappy_amd_destroy(snappy_amd_ctx *c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    void *bufs[] = {c->sizes, c->tokens, c->ntok, c->seg_off, c->status, c->total, c->k5res,
                    c->d_a, c->d_b, c->d_idx, c->k5buf, c->k5copy};
    for (void *b : bufs) if (b) (void)hipFree(b);
    if (c->h_total) (void)hipHostFree(c->h_total);
    if (c->h_status) (void)hipHostFree(c->h_status);
    for (int i = 0; i < 5; i++) if (c->ev[i]) (void)hipEventDestroy(c->ev[i]);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
}

size_t snappy_amd_device_bytes(snappy_amd_ctx *c)
{
    if (!c) return 0;
    return c->sizes_cap + c->tokens_cap + c->ntok_cap + c->seg_off_cap + c->status_cap + c->d_a_cap + c->d_b_cap +
           c->d_idx_cap + c->k5buf_cap + c->k5copy_cap + 128;
}

int snappy_amd_trim(snappy_amd_ctx *c)
{
    if (!c) return SNAPPY_AMD_ERR_ARG;
    HIP_OK(hipSetDevice(c->device));
    if (c->stream) HIP_OK(hipStreamSynchronize(c->stream));
    struct { void **p; size_t *cap; } bufs[] = {
        {reinterpret_cast<void **>(&c->tokens), &c->tokens_cap}, {reinterpret_cast<void **>(&c->seg_off), &c->seg_off_cap},
        {reinterpret_cast<void **>(&c->ntok), &c->ntok_cap}, {reinterpret_cast<void **>(&c->sizes), &c->sizes_cap},
        {reinterpret_cast<void **>(&c->d_a), &c->d_a_cap}, {reinterpret_cast<void **>(&c->d_b), &c->d_b_cap},
        {reinterpret_cast<void **>(&c->d_idx), &c->d_idx_cap}, {reinterpret_cast<void **>(&c->k5buf), &c->k5buf_cap},
        {reinterpret_cast<void **>(&c->k5copy), &c->k5copy_cap},
        // a decode's status words only once its status has been read (the result is kept)
        {reinterpret_cast<void **>(&c->status), c->status_pending ? nullptr : &c->status_cap}};
    for (auto &b : bufs) {
        if (!b.cap) continue;
        if (*b.p) (void)hipFree(*b.p);
        *b.p = nullptr;
        *b.cap = 0;
    }
    if (!c->status_pending && c->h_status) {
        (void)hipHostFree(c->h_status);
        c->h_status = nullptr;
        c->h_status_cap = 0;
    }
    return SNAPPY_AMD_OK;
}

int snappy_amd_set_option(snappy_amd_ctx *c, int option, int64_t value)
{
    if (!c) return SNAPPY_AMD_ERR_ARG;
    switch (option) {
    case SNAPPY_AMD_OPT_SERIAL_INDEX: c->serial_index = value != 0; return SNAPPY_AMD_OK;
    case SNAPPY_AMD_OPT_K1R_EXTRA_LDS:
        if (value < 0 || value > 65536) return SNAPPY_AMD_ERR_ARG;
        c->k1r_extra_lds = (uint32_t)value;
        return SNAPPY_AMD_OK;
    default: return SNAPPY_AMD_ERR_ARG;
    }
}

int snappy_amd_set_stream(snappy_amd_ctx *c, void *s)
{
    if (!c) return SNAPPY_AMD_ERR_ARG;
    c->stream = s ? static_cast<hipStream_t>(s) : c->own;  // (own: created at the next use if none yet)
    return SNAPPY_AMD_OK;
}

void *snappy_amd_get_stream(snappy_amd_ctx *c) { return c && ctx_stream(c) == SNAPPY_AMD_OK ? c->stream : nullptr; }

int snappy_amd_enable_timing(snappy_amd_ctx *c, int on)
{
    if (!c) return SNAPPY_AMD_ERR_ARG;
    c->timing = on != 0;
    return SNAPPY_AMD_OK;
}

int snappy_amd_last_timings(snappy_amd_ctx *c, float *k1, float *k3, float *k4)
{
    if (!c) return SNAPPY_AMD_ERR_ARG;
    if (c->timing) {
        // resolve whatever the stream has recorded so far (waits for it)
        // (only events a launch recorded: an elapsed time of an unrecorded event
        // fails, and its error would stay pending for the thread's next check)
        (void)hipSetDevice(c->device);
        if (c->ev_compress && hipEventSynchronize(c->ev[2]) == hipSuccess) {
            (void)hipEventElapsedTime(&c->k1_ms, c->ev[0], c->ev[1]);
            (void)hipEventElapsedTime(&c->k3_ms, c->ev[1], c->ev[2]);
        }
        if (c->ev_decode && c->last_units && hipEventSynchronize(c->ev[4]) == hipSuccess)
            (void)hipEventElapsedTime(&c->k4_ms, c->ev[3], c->ev[4]);
    }
    if (k1) *k1 = c->k1_ms;
    if (k3) *k3 = c->k3_ms;
    if (k4) *k4 = c->k4_ms;
    return SNAPPY_AMD_OK;
}

size_t snappy_amd_num_units(size_t n, uint32_t chunk, int layout)
{
    uint32_t unit = layout == SNAPPY_AMD_SINGLE ? SNAPPY_AMD_BLOCK : chunk;
    if (unit == 0) return 0;
    return (n + unit - 1) / unit;
}

size_t snappy_amd_max_output(size_t n, uint32_t chunk, int layout)
{
    uint32_t unit = layout == SNAPPY_AMD_SINGLE ? SNAPPY_AMD_BLOCK : chunk;
    if (unit == 0) return 0;
    size_t units = (n + unit - 1) / unit;
    return n + units * (unit / 32 + 32) + 16;
}

static uint32_t hdr_mode_of(int layout, uint32_t flags)
{
    if (layout == SNAPPY_AMD_STREAMS) return SNAPPY_HDR_EVERY_UNIT;
    return (flags & SNAPPY_AMD_NO_PREAMBLE) ? SNAPPY_HDR_NONE : SNAPPY_HDR_FIRST_UNIT;
}

int compress_impl(snappy_amd_ctx *c, const void *d_in, size_t n, uint32_t chunk, int layout, uint32_t flags,
                         uint64_t header_value, void *d_out, uint64_t *d_offsets, size_t *out_len)
{
    if (!c || (!d_in && n) || !d_out || !d_offsets) return SNAPPY_AMD_ERR_ARG;
    if (layout != SNAPPY_AMD_SINGLE && layout != SNAPPY_AMD_STREAMS) return SNAPPY_AMD_ERR_ARG;
    const uint32_t unit = layout == SNAPPY_AMD_SINGLE ? SNAPPY_AMD_BLOCK : chunk;
    if (unit == 0 || unit > SNAPPY_AMD_BLOCK) return SNAPPY_AMD_ERR_ARG;
    HIP_OK(hipSetDevice(c->device));
    if (ctx_stream(c)) return SNAPPY_AMD_ERR_DEVICE;
    if (n == 0) {
        // src/snappy_compression.c:417-421: no block, so no header either
        HIP_OK(hipMemsetAsync(d_offsets, 0, sizeof(uint64_t), c->stream));
        if (out_len) *out_len = 0;
        return SNAPPY_AMD_OK;
    }
    const size_t units = (n + unit - 1) / unit;
    int rc;
    // register-resident match finder -> tokens; scan; emit in place
    const uint32_t tok_cap = unit / 4 + 2;
    if ((rc = grow(reinterpret_cast<void **>(&c->tokens), &c->tokens_cap,
                   units * tok_cap * sizeof(uint2) + units * 4 * sizeof(uint64_t))))
        return rc;
    if ((rc = grow(reinterpret_cast<void **>(&c->ntok), &c->ntok_cap, units * sizeof(uint32_t)))) return rc;
    if ((rc = grow(reinterpret_cast<void **>(&c->sizes), &c->sizes_cap, units * sizeof(uint32_t)))) return rc;
    // segments per unit: tokens 0..ntok (the tail literal is token ntok <= tok_cap - 1)
    const uint32_t segs = (tok_cap + SNAPPY_K2_SEG - 1) / SNAPPY_K2_SEG;
    if ((rc = grow(reinterpret_cast<void **>(&c->seg_off), &c->seg_off_cap, units * segs * 2 * sizeof(uint32_t))))
        return rc;
    const uint32_t hm = hdr_mode_of(layout, flags);
    // launch errors are read with hipGetLastError: clear one a runtime call of
    // the caller's (or of another context on this thread) left pending
    (void)hipGetLastError();
    if (c->timing) (void)hipEventRecord(c->ev[0], c->stream);
    // units <= 32 KiB: the unit in 128 VGPRs; 65,536-byte blocks: its last 128
    // segments in a 128-VGPR ring fed by LDS-DMA (both 3 waves/SIMD).
    // Extra dynamic LDS per unit: occupancy experiments only (SNAPPY_AMD_OPT_K1R_EXTRA_LDS)
    const uint32_t dyn_lds = c->k1r_extra_lds;
    if (unit <= SNAPPY_K1R_MAX_UNIT)
        hipLaunchKernelGGL(k1r_match_units, dim3((uint32_t)units), dim3(64), dyn_lds, c->stream,
                           static_cast<const uint8_t *>(d_in), (uint64_t)n, unit, hm, header_value,
                           static_cast<uint2 *>(c->tokens), tok_cap, c->ntok, c->sizes, c->seg_off, segs);
    else
        hipLaunchKernelGGL(k1r_match_units64, dim3((uint32_t)units), dim3(64), 0, c->stream,
                           static_cast<const uint8_t *>(d_in), (uint64_t)n, unit, hm, header_value,
                           static_cast<uint2 *>(c->tokens), tok_cap, c->ntok, c->sizes, c->seg_off, segs);
    HIP_OK(hipGetLastError());
    if (c->timing) (void)hipEventRecord(c->ev[1], c->stream);
    if (units <= SNAPPY_K3_WAVE_MAX)
        hipLaunchKernelGGL(k3_scan_wave, dim3(1), dim3(64), 0, c->stream, c->sizes, (uint64_t)units, d_offsets, c->total);
    else
        hipLaunchKernelGGL(k3_scan, dim3(1), dim3(1024), 0, c->stream, c->sizes, (uint64_t)units, d_offsets, c->total);
    // K1r wrote the sizes and segment offsets; K2: a few waves per unit, each taking
    // every SNAPPY_K2_WAVES-th segment (text fills ~12 segments of 32 KiB units)
    hipLaunchKernelGGL(k2_emit_units, dim3((uint32_t)units, segs < SNAPPY_K2_WAVES ? segs : SNAPPY_K2_WAVES), dim3(64), 0, c->stream,
                       static_cast<const uint8_t *>(d_in), (uint64_t)n, unit, hm, header_value,
                       static_cast<const uint2 *>(c->tokens), tok_cap, c->ntok, c->seg_off, segs, d_offsets,
                       static_cast<uint8_t *>(d_out));
    HIP_OK(hipGetLastError());
    if (c->timing) {
        (void)hipEventRecord(c->ev[2], c->stream);
        c->ev_compress = true;
    }
    if (out_len) {
        HIP_OK(hipMemcpyAsync(c->h_total, c->total, sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
        HIP_OK(hipStreamSynchronize(c->stream));
        *out_len = (size_t)*c->h_total;
        if (c->timing) {
            (void)hipEventElapsedTime(&c->k1_ms, c->ev[0], c->ev[1]);
            (void)hipEventElapsedTime(&c->k3_ms, c->ev[1], c->ev[2]);
        }
    }
    return SNAPPY_AMD_OK;
}

int snappy_amd_compress_device(snappy_amd_ctx *c, const void *d_in, size_t n, uint32_t chunk, int layout, void *d_out,
                               uint64_t *d_offsets, size_t *out_len)
{
    return compress_impl(c, d_in, n, chunk, layout, 0, (uint64_t)n, d_out, d_offsets, out_len);
}

int snappy_amd_compress_device_ex(snappy_amd_ctx *c, const void *d_in, size_t n, uint32_t chunk, int layout,
                                  uint32_t flags, uint64_t header_value, void *d_out, uint64_t *d_offsets,
                                  size_t *out_len)
{
    return compress_impl(c, d_in, n, chunk, layout, flags, header_value, d_out, d_offsets, out_len);
}

static int decompress_launch(snappy_amd_ctx *c, const void *d_comp, const uint64_t *d_offsets, size_t n,
                             uint32_t chunk, int layout, uint32_t flags, uint64_t header_value, void *d_out)
{
    if (!c || !d_comp || !d_offsets || (!d_out && n)) return SNAPPY_AMD_ERR_ARG;
    if (layout != SNAPPY_AMD_SINGLE && layout != SNAPPY_AMD_STREAMS) return SNAPPY_AMD_ERR_ARG;
    const uint32_t unit = layout == SNAPPY_AMD_SINGLE ? SNAPPY_AMD_BLOCK : chunk;
    if (unit == 0 || unit > SNAPPY_AMD_BLOCK) return SNAPPY_AMD_ERR_ARG;
    HIP_OK(hipSetDevice(c->device));
    if (ctx_stream(c)) return SNAPPY_AMD_ERR_DEVICE;
    c->last_units = 0;
    c->status_pending = false;
    c->last_status = SNAPPY_AMD_OK;
    if (n == 0) return SNAPPY_AMD_OK;
    const size_t units = (n + unit - 1) / unit;
    if (units > 0xFFFFFFFFull) return SNAPPY_AMD_ERR_ARG;
    int rc;
    // status: one word per unit + pass 2's ticket counter and defer flag
    if ((rc = grow(reinterpret_cast<void **>(&c->status), &c->status_cap, (units + 2) * sizeof(int32_t)))) return rc;
    // one whole stream (SINGLE): elements may straddle blocks and copies may
    // reach into earlier blocks (src/snappy_decompression.c:253-280, 345-363);
    // pass 1 decodes every self-contained block, pass 2 the others in order
    const uint32_t allow_back = layout == SNAPPY_AMD_SINGLE ? 1u : 0u;
    (void)hipGetLastError();  // (a pending error that is not this launch's, as in compress_impl)
    if (c->timing) (void)hipEventRecord(c->ev[3], c->stream);
    if (allow_back) HIP_OK(hipMemsetAsync(c->status + units, 0, 2 * sizeof(int32_t), c->stream));
    const uint32_t hm = hdr_mode_of(layout, flags);
    // the kernel reads aligned dwords: pass the stream as an aligned base + bias
    const uint32_t bias = (uint32_t)(reinterpret_cast<uintptr_t>(d_comp) & 3);
    const uint8_t *comp = static_cast<const uint8_t *>(d_comp) - bias;
    hipLaunchKernelGGL(k4_decompress_units, dim3((uint32_t)units), dim3(64), 0, c->stream, comp, d_offsets,
                       (uint64_t)n, unit, hm, header_value, allow_back, bias, static_cast<uint8_t *>(d_out),
                       c->status);
    HIP_OK(hipGetLastError());
    if (allow_back) {
        hipLaunchKernelGGL(k4_decompress_back, dim3((uint32_t)units), dim3(64), 0, c->stream, comp,
                           d_offsets, (uint64_t)n, unit, hm, header_value, bias, static_cast<uint8_t *>(d_out),
                           c->status);
        HIP_OK(hipGetLastError());
    }
    if (c->timing) {
        (void)hipEventRecord(c->ev[4], c->stream);
        c->ev_decode = true;
    }
    c->last_units = units;
    c->last_layout = layout;
    c->status_pending = true;
    return SNAPPY_AMD_OK;
}

int snappy_amd_decompress_status(snappy_amd_ctx *c)
{
    if (!c) return SNAPPY_AMD_ERR_ARG;
    if (!c->status_pending) return c->last_status;  // (read before, or no decode since)
    HIP_OK(hipSetDevice(c->device));
    const size_t bytes = c->last_units * sizeof(int32_t);
    if (bytes > c->h_status_cap) {
        if (c->h_status) (void)hipHostFree(c->h_status);
        c->h_status = nullptr;
        c->h_status_cap = 0;
        HIP_OK(hipHostMalloc(&c->h_status, bytes, hipHostMallocDefault));
        c->h_status_cap = bytes;
    }
    HIP_OK(hipMemcpyAsync(c->h_status, c->status, bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    if (c->timing && c->ev_decode) (void)hipEventElapsedTime(&c->k4_ms, c->ev[3], c->ev[4]);
    int r = SNAPPY_AMD_OK;
    for (size_t i = 0; i < c->last_units && r == SNAPPY_AMD_OK; i++) {
        // DEFER survives a STREAMS launch (no pass 2) only for a copy reaching
        // before the start of its own stream; after a SINGLE launch pass 2 ends
        // every deferred unit, so a DEFER left over is an internal failure
        if (c->h_status[i] > 0) r = c->last_layout == SNAPPY_AMD_STREAMS ? SNAPPY_AMD_ERR_OFFSET : SNAPPY_AMD_ERR_DEVICE;
        else if (c->h_status[i] != SNAPPY_ST_OK) r = c->h_status[i];
    }
    c->last_status = r;
    c->status_pending = false;
    return r;
}

int snappy_amd_decompress_device_async(snappy_amd_ctx *c, const void *d_comp, const uint64_t *d_offsets, size_t n,
                                       uint32_t chunk, int layout, void *d_out)
{
    return decompress_launch(c, d_comp, d_offsets, n, chunk, layout, 0, (uint64_t)n, d_out);
}

int snappy_amd_decompress_device_ex(snappy_amd_ctx *c, const void *d_comp, const uint64_t *d_offsets, size_t n,
                                    uint32_t chunk, int layout, uint32_t flags, uint64_t header_value, void *d_out,
                                    int sync)
{
    int rc = decompress_launch(c, d_comp, d_offsets, n, chunk, layout, flags, header_value, d_out);
    if (rc || !sync) return rc;
    return snappy_amd_decompress_status(c);
}

int snappy_amd_decompress_device(snappy_amd_ctx *c, const void *d_comp, const uint64_t *d_offsets, size_t n,
                                 uint32_t chunk, int layout, void *d_out)
{
    int rc = decompress_launch(c, d_comp, d_offsets, n, chunk, layout, 0, (uint64_t)n, d_out);
    if (rc) return rc;
    return snappy_amd_decompress_status(c);
}

int snappy_amd_index_device(snappy_amd_ctx *c, const void *d_comp, size_t clen, uint64_t *d_offsets, size_t max_units,
                            size_t *n_out)
{
    if (!c || !d_comp || !d_offsets) return SNAPPY_AMD_ERR_ARG;
    HIP_OK(hipSetDevice(c->device));
    if (ctx_stream(c)) return SNAPPY_AMD_ERR_DEVICE;
    (void)hipGetLastError();  // (a pending error that is not this launch's, as in compress_impl)
    const uint8_t *comp = static_cast<const uint8_t *>(d_comp);
    const bool serial = c->serial_index;
    if (!serial && clen >= 4 * (size_t)K5_CHUNK && (reinterpret_cast<uintptr_t>(d_comp) & 3)) {
        // K5p stages 4-aligned dwords of the stream: a stream at an odd address
        // is first moved to an aligned scratch copy (one HBM pass, a few % of
        // the index time) instead of falling back to the one-wave serial walk;
        // the index entries are stream-relative, so they are the same
        int rc = grow(reinterpret_cast<void **>(&c->k5copy), &c->k5copy_cap, clen + 16);
        if (rc) return rc;
        HIP_OK(hipMemcpyAsync(c->k5copy, d_comp, clen, hipMemcpyDeviceToDevice, c->stream));
        comp = c->k5copy;
    }
    if (serial || clen < 4 * (size_t)K5_CHUNK) {
        hipLaunchKernelGGL(k5_index_stream, dim3(1), dim3(64), 0, c->stream, comp, (uint64_t)clen, d_offsets,
                           (uint64_t)max_units, c->k5res);
    } else {
        // chunk-parallel walk (K5a..K5d); chunk c covers [hdr + c*K5_CHUNK, +K5_CHUNK)
        const uint32_t nch = (uint32_t)((clen + K5_CHUNK - 1) / K5_CHUNK);
        // per chunk: X, O (u64 x 64), P (u32 x 64), Ent, Base, status; per 64-chunk
        // block: F (u64 x 64), BE, BB
        const uint32_t nblk = (nch + 63) / 64;
        const size_t per = 2 * 64 * 8 + 64 * 4 + 2 * 8 + 4;
        int rc = grow(reinterpret_cast<void **>(&c->k5buf), &c->k5buf_cap, per * nch + (64 * 8 + 16) * (size_t)nblk + 128);
        if (rc) return rc;
        uint64_t *X = reinterpret_cast<uint64_t *>(c->k5buf);
        uint64_t *O = X + 64 * (size_t)nch, *Ent = O + 64 * (size_t)nch, *Base = Ent + nch, *fin = Base + nch;
        uint64_t *F = fin + 8, *BE = F + 64 * (size_t)nblk, *BB = BE + nblk;
        int32_t *cst = reinterpret_cast<int32_t *>(BB + nblk);
        uint32_t *P = reinterpret_cast<uint32_t *>(cst + nch);
        hipLaunchKernelGGL(k5a_chunk_walk, dim3(nch), dim3(64), 0, c->stream, comp, (uint64_t)clen, X, O, P);
        hipLaunchKernelGGL(k5b1_compose, dim3(nblk), dim3(64), 0, c->stream, (const uint32_t *)P, nch, F);
        hipLaunchKernelGGL(k5b_carry, dim3(1), dim3(64), 0, c->stream, comp, (uint64_t)clen, nch, X, O,
                           (const uint64_t *)F, BE, BB, Ent, Base, c->k5res);
        hipLaunchKernelGGL(k5b3_fill, dim3(nblk), dim3(64), 0, c->stream, comp, (uint64_t)clen, (const uint32_t *)P,
                           nch, (const uint64_t *)BE, (const uint64_t *)BB, Ent, Base);
        hipLaunchKernelGGL(k5c_mark, dim3(nch), dim3(64), 0, c->stream, comp, (uint64_t)clen, Ent, Base, d_offsets,
                           (uint64_t)max_units, cst, fin);
        hipLaunchKernelGGL(k5d_result, dim3(1), dim3(64), 0, c->stream, nch, cst, c->k5res, d_offsets,
                           (uint64_t)max_units);
    }
    HIP_OK(hipGetLastError());
    int64_t res[3];
    HIP_OK(hipMemcpyAsync(res, c->k5res, sizeof(res), hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    if (n_out) *n_out = (size_t)res[1];
    return (int)res[0];
}

}  // extern "C"
