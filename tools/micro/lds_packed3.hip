// Packed 3-byte LDS records (u16 position + u8 tag at byte 3*slot): unaligned
// ds_write_b16 + ds_write_b8_d16_hi from 64 lanes with shared slots -- does the
// highest lane win both parts of a slot?  And ds_read_b32 at 3*slot reads
// position | tag << 16 (+ the next record's first byte)?
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(64) void k(const uint32_t *slots, uint32_t *out)
{
    __shared__ __attribute__((aligned(16))) uint8_t t[3 * 64 + 4];
    const uint32_t lane = threadIdx.x;
    for (uint32_t i = lane; i < sizeof(t); i += 64) t[i] = 0;
    __syncthreads();
    const uint32_t s = slots[lane];
    const uint32_t word = (0x1000u + lane * 0x101u) | ((0x80u + lane) << 16);  // pos | tag << 16
    const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t *)t;
    const uint32_t a = base + 3 * s;
    asm volatile("ds_write_b16 %0, %1\n\tds_write_b8_d16_hi %0, %1 offset:2\n\ts_waitcnt lgkmcnt(0)" ::"v"(a), "v"(word)
                 : "memory");
    __syncthreads();
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(base + 3 * lane) : "memory");
    out[lane] = v & 0xFFFFFF;
    // ds_bpermute with addresses past 255: does the lane index wrap (addr[7:2])?
    const uint32_t bp = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4 * lane + 256 * (lane & 3) + 4), (int)(lane * 3 + 1));
    out[64 + lane] = bp;
}

int main()
{
    uint32_t hs[64], h[128];
    for (int l = 0; l < 64; l++) hs[l] = (l * 37 + (l >> 3)) % 23;  // collisions, mixed parity
    uint32_t *ds, *d;
    (void)hipMalloc(&ds, sizeof(hs));
    (void)hipMalloc(&d, sizeof(h));
    (void)hipMemcpy(ds, hs, sizeof(hs), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, ds, d);
    hipError_t e = hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int bad = 0;
    for (uint32_t slot = 0; slot < 64; slot++) {
        int win = -1;
        for (int l = 0; l < 64; l++)
            if (hs[l] == slot) win = l;
        const uint32_t want = win < 0 ? 0 : ((0x1000u + win * 0x101u) & 0xFFFF) | ((0x80u + win) << 16);
        if (h[slot] != want) {
            if (bad < 8) printf("slot %u: got %06x want %06x (highest lane %d)\n", slot, h[slot], want, win);
            bad++;
        }
    }
    printf("hip %d; packed 3-byte records, highest lane wins: %s (%d bad slots)\n", (int)e, bad ? "WRONG" : "ok", bad);
    int wrap = 0, other = 0;
    for (uint32_t l = 0; l < 64; l++) {
        if (h[64 + l] == ((l + 1) & 63) * 3 + 1) wrap++;
        else other++;
    }
    printf("ds_bpermute address >= 256: %d lanes wrap to addr[7:2], %d lanes differ (lane 1: %u)\n", wrap, other, h[65]);
    return 0;
}
