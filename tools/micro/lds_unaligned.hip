// Unaligned LDS dword/qword access on gfx950 (ds_read_b32 / ds_write_b32 at byte
// offsets 1..3): correct data? (SH_MEM_CONFIG alignment mode is the driver's choice)
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(64) void k(uint32_t *out)
{
    __shared__ __attribute__((aligned(16))) uint8_t b[1024];
    const uint32_t lane = threadIdx.x;
    for (uint32_t i = lane; i < 1024; i += 64) b[i] = (uint8_t)(i * 7 + 1);
    __syncthreads();
    // unaligned read of 4 bytes at 4*lane + 1
    const uint32_t a = 4 * lane + 1;
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
    out[lane] = v;
    __syncthreads();
    // unaligned write of 0xAABBCCDD at 8*lane + 515 (disjoint), then byte readback
    const uint32_t w = 8 * lane + 515;
    asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(w), "v"(0xAABBCCDDu) : "memory");
    __syncthreads();
    out[64 + lane] = (uint32_t)b[w] | ((uint32_t)b[w + 1] << 8) | ((uint32_t)b[w + 2] << 16) | ((uint32_t)b[w + 3] << 24);
}

int main()
{
    uint32_t *d, h[128];
    (void)hipMalloc(&d, sizeof(h));
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    hipError_t e = hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int bad_r = 0, bad_w = 0;
    for (uint32_t l = 0; l < 64; l++) {
        uint32_t want = 0;
        for (int k = 0; k < 4; k++) want |= (uint32_t)(uint8_t)((4 * l + 1 + k) * 7 + 1) << (8 * k);
        if (h[l] != want) bad_r++;
        if (h[64 + l] != 0xAABBCCDDu) bad_w++;
    }
    printf("hip %d; unaligned ds_read_b32: %s (%d bad, lane0 %08x); unaligned ds_write_b32: %s (%d bad, lane0 %08x)\n", (int)e,
           bad_r ? "WRONG" : "ok", bad_r, h[0], bad_w ? "WRONG" : "ok", bad_w, h[64]);
    return 0;
}
