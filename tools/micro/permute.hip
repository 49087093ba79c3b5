// ds_permute_b32 (forward permute) semantics on gfx950: what do lanes nobody
// writes receive, and who wins when several lanes write the same lane?
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(64) void k(uint32_t *out, uint32_t mode)
{
    const uint32_t lane = threadIdx.x;
    uint32_t addr, data;
    if (mode == 0) {  // lanes 0..9 -> lane 2l (data l+1); lanes >= 10 -> lane 63 (data 100+l)
        addr = lane < 10 ? 2 * lane : 63;
        data = lane < 10 ? lane + 1 : 100 + lane;
    } else {  // every lane -> lane 5, data 100+l
        addr = 5;
        data = 100 + lane;
    }
    const uint32_t r = (uint32_t)__builtin_amdgcn_ds_permute((int)(addr << 2), (int)data);
    out[mode * 64 + lane] = r;
}

int main()
{
    uint32_t *d, h[128];
    (void)hipMalloc(&d, sizeof(h));
    for (uint32_t m = 0; m < 2; m++) hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, m);
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("mode0 (scatter 0..9 -> 2l, rest -> 63):");
    for (int l = 0; l < 64; l++) printf(" %u", h[l]);
    printf("\nmode1 (all -> lane 5): lane5=%u lane0=%u lane6=%u\n", h[64 + 5], h[64], h[64 + 6]);
    return 0;
}
