// Does s_set_gpr_idx_on (SRC0) index a 64-bit v_mov_b64 source pair on gfx950?
// v[2+i] = 1000*i + lane; v_mov_b64 of v[2+idx : 3+idx] must give (1000*idx + lane, 1000*(idx+1) + lane).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef uint32_t v32 __attribute__((ext_vector_type(32)));

__global__ __launch_bounds__(64) void k(const uint32_t *sel, uint64_t *out)
{
    const uint32_t lane = threadIdx.x;
    v32 g;
    for (int i = 0; i < 32; i++) g[i] = 1000u * i + lane + sel[64 + i];  // sel[64..95] = 0 (defeats folding)
    for (uint32_t j = 0; j < 31; j++) {
        const uint32_t idx = __builtin_amdgcn_readfirstlane(sel[j]);
        uint64_t v;
        asm volatile("s_set_gpr_idx_on %1, gpr_idx(SRC0)\n\tv_mov_b64 %0, v[2:3]\n\ts_set_gpr_idx_off"
                     : "=&v"(v)
                     : "s"(idx), "{v[2:33]}"(g));
        out[j * 64 + lane] = v;
    }
}

int main()
{
    std::vector<uint32_t> hs(96, 0);
    for (uint32_t j = 0; j < 31; j++) hs[j] = j;
    uint32_t *ds;
    uint64_t *d;
    (void)hipMalloc(&ds, 96 * 4);
    (void)hipMalloc(&d, 31 * 64 * 8);
    (void)hipMemcpy(ds, hs.data(), 96 * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, ds, d);
    std::vector<uint64_t> h(31 * 64);
    (void)hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    int bad = 0;
    for (uint32_t j = 0; j < 31; j++)
        for (uint32_t l = 0; l < 64; l++) {
            const uint64_t want = (uint64_t)(1000u * j + l) | ((uint64_t)(1000u * (j + 1) + l) << 32);
            if (h[j * 64 + l] != want) {
                if (bad < 5) printf("idx %u lane %u got %llx want %llx\n", j, l, (unsigned long long)h[j * 64 + l], (unsigned long long)want);
                bad++;
            }
        }
    printf("v_mov_b64 gpr_idx: %s (%d mismatches)\n", bad ? "NO" : "yes", bad);
    return 0;
}
