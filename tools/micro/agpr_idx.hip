// Does s_set_gpr_idx_on (SRC0) index AGPRs through v_accvgpr_read_b32 on gfx950?
// a[i] = 1000*i + lane for i < 64; read a[idx] for idx = 0..63 with a uniform
// SGPR index; out[idx*64 + lane] must equal 1000*idx + lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float v64f __attribute__((ext_vector_type(32)));

__global__ __launch_bounds__(64) void k(uint32_t *out)
{
    const uint32_t lane = threadIdx.x;
    // fill a[0..63]
#define W(i) asm volatile("v_accvgpr_write_b32 a" #i ", %0" ::"v"(1000u * i + lane) : "a" #i);
    W(0) W(1) W(2) W(3) W(4) W(5) W(6) W(7) W(8) W(9) W(10) W(11) W(12) W(13) W(14) W(15)
    W(16) W(17) W(18) W(19) W(20) W(21) W(22) W(23) W(24) W(25) W(26) W(27) W(28) W(29) W(30) W(31)
    W(32) W(33) W(34) W(35) W(36) W(37) W(38) W(39) W(40) W(41) W(42) W(43) W(44) W(45) W(46) W(47)
    W(48) W(49) W(50) W(51) W(52) W(53) W(54) W(55) W(56) W(57) W(58) W(59) W(60) W(61) W(62) W(63)
    for (uint32_t idx = 0; idx < 64; idx++) {
        uint32_t v;
        asm volatile("s_set_gpr_idx_on %1, gpr_idx(SRC0)\n\tv_accvgpr_read_b32 %0, a0\n\ts_set_gpr_idx_off"
                     : "=v"(v)
                     : "s"(__builtin_amdgcn_readfirstlane(idx))
                     : "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13",
                       "a14", "a15", "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26",
                       "a27", "a28", "a29", "a30", "a31", "a32", "a33", "a34", "a35", "a36", "a37", "a38", "a39",
                       "a40", "a41", "a42", "a43", "a44", "a45", "a46", "a47", "a48", "a49", "a50", "a51", "a52",
                       "a53", "a54", "a55", "a56", "a57", "a58", "a59", "a60", "a61", "a62", "a63");
        out[idx * 64 + lane] = v;
    }
}

int main()
{
    uint32_t *d;
    (void)hipMalloc(&d, 64 * 64 * 4);
    (void)hipMemset(d, 0xFF, 64 * 64 * 4);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    std::vector<uint32_t> h(64 * 64);
    (void)hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (uint32_t i = 0; i < 64; i++)
        for (uint32_t l = 0; l < 64; l++)
            if (h[i * 64 + l] != 1000u * i + l) {
                if (bad < 5) printf("idx %u lane %u got %u want %u\n", i, l, h[i * 64 + l], 1000u * i + l);
                bad++;
            }
    printf("agpr gpr_idx: %s (%d mismatches)\n", bad ? "NO" : "yes", bad);
    return 0;
}
