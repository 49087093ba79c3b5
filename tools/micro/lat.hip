// Latency microbenchmarks for the K1r probe chain (cycles per dependent step).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef uint32_t v32 __attribute__((ext_vector_type(32)));
#define REG_OF(r) ({ uint32_t _v; asm volatile("s_set_gpr_idx_on %1, gpr_idx(SRC0)\n\tv_mov_b32 %0, v2\n\ts_set_gpr_idx_off" : "=&v"(_v) : "s"((uint32_t)(r)), "{v[2:33]}"(g0), "{v[34:65]}"(g1), "{v[66:97]}"(g2), "{v[98:129]}"(g3)); _v; })

template <int MODE>
__global__ __launch_bounds__(64) void k(const uint32_t* in, uint64_t* out, uint32_t iters) {
  __shared__ uint16_t tab[4096];
  v32 g0, g1, g2, g3;
  const uint32_t l = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 32; i++) { g0[i] = in[i*64+l]; g1[i] = in[(32+i)*64+l]; g2[i] = in[(64+i)*64+l]; g3[i] = in[(96+i)*64+l]; }
  for (int i = l; i < 4096; i += 64) tab[i] = (uint16_t)(i * 2654435761u >> 20);
  __syncthreads();
  uint32_t x = 1;
  uint64_t t0 = clock64();
  for (uint32_t s = 0; s < iters; s++) {
    if (MODE == 0) {  // readlane from a fixed VGPR
      x = __builtin_amdgcn_readlane(g0[5], x & 63) + s;
    } else if (MODE == 1) {  // gpr_idx + readlane
      uint32_t v = REG_OF(x & 127);
      x = __builtin_amdgcn_readlane(v, (x >> 7) & 63) + s;
    } else if (MODE == 2) {  // LDS dependent chain
      x = __builtin_amdgcn_readfirstlane(tab[x & 4095]) + s;
    } else if (MODE == 3) {  // both
      uint32_t v = REG_OF(x & 127);
      uint32_t y = __builtin_amdgcn_readlane(v, (x >> 7) & 63);
      x = __builtin_amdgcn_readfirstlane(tab[y & 4095]) + s;
    } else if (MODE == 4) {  // LDS chain + 2 single-lane writes
      x = __builtin_amdgcn_readfirstlane(tab[x & 4095]) + s;
      if (l == 0) { tab[(x * 7) & 4095] = (uint16_t)s; tab[(x * 13) & 4095] = (uint16_t)x; }
    }
  }
  uint64_t t1 = clock64();
  if (l == 0) out[blockIdx.x] = (t1 - t0) * 1000 / iters + (x & 0);
  if (x == 0xdeadbeef) out[0] = 1;
}

int main() {
  uint32_t* din; uint64_t* dout;
  hipMalloc(&din, 8192 * 4); hipMalloc(&dout, 4096 * 8);
  hipMemset(din, 0x5a, 8192 * 4);
  uint64_t h[4096];
  const char* names[] = {"readlane", "gpridx+readlane", "lds chain", "gpridx+readlane+lds", "lds+2writes"};
  for (int mode = 0; mode < 5; mode++) {
    for (int blocks : {1, 256 * 4, 256 * 12}) {
      auto launch = [&](uint32_t it) {
        if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(64), 0, 0, din, dout, it);
        if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(64), 0, 0, din, dout, it);
        if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(64), 0, 0, din, dout, it);
        if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(64), 0, 0, din, dout, it);
        if (mode == 4) hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(64), 0, 0, din, dout, it);
      };
      launch(1000); hipDeviceSynchronize();
      hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
      hipEventRecord(e0); launch(20000); hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      hipMemcpy(h, dout, 8 * (blocks < 4096 ? blocks : 4096), hipMemcpyDeviceToHost);
      double avg = 0; for (int i = 0; i < blocks && i < 4096; i++) avg += h[i]; avg /= (blocks < 4096 ? blocks : 4096);
      printf("%-22s blocks %5d: %.1f cycles/iter (clock64), wall %.3f ms -> %.1f ns/iter/wave\n", names[mode], blocks, avg / 1000.0, ms, ms * 1e6 / 20000);
    }
  }
  return 0;
}
