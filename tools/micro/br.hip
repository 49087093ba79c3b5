// Cost of taken scalar branches, s_waitcnt vmcnt with nothing outstanding, and ds byte read->write.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
template <int MODE>
__global__ __launch_bounds__(64) void k(uint64_t* out, uint32_t iters, uint32_t salt) {
  __shared__ uint8_t ob[32768];
  const uint32_t l = threadIdx.x;
  for (int i = l; i < 32768; i += 64) ob[i] = (uint8_t)i;
  __syncthreads();
  uint32_t x = salt, acc = 0;
  uint64_t t0 = clock64();
  for (uint32_t s = 0; s < iters; s++) {
    if (MODE == 0) {  // 4 data-dependent uniform branches (alternating)
      x = x * 1664525u + 1013904223u;
      if (x & 0x10000) acc += 3; else acc ^= 5;
      if (x & 0x20000) acc += 7; else acc ^= 11;
      if (x & 0x40000) acc += 13; else acc ^= 17;
      if (x & 0x80000) acc += 19; else acc ^= 23;
    } else if (MODE == 1) {  // same arithmetic, branch-free
      x = x * 1664525u + 1013904223u;
      acc += (x & 0x10000) ? 3 : 0; acc ^= (x & 0x20000) ? 7 : 11;
      acc += (x & 0x40000) ? 13 : 0; acc ^= (x & 0x80000) ? 19 : 23;
    } else if (MODE == 2) {  // LDS byte copy chain: read 64 bytes -> write 64 bytes
      uint32_t src = (x & 16383), dst = 16384 + ((x >> 14) & 16383);
      if (dst + 64 > 32768) dst -= 64;
      ob[dst + l] = ob[src + l];
      x = x * 1664525u + 1013904223u;
    } else if (MODE == 3) {  // dependent LDS byte copy (next src = prev dst)
      uint32_t src = x & 32767; if (src + 64 > 32768) src -= 64;
      uint32_t dst = (src + 97) & 32767; if (dst + 64 > 32768) dst -= 64;
      ob[dst + l] = ob[src + l];
      x = dst + __builtin_amdgcn_readfirstlane(ob[dst]);
    }
  }
  uint64_t t1 = clock64();
  if (l == 0) out[blockIdx.x] = (t1 - t0) * 1000 / iters;
  if (acc == 0xdeadbeef) out[1] = x;
}
int main() {
  uint64_t* dout; hipMalloc(&dout, 4096 * 8);
  uint64_t h[4];
  const char* names[] = {"4 uniform branches", "branch-free same math", "lds 64B copy (indep)", "lds 64B copy (dependent)"};
  for (int m = 0; m < 4; m++) {
    auto launch = [&](uint32_t it) {
      if (m == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, dout, it, 12345u);
      if (m == 1) hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, dout, it, 12345u);
      if (m == 2) hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, dout, it, 12345u);
      if (m == 3) hipLaunchKernelGGL(k<3>, dim3(1), dim3(64), 0, 0, dout, it, 12345u);
    };
    launch(100); hipDeviceSynchronize(); launch(20000); hipDeviceSynchronize();
    hipMemcpy(h, dout, 8, hipMemcpyDeviceToHost);
    printf("%-28s %.1f cycles/iter\n", names[m], h[0] / 1000.0);
  }
  return 0;
}
