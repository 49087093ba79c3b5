// More latency microbenchmarks (cycles per dependent step, clock64 = s_memtime).
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
  uint32_t x = 1, y = 7;
  uint32_t vx = l;
  uint64_t t0 = clock64();
  for (uint32_t s = 0; s < iters; s++) {
    if (MODE == 5) {  // LDS chain + 2 all-lane same-address writes
      x = __builtin_amdgcn_readfirstlane(tab[x & 4095]) + s;
      tab[(x * 7) & 4095] = (uint16_t)s; tab[(x * 13) & 4095] = (uint16_t)x;
    } else if (MODE == 6) {  // gpr_idx + 2 readlanes (pair) + funnel, branch-free
      uint32_t d = x & 8191, r = d / 63, ln = d - 63 * r;
      uint32_t v = REG_OF(r & 127);
      uint32_t hi = __builtin_amdgcn_readlane(v, ln), lo = __builtin_amdgcn_readlane(v, ln + 1);
      x = (uint32_t)(((((uint64_t)hi << 32) | lo) << (8 * (s & 3))) >> 32) + s;
    } else if (MODE == 7) {  // two independent mode-6 chains
      uint32_t d = x & 8191, r = d / 63, ln = d - 63 * r;
      uint32_t e = y & 8191, r2 = e / 63, ln2 = e - 63 * r2;
      uint32_t v = REG_OF(r & 127);
      uint32_t w = REG_OF(r2 & 127);
      uint32_t hi = __builtin_amdgcn_readlane(v, ln), lo = __builtin_amdgcn_readlane(v, ln + 1);
      uint32_t hi2 = __builtin_amdgcn_readlane(w, ln2), lo2 = __builtin_amdgcn_readlane(w, ln2 + 1);
      x = (uint32_t)(((((uint64_t)hi << 32) | lo) << (8 * (s & 3))) >> 32) + s;
      y = (uint32_t)(((((uint64_t)hi2 << 32) | lo2) << (8 * (s & 3))) >> 32) + s;
    } else if (MODE == 9) {  // VALU-resident LDS chain (no readfirstlane)
      vx = tab[vx & 4095] + s;
    } else if (MODE == 10) {  // 4 independent table reads in 4 lanes + 4 readlanes
      uint32_t a = (x * 0x9E3779B1u) >> 20;
      uint32_t addr = (a + l * 977) & 4095;
      uint32_t t = tab[addr];
      uint32_t t0 = __builtin_amdgcn_readlane(t, 0), t1 = __builtin_amdgcn_readlane(t, 1);
      uint32_t t2 = __builtin_amdgcn_readlane(t, 2), t3 = __builtin_amdgcn_readlane(t, 3);
      x = t0 + t1 * 3 + t2 * 5 + t3 * 7 + s;
    }
  }
  uint64_t t1 = clock64();
  if (l == 0) out[blockIdx.x] = (t1 - t0) * 1000 / iters;
  if ((x ^ y ^ vx) == 0xdeadbeef) out[1] = 1;
}

__global__ void dup(uint32_t* res) {
  __shared__ uint32_t cell[4];
  if (threadIdx.x == 0) cell[0] = 0xFFFFFFFF;
  __syncthreads();
  cell[0] = threadIdx.x;          // 64 lanes, same address
  __syncthreads();
  if (threadIdx.x == 0) res[0] = cell[0];
  __syncthreads();
  __shared__ uint16_t c16[4];
  c16[1] = (uint16_t)(threadIdx.x + 100);
  __syncthreads();
  if (threadIdx.x == 0) res[1] = c16[1];
}

int main() {
  uint32_t* din; uint64_t* dout; uint32_t* dres;
  hipMalloc(&din, 8192 * 4); hipMalloc(&dout, 4096 * 8); hipMalloc(&dres, 64);
  hipMemset(din, 0x5a, 8192 * 4);
  uint64_t h[4096];
  struct M { int mode; const char* name; } modes[] = {{5, "lds+2 all-lane writes"}, {6, "gpridx+pair, no branch"}, {7, "2 chains of gpridx+pair"}, {9, "VALU lds chain"}, {10, "4-lane table read+4 readlane"}};
  for (auto m : modes) {
    for (int blocks : {1, 256 * 12}) {
      auto launch = [&](uint32_t it) {
        if (m.mode == 5) hipLaunchKernelGGL(k<5>, dim3(blocks), dim3(64), 0, 0, din, dout, it);
        if (m.mode == 6) hipLaunchKernelGGL(k<6>, dim3(blocks), dim3(64), 0, 0, din, dout, it);
        if (m.mode == 7) hipLaunchKernelGGL(k<7>, dim3(blocks), dim3(64), 0, 0, din, dout, it);
        if (m.mode == 9) hipLaunchKernelGGL(k<9>, dim3(blocks), dim3(64), 0, 0, din, dout, it);
        if (m.mode == 10) hipLaunchKernelGGL(k<10>, dim3(blocks), dim3(64), 0, 0, din, dout, it);
      };
      launch(1000); hipDeviceSynchronize();
      launch(20000); hipDeviceSynchronize();
      hipMemcpy(h, dout, 8 * (blocks < 4096 ? blocks : 4096), hipMemcpyDeviceToHost);
      double avg = 0; int nb = blocks < 4096 ? blocks : 4096; for (int i = 0; i < nb; i++) avg += h[i]; avg /= nb;
      printf("%-30s blocks %5d: %.1f cycles/iter\n", m.name, blocks, avg / 1000.0);
    }
  }
  hipLaunchKernelGGL(dup, dim3(1), dim3(64), 0, 0, dres);
  uint32_t r[2]; hipMemcpy(r, dres, 8, hipMemcpyDeviceToHost);
  printf("same-address LDS write winner: u32 lane %u, u16 value %u\n", r[0], r[1]);
  return 0;
}
