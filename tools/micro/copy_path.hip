// Which pageable-copy path does the runtime take on a stream?  In the host
// API trace (profiles/r04f_host_trace) copies on the host context's stream
// ran as 1 MiB blit kernels (~26 GB/s) while the pipeline lanes' streams
// used the DMA engines (56 GB/s).  Times pageable H2D / D2H of 145 MB on
// streams created in order, idle or right after a kernel, blocking or not.
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/copy_path tools/micro/copy_path.hip && /tmp/copy_path
#include <hip/hip_runtime.h>
#include <chrono>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

__global__ void spin(int *p, int n)
{
    int x = threadIdx.x;
    for (int i = 0; i < n; i++) x = x * 1664525 + 1013904223;
    if (x == 42) p[0] = x;
}

static double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main()
{
    const size_t n = 145000001;
    uint8_t *h = (uint8_t *)malloc(n), *h2 = (uint8_t *)malloc(n);
    memset(h, 1, n);
    memset(h2, 2, n);
    uint8_t *d;
    int *dp;
    if (hipMalloc(&d, n) != hipSuccess || hipMalloc(&dp, 64) != hipSuccess) return 1;
    hipStream_t s[4];
    hipStreamCreateWithFlags(&s[0], hipStreamDefault);
    hipStreamCreateWithFlags(&s[1], hipStreamDefault);
    hipStreamCreateWithFlags(&s[2], hipStreamNonBlocking);
    hipStreamCreateWithFlags(&s[3], hipStreamDefault);
    const char *names[4] = {"first blocking", "second blocking", "non-blocking", "fourth blocking"};
    for (int rep = 0; rep < 2; rep++)
        for (int k = 0; k < 4; k++)
            for (int after_kernel = 0; after_kernel < 2; after_kernel++) {
                hipDeviceSynchronize();
                if (after_kernel) {
                    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s[k], dp, 1000);
                    hipStreamSynchronize(s[k]);
                    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s[k], dp, 10);
                }
                double t0 = now();
                hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s[k]);
                hipStreamSynchronize(s[k]);
                double t1 = now();
                if (after_kernel) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s[k], dp, 10);
                double t2 = now();
                hipMemcpyAsync(h2, d, n, hipMemcpyDeviceToHost, s[k]);
                hipStreamSynchronize(s[k]);
                double t3 = now();
                printf("rep %d stream %-16s %-12s h2d %6.1f GB/s  d2h %6.1f GB/s\n", rep, names[k],
                       after_kernel ? "after kernel" : "idle", n / (t1 - t0) / 1e9, n / (t3 - t2) / 1e9);
            }
    hipStream_t nul = 0;
    for (int rep = 0; rep < 2; rep++) {
        double t0 = now();
        hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, nul);
        hipStreamSynchronize(nul);
        double t1 = now();
        hipMemcpy(h2, d, n, hipMemcpyDeviceToHost);
        double t2 = now();
        printf("rep %d null stream h2d %6.1f GB/s, hipMemcpy d2h %6.1f GB/s\n", rep, n / (t1 - t0) / 1e9,
               n / (t2 - t1) / 1e9);
    }
    return 0;
}
