// dispatch_probe.hip — how fast does the dispatcher fill the chip? Each
// workgroup stamps s_memrealtime (100 MHz) at entry and exit and spins for
// a fixed time in between. Reports active workgroups per 2 us. Diagnostic.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/dispatch_probe tools/dispatch_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

__global__ __launch_bounds__(256, 1) void probe(unsigned long long *st, unsigned spin_ticks)
{
    extern __shared__ unsigned lds[];
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    unsigned long long t = t0;
    while (t - t0 < spin_ticks) { __builtin_amdgcn_s_sleep(2); t = __builtin_amdgcn_s_memrealtime(); }
    if (threadIdx.x == 0) { st[blockIdx.x * 2] = t0; st[blockIdx.x * 2 + 1] = t + lds[5]; }
}

int main(int argc, char **argv)
{
    const unsigned nwg = argc > 1 ? atoi(argv[1]) : 12288;
    const unsigned lds = argc > 2 ? atoi(argv[2]) : 27 * 1024;
    const unsigned spin = argc > 3 ? atoi(argv[3]) : 2000;   // ticks of 10 ns
    unsigned long long *d;
    hipMalloc(&d, nwg * 16ull);
    for (int r = 0; r < 3; r++) {
        hipLaunchKernelGGL(probe, dim3(nwg), dim3(256), lds, 0, d, spin);
        hipDeviceSynchronize();
    }
    std::vector<unsigned long long> h(nwg * 2);
    hipMemcpy(h.data(), d, nwg * 16ull, hipMemcpyDeviceToHost);
    unsigned long long t0 = ~0ull, t1 = 0;
    for (unsigned i = 0; i < nwg; i++) { t0 = std::min(t0, h[2 * i]); t1 = std::max(t1, h[2 * i + 1]); }
    printf("wgs %u lds %u spin %.1f us: span %.1f us\n", nwg, lds, spin / 100.0, (t1 - t0) / 100.0);
    printf("first 40 starts (us, by blockIdx):");
    for (unsigned i = 0; i < 40 && i < nwg; i++) printf(" %.2f", (h[2 * i] - t0) / 100.0);
    printf("\nactive per 2us:");
    for (double e = 0; e < (t1 - t0) / 100.0; e += 2) {
        int a = 0;
        for (unsigned i = 0; i < nwg; i++) {
            double s = (h[2 * i] - t0) / 100.0, f = (h[2 * i + 1] - t0) / 100.0;
            if (s < e + 2 && f > e) a++;
        }
        printf(" %d", a);
    }
    printf("\n");
    return 0;
}
