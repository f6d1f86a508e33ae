// probebench.hip — calibration of isolated 4-byte random table probes
// (measurement tooling, not the product).
//
// Each case reads a KNOWN number of random dword probes, so under
// rocprofv3 --pmc FETCH_SIZE (or TCC_EA0_RDREQ) the counter value per probe
// is measured directly (tools/pmc_traffic.py applies it to the probe share of
// the pipeline's traffic), and the timed rate is the box's random-probe
// ceiling for the same table sizes as the pipeline's DIR-24-8 tbl24s:
//   rand64   : 2^24-entry (64 MiB) table, 8 packets x 1 probe per lane
//   rand2x64 : two 64 MiB tables, 8 packets x 2 probes per lane (config 5)
//   rand2g   : a 2 GiB table (beyond the 256 MiB Infinity Cache: HBM)
//   pair64   : per lane one probe, then an L1-bypassing load 64 B further in
//              the same 128-byte line (fill granularity: 1 or 2 requests)
//   pair32   : the same 32 B further (same 64-byte half: always 1 request)
//   spair64/32: the two loads issued together (plain loads: a miss fill that
//              covers both offsets merges them into one request)
//   rand16g  : a 16 GiB table (almost no Infinity-Cache hits)
// Prints one line per case: name, probes, median us, Gprobes/s.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "probe_kernels.h"

#define CHK(x)                                                                   \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            printf("%s: %s\n", #x, hipGetErrorString(e));                        \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

int main()
{
    const size_t big = (size_t)2 << 30;
    uint32_t *t0, *t1, *tb, *out;
    CHK(hipMalloc(&t0, 64u << 20));
    CHK(hipMalloc(&t1, 64u << 20));
    CHK(hipMalloc(&tb, big));
    CHK(hipMemset(t0, 0x11, 64u << 20));
    CHK(hipMemset(t1, 0x22, 64u << 20));
    CHK(hipMemset(tb, 0x33, big));
    const uint32_t grid = 256 * 16;
    CHK(hipMalloc(&out, (size_t)grid * 256 * 4));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, double probes, auto launch) {
        std::vector<float> v;
        for (int r = 0; r < 9; r++) {
            CHK(hipEventRecord(e0));
            launch((uint64_t)r * 0x9E3779B9ull);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            if (r) v.push_back(ms);
        }
        std::sort(v.begin(), v.end());
        const float med = v[v.size() / 2];
        printf("%-10s probes %12.0f  %9.1f us  %7.2f Gprobes/s\n", name, probes, med * 1e3, probes / (med * 1e-3) / 1e9);
    };
    const int rounds = 4;
    const double lanes = (double)grid * 256;
    timeit("rand64", lanes * 8 * rounds, [&](uint64_t s) {
        hipLaunchKernelGGL(probek::probe_rand<8>, dim3(grid), dim3(256), 0, 0, t0, t1, 1u << 24, 1, rounds, s, out);
    });
    timeit("rand2x64", lanes * 16 * rounds, [&](uint64_t s) {
        hipLaunchKernelGGL(probek::probe_rand<8>, dim3(grid), dim3(256), 0, 0, t0, t1, 1u << 24, 2, rounds, s, out);
    });
    timeit("rand2g", lanes * 8 * rounds, [&](uint64_t s) {
        hipLaunchKernelGGL(probek::probe_rand<8>, dim3(grid), dim3(256), 0, 0, tb, tb, (uint32_t)(big / 4), 1, rounds,
                           s, out);
    });
    timeit("pair64", lanes * 2, [&](uint64_t s) {
        hipLaunchKernelGGL(probek::probe_pair, dim3(grid), dim3(256), 0, 0, tb, (uint32_t)(big / 128), 0u, 64u, s, out);
    });
    timeit("pair32", lanes * 2, [&](uint64_t s) {
        hipLaunchKernelGGL(probek::probe_pair, dim3(grid), dim3(256), 0, 0, tb, (uint32_t)(big / 128), 0u, 32u, s, out);
    });
    timeit("spair64", lanes * 2, [&](uint64_t s) {
        hipLaunchKernelGGL(probek::probe_pair_sim, dim3(grid), dim3(256), 0, 0, tb, (uint32_t)(big / 128), 0u, 64u, s,
                           out);
    });
    timeit("spair32", lanes * 2, [&](uint64_t s) {
        hipLaunchKernelGGL(probek::probe_pair_sim, dim3(grid), dim3(256), 0, 0, tb, (uint32_t)(big / 128), 0u, 32u, s,
                           out);
    });
    // a 16 GiB table: Infinity-Cache hits ~1.6 %, so the rate is what HBM
    // serves for isolated probes (128-byte fills would cap it near 6.3 TB/s /
    // 128 B = 49 Gprobes/s)
    uint32_t *th = nullptr;
    const size_t huge = (size_t)16 << 30;
    if (hipMalloc(&th, huge) == hipSuccess) {
        CHK(hipMemset(th, 0x44, huge));
        timeit("rand16g", lanes * 8 * rounds, [&](uint64_t s) {
            hipLaunchKernelGGL(probek::probe_rand<8>, dim3(grid), dim3(256), 0, 0, th, th, (uint32_t)(huge / 4 - 1) + 1u,
                               1, rounds, s, out);
        });
        CHK(hipFree(th));
    }
    return 0;
}
