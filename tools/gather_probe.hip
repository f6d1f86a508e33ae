// gather_probe.hip — diagnostic: how fast can the GPU gather packet headers
// from an mbuf pool in HOST memory itself ("GPU-side
// gather")? The host hands over only the burst's mbuf pointers; the kernel
// reads each mbuf's buf_addr and data_off (rte_pktmbuf_mtod) and the 24
// header bytes the pipeline needs, over PCIe, and writes 16-byte header
// records (COP_HDR16 layout) to device memory. Compared with the host
// gather of the same records (one thread). Not the product.
//
// Pool: malloc'd, hipHostRegister'ed (as a DPDK hugepage pool would be),
// 2176-byte mbufs, buf_addr = mbuf + 128, data_off = 128. Every pointer is
// range-checked before it is dereferenced.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CHK(x)                                                                            \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                       \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x2a __attribute__((ext_vector_type(2), aligned(4)));

constexpr uint32_t MBUF = 2176;

__global__ void gather(const unsigned long long *ptrs, uint32_t n, unsigned long long lo, unsigned long long hi,
                       long long delta, u32x4 *out, uint32_t *bad)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned long long m = ptrs[i];
    u32x4 r = {0u, 0u, 0u, 0u};
    if (m >= lo && m + 64 <= hi) {
        const unsigned long long buf = *(const unsigned long long *)(m + delta);
        const uint16_t doff = *(const uint16_t *)(m + delta + 16);
        const unsigned long long pk = buf + doff;
        if (pk >= lo && pk + 36 <= hi && (pk & 3) == 0) {
            const u32x4a a = *(const u32x4a *)(pk + delta + 12);
            const u32x2a b = *(const u32x2a *)(pk + delta + 28);
            r = u32x4{a.x, a.w, b.x, b.y};
        } else {
            atomicAdd(bad, 1u);
        }
    } else {
        atomicAdd(bad, 1u);
    }
    out[i] = r;
}

int main(int argc, char **argv)
{
    const uint32_t n_mbuf = 262144;
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);
    const size_t pool_bytes = (size_t)n_mbuf * MBUF;
    uint8_t *pool = (uint8_t *)aligned_alloc(4096, pool_bytes);
    std::mt19937_64 rng(42);
    for (uint32_t k = 0; k < n_mbuf; k++) {
        uint8_t *mb = pool + (size_t)k * MBUF;
        memset(mb, 0, 256);
        const unsigned long long buf = (unsigned long long)(mb + 128);
        const uint16_t doff = 128;
        memcpy(mb, &buf, 8);
        memcpy(mb + 16, &doff, 2);
        for (int b = 0; b < 64; b++) mb[256 + b] = (uint8_t)rng();
    }
    CHK(hipHostRegister(pool, pool_bytes, hipHostRegisterMapped));
    void *dpool = nullptr;
    CHK(hipHostGetDevicePointer(&dpool, pool, 0));
    const long long delta = (long long)((uint8_t *)dpool - pool);
    printf("pool %zu MiB registered: host %p device %p (delta %lld)\n", pool_bytes >> 20, (void *)pool, dpool, delta);

    unsigned long long *hptr = nullptr, *dptr = nullptr;
    CHK(hipHostMalloc(&hptr, (size_t)n * 8, hipHostMallocMapped));
    CHK(hipHostGetDevicePointer((void **)&dptr, hptr, 0));
    for (uint32_t i = 0; i < n; i++) hptr[i] = (unsigned long long)(pool + (size_t)(rng() % n_mbuf) * MBUF);
    u32x4 *dout = nullptr;
    uint32_t *dbad = nullptr;
    CHK(hipMalloc(&dout, (size_t)n * 16));
    CHK(hipMalloc(&dbad, 4));
    CHK(hipMemset(dbad, 0, 4));

    // host gather of the same records (one thread), the reference point
    std::vector<uint32_t> href((size_t)n * 4);
    const auto h0 = std::chrono::steady_clock::now();
    for (uint32_t i = 0; i < n; i++) {
        const uint8_t *m = (const uint8_t *)hptr[i];
        unsigned long long buf;
        uint16_t doff;
        memcpy(&buf, m, 8);
        memcpy(&doff, m + 16, 2);
        const uint8_t *pk = (const uint8_t *)buf + doff;
        memcpy(&href[4 * (size_t)i], pk + 12, 4);
        memcpy(&href[4 * (size_t)i + 1], pk + 24, 12);
    }
    const double host_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - h0).count();

    const unsigned long long lo = (unsigned long long)pool, hi = lo + pool_bytes;
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    std::vector<float> ms;
    for (int rep = 0; rep < 12; rep++) {
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL(gather, dim3((n + 255) / 256), dim3(256), 0, 0, dptr, n, lo, hi, delta, dout, dbad);
        CHK(hipGetLastError());
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float t = 0;
        CHK(hipEventElapsedTime(&t, e0, e1));
        if (rep >= 2) ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    std::vector<uint32_t> got((size_t)n * 4);
    CHK(hipMemcpy(got.data(), dout, (size_t)n * 16, hipMemcpyDeviceToHost));
    uint32_t bad = 0;
    CHK(hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost));
    const bool same = got == href;
    const double med = ms[ms.size() / 2];
    printf("GPU gather: %u packets in %.1f us (median of %zu) = %.1f Mpkt/s; records %s the host gather's; %u bad\n", n,
           med * 1e3, ms.size(), n / (med * 1e-3) / 1e6, same ? "equal" : "DIFFER from", bad);
    printf("host gather (1 thread): %.1f Mpkt/s\n", n / host_s / 1e6);
    CHK(hipHostUnregister(pool));
    free(pool);
    return same && bad == 0 ? 0 : 1;
}
