// membench3.hip — what the 8 B record stream costs next to the 64 B slot
// reads, and whether deferring a workgroup's records into one LDS-staged
// burst changes it. Same 1.5 GiB pool as membench2 (24 Mi slots), Infinity
// Cache flushed between runs, median of 7.
//   R   read only (dwordx4 nt grid-stride)                    64 B/slot
//   W   write only (8 B nt record per slot)                    8 B/slot
//   I   one-shot workgroup of 4096 slots, record written as soon as its
//       slot is read (the pipeline's order)                   72 B/slot
//   B   same reads, records staged in LDS (8 B x slots per workgroup) and
//       written as one contiguous dwordx4 burst at the end   72 B/slot
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/membench3 tools/membench3.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include <string>
#include <string.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void kFill(uint32_t *p, uint64_t nw) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nw; i += (uint64_t)gridDim.x * 256) {
        uint64_t x = i * 0x9E3779B97F4A7C15ull; x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32;
        p[i] = (uint32_t)x;
    }
}

__global__ __launch_bounds__(256) void kR(const u32x4 *__restrict__ pk, uint32_t *__restrict__ sink, uint64_t n16) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        const u32x4 v = __builtin_nontemporal_load(&pk[i]);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    sink[blockIdx.x * 256 + threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void kW(u32x2 *__restrict__ out, uint32_t n) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        u32x2 r; r.x = i; r.y = i * 3u;
        __builtin_nontemporal_store(r, &out[i]);
    }
}

// SPW slots per workgroup = 4*SPW 16-byte chunks; U chunks per lane in flight
template <bool DEFER, int U, int SPW = 4096>
__global__ __launch_bounds__(256) void kB(const u32x4 *__restrict__ pk, u32x2 *__restrict__ out) {
    __shared__ u32x2 rec[SPW];
    const uint64_t c0 = (uint64_t)blockIdx.x * (4u * SPW);
    const uint32_t t = threadIdx.x;
    for (uint32_t it = 0; it < SPW / 64; it += U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = __builtin_nontemporal_load(&pk[c0 + (it + u) * 256u + t]);
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t x = v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
            const uint32_t y = __shfl_xor(x, 1) + __shfl_xor(x, 2);
            const uint32_t slot = ((it + u) * 256u + t) >> 2;   // within the workgroup
            if ((t & 3) == 0) {
                u32x2 r; r.x = x; r.y = y;
                if (DEFER) rec[slot] = r;
                else __builtin_nontemporal_store(r, &out[(uint64_t)blockIdx.x * SPW + slot]);
            }
        }
    }
    if (DEFER) {
        __syncthreads();
        const u32x4 *s = (const u32x4 *)rec;
        u32x4 *o = (u32x4 *)(out + (uint64_t)blockIdx.x * SPW);
#pragma unroll
        for (int k = 0; k < SPW / 512; k++) __builtin_nontemporal_store(s[k * 256 + t], &o[k * 256 + t]);
    }
}

// T consecutive sub-tiles of 2048 slots per workgroup; each sub-tile's
// records staged in LDS and written as one 16 KiB burst at its end (the
// pipeline's per-tile record burst, with T tiles per workgroup)
template <int T, int U>
__global__ __launch_bounds__(256) void kC(const u32x4 *__restrict__ pk, u32x2 *__restrict__ out) {
    __shared__ u32x2 rec[2048];
    const uint32_t t = threadIdx.x;
    for (int st = 0; st < T; st++) {
        const uint64_t tile = (uint64_t)blockIdx.x * T + st;
        const uint64_t c0 = tile * 8192u;
        for (uint32_t it = 0; it < 32; it += U) {
            u32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; u++) v[u] = __builtin_nontemporal_load(&pk[c0 + (it + u) * 256u + t]);
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint32_t x = v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
                const uint32_t y = __shfl_xor(x, 1) + __shfl_xor(x, 2);
                const uint32_t slot = ((it + u) * 256u + t) >> 2;
                if ((t & 3) == 0) { u32x2 r; r.x = x; r.y = y; rec[slot] = r; }
            }
        }
        __syncthreads();
        const u32x4 *s = (const u32x4 *)rec;
        u32x4 *o = (u32x4 *)(out + tile * 2048u);
#pragma unroll
        for (int k = 0; k < 4; k++) __builtin_nontemporal_store(s[k * 256 + t], &o[k * 256 + t]);
        __syncthreads();
    }
}

// the one-shot pipeline's memory behaviour without its classification: a
// tile of 256*PPT slots per workgroup, each lane loads its PPT slots whole
// (4 x dwordx4), then writes their 8 B records (512 B per wave store);
// occupancy set by dynamic LDS
template <int PPT>
__global__ __launch_bounds__(256) void kP(const u32x4 *__restrict__ pk, u32x2 *__restrict__ out) {
    const uint64_t base = (uint64_t)blockIdx.x * (256u * PPT);
    const uint32_t t = threadIdx.x;
    u32x4 v[PPT][4];
#pragma unroll
    for (int k = 0; k < PPT; k++)
#pragma unroll
        for (int c = 0; c < 4; c++) v[k][c] = __builtin_nontemporal_load(&pk[(base + k * 256u + t) * 4u + c]);
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        const u32x4 a = v[k][0] ^ v[k][1] ^ v[k][2] ^ v[k][3];
        u32x2 r; r.x = a.x ^ a.y; r.y = a.z + a.w;
        __builtin_nontemporal_store(r, &out[base + k * 256u + t]);
    }
}

int main() {
    const uint32_t n = 24u << 20;             // 24 Mi slots = 1.5 GiB
    int cus = 0; CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    printf("%d CUs\n", cus);
    uint8_t *pk; u32x2 *out;
    CHK(hipMalloc(&pk, (size_t)n * 64));
    CHK(hipMalloc(&out, (size_t)n * 8));
    hipLaunchKernelGGL(kFill, dim3(4096), dim3(256), 0, 0, (uint32_t *)pk, (uint64_t)n * 16);
    uint8_t *flush; const size_t fl = 512u << 20;
    CHK(hipMalloc(&flush, fl));
    CHK(hipMemset(flush, 1, fl));
    uint32_t *sink; CHK(hipMalloc(&sink, 8192 * 256 * 4));
    hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    std::vector<u32x2> ref(n), got(n);
    auto timeit = [&](const char *name, auto launch, double bytes, int check) {
        std::vector<float> v;
        for (int r = 0; r < 7; r++) {
            hipLaunchKernelGGL(kR, dim3(2048), dim3(256), 0, 0, (const u32x4 *)flush, sink, (uint64_t)fl / 16);
            CHK(hipMemsetAsync(out, 0, (size_t)n * 8, 0));
            hipLaunchKernelGGL(kR, dim3(2048), dim3(256), 0, 0, (const u32x4 *)flush, sink, (uint64_t)fl / 16);
            CHK(hipEventRecord(e0)); launch(); CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
            float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); v.push_back(ms);
        }
        CHK(hipGetLastError());
        std::sort(v.begin(), v.end());
        const float med = v[v.size() / 2];
        const char *ok = "";
        if (check) {
            CHK(hipMemcpy(check == 1 ? ref.data() : got.data(), out, (size_t)n * 8, hipMemcpyDeviceToHost));
            ok = check == 1 ? "(ref)" : (memcmp(ref.data(), got.data(), (size_t)n * 8) == 0 ? "ok" : "MISMATCH");
        }
        printf("%-34s %8.1f us  %7.0f GB/s  %s\n", name, med * 1e3, bytes / (med * 1e-3) / 1e9, ok);
        fflush(stdout);
    };
    const uint32_t nwg = n / 4096;
    for (int g : {1024, 2048, 4096})
        timeit(("R read only g=" + std::to_string(g)).c_str(), [&] {
            hipLaunchKernelGGL(kR, dim3(g), dim3(256), 0, 0, (const u32x4 *)pk, sink, (uint64_t)n * 4); }, 64.0 * n, 0);
    for (int g : {1024, 4096})
        timeit(("W write only g=" + std::to_string(g)).c_str(), [&] {
            hipLaunchKernelGGL(kW, dim3(g), dim3(256), 0, 0, out, n); }, 8.0 * n, 0);
    timeit("I immediate records U4", [&] { hipLaunchKernelGGL((kB<false, 4>), dim3(nwg), dim3(256), 0, 0, (const u32x4 *)pk, out); }, 72.0 * n, 1);
    timeit("B LDS-deferred records U4", [&] { hipLaunchKernelGGL((kB<true, 4>), dim3(nwg), dim3(256), 0, 0, (const u32x4 *)pk, out); }, 72.0 * n, 2);
    timeit("I immediate records U8", [&] { hipLaunchKernelGGL((kB<false, 8>), dim3(nwg), dim3(256), 0, 0, (const u32x4 *)pk, out); }, 72.0 * n, 2);
    timeit("B LDS-deferred records U8", [&] { hipLaunchKernelGGL((kB<true, 8>), dim3(nwg), dim3(256), 0, 0, (const u32x4 *)pk, out); }, 72.0 * n, 2);
    timeit("B deferred U4 1024 slots/WG", [&] { hipLaunchKernelGGL((kB<true, 4, 1024>), dim3(n / 1024), dim3(256), 0, 0, (const u32x4 *)pk, out); }, 72.0 * n, 2);
    timeit("B deferred U4 2048 slots/WG", [&] { hipLaunchKernelGGL((kB<true, 4, 2048>), dim3(n / 2048), dim3(256), 0, 0, (const u32x4 *)pk, out); }, 72.0 * n, 2);
    timeit("B deferred U4 8192 slots/WG", [&] { hipLaunchKernelGGL((kB<true, 4, 8192>), dim3(n / 8192), dim3(256), 0, 0, (const u32x4 *)pk, out); }, 72.0 * n, 2);
    timeit("I immediate U4 2048 slots/WG", [&] { hipLaunchKernelGGL((kB<false, 4, 2048>), dim3(n / 2048), dim3(256), 0, 0, (const u32x4 *)pk, out); }, 72.0 * n, 2);
    timeit("C 2048-tiles x1 per WG U4", [&] { hipLaunchKernelGGL((kC<1, 4>), dim3(n / 2048), dim3(256), 0, 0, (const u32x4 *)pk, out); }, 72.0 * n, 2);
    timeit("C 2048-tiles x2 per WG U4", [&] { hipLaunchKernelGGL((kC<2, 4>), dim3(n / 4096), dim3(256), 0, 0, (const u32x4 *)pk, out); }, 72.0 * n, 2);
    timeit("C 2048-tiles x4 per WG U4", [&] { hipLaunchKernelGGL((kC<4, 4>), dim3(n / 8192), dim3(256), 0, 0, (const u32x4 *)pk, out); }, 72.0 * n, 2);
    timeit("C 2048-tiles x8 per WG U4", [&] { hipLaunchKernelGGL((kC<8, 4>), dim3(n / 16384), dim3(256), 0, 0, (const u32x4 *)pk, out); }, 72.0 * n, 2);
    timeit("C 2048-tiles x4 per WG U8", [&] { hipLaunchKernelGGL((kC<4, 8>), dim3(n / 8192), dim3(256), 0, 0, (const u32x4 *)pk, out); }, 72.0 * n, 2);
    timeit("B deferred U4 16384 slots/WG", [&] { hipLaunchKernelGGL((kB<true, 4, 16384>), dim3(n / 16384), dim3(256), 0, 0, (const u32x4 *)pk, out); }, 72.0 * n, 2);
    CHK(hipFuncSetAttribute((const void *)kC<4, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10));
    CHK(hipFuncSetAttribute((const void *)kP<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10));
    CHK(hipFuncSetAttribute((const void *)kP<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10));
    for (int lds : {36 << 10, 60 << 10}) {
        timeit(("C 2048-tiles x4 U4 +LDS " + std::to_string(lds >> 10) + "K").c_str(), [&] {
            hipLaunchKernelGGL((kC<4, 4>), dim3(n / 8192), dim3(256), lds, 0, (const u32x4 *)pk, out); }, 72.0 * n, 2);
    }
    for (int lds : {0, 20 << 10, 36 << 10, 60 << 10}) {
        timeit(("P ppt8 one-shot +LDS " + std::to_string(lds >> 10) + "K").c_str(), [&] {
            hipLaunchKernelGGL((kP<8>), dim3(n / 2048), dim3(256), lds, 0, (const u32x4 *)pk, out); }, 72.0 * n, 0);
        timeit(("P ppt4 one-shot +LDS " + std::to_string(lds >> 10) + "K").c_str(), [&] {
            hipLaunchKernelGGL((kP<4>), dim3(n / 1024), dim3(256), lds, 0, (const u32x4 *)pk, out); }, 72.0 * n, 0);
    }
    timeit("R+W back to back g=2048", [&] {
        hipLaunchKernelGGL(kR, dim3(2048), dim3(256), 0, 0, (const u32x4 *)pk, sink, (uint64_t)n * 4);
        hipLaunchKernelGGL(kW, dim3(2048), dim3(256), 0, 0, out, n); }, 72.0 * n, 0);
    return 0;
}
