// membench.hip — read-pattern microbenchmark for 64-byte packet slots.
// Measures what the header-read pattern alone can sustain on MI355X:
//   A: per-lane strided   dword@12 + dwordx3@24 (+ dword@32) per 64 B slot
//   B: coalesced          4 x dwordx4 per lane, a wave reads 4 KiB contiguous
//   C: LDS-DMA            4 x global_load_lds_dwordx4 per wave (4 KiB) then
//                         ds_read_b128 of the packet's three chunks
//   D: plain copy-read    dwordx4 streaming (roofline reference)
// Each variant writes one u32 per packet (so nothing is dead) and streams
// ~320 MiB of slots. Build: hipcc --offload-arch=gfx950 -O3 membench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

__device__ __forceinline__ uint32_t mixw(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return a ^ (b * 3u) ^ (c * 5u) ^ (d * 7u);
}

template <int PPT>
__global__ __launch_bounds__(256) void kA(const uint8_t *__restrict__ pk, uint32_t *__restrict__ out, uint32_t n) {
    const uint32_t base = blockIdx.x * 256 * PPT;
    uint32_t w3[PPT], w6[PPT], w7[PPT], w8[PPT];
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        uint32_t i = min(base + k * 256 + threadIdx.x, n - 1);
        const uint8_t *p = pk + (size_t)i * 64;
        w3[k] = *(const uint32_t *)(p + 12);
        uint2 v = *(const uint2 *)(p + 24);
        w6[k] = v.x; w7[k] = v.y;
        w8[k] = *(const uint32_t *)(p + 32);
    }
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        uint32_t i = base + k * 256 + threadIdx.x;
        if (i < n) out[i] = mixw(w3[k], w6[k], w7[k], w8[k]);
    }
}

// kA with grid-interleaved steps: at step k every workgroup reads inside one
// contiguous window (packet = k*grid*256 + blockIdx*256 + tid)
template <int PPT>
__global__ __launch_bounds__(256) void kE(const uint8_t *__restrict__ pk, uint32_t *__restrict__ out, uint32_t n) {
    uint32_t w3[PPT], w6[PPT], w7[PPT], w8[PPT];
    const uint32_t span = gridDim.x * 256;
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        uint32_t i = min(k * span + blockIdx.x * 256 + threadIdx.x, n - 1);
        const uint8_t *p = pk + (size_t)i * 64;
        w3[k] = *(const uint32_t *)(p + 12);
        uint2 v = *(const uint2 *)(p + 24);
        w6[k] = v.x; w7[k] = v.y;
        w8[k] = *(const uint32_t *)(p + 32);
    }
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        uint32_t i = k * span + blockIdx.x * 256 + threadIdx.x;
        if (i < n) out[i] = mixw(w3[k], w6[k], w7[k], w8[k]);
    }
}

// kA with 8-byte result records written per packet (the pipeline's write mix)
template <int PPT>
__global__ __launch_bounds__(256) void kF(const uint8_t *__restrict__ pk, uint2 *__restrict__ out, uint32_t n) {
    const uint32_t base = blockIdx.x * 256 * PPT;
    uint32_t w3[PPT], w6[PPT], w7[PPT], w8[PPT];
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        uint32_t i = min(base + k * 256 + threadIdx.x, n - 1);
        const uint8_t *p = pk + (size_t)i * 64;
        w3[k] = *(const uint32_t *)(p + 12);
        uint2 v = *(const uint2 *)(p + 24);
        w6[k] = v.x; w7[k] = v.y;
        w8[k] = *(const uint32_t *)(p + 32);
    }
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        uint32_t i = base + k * 256 + threadIdx.x;
        if (i < n) out[i] = make_uint2(mixw(w3[k], w6[k], w7[k], w8[k]), w3[k]);
    }
}

template <int PPT>
__global__ __launch_bounds__(256) void kB(const uint8_t *__restrict__ pk, uint32_t *__restrict__ out, uint32_t n) {
    // wave w of the block handles packets [base + w*64*PPT + s*64, +64) per step s;
    // lane l loads 16 B at byte (c*64 + l)*16 of the step's 4 KiB, c = 0..3
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t base = blockIdx.x * 256 * PPT + wave * 64 * PPT;
    __shared__ uint4 sh[4][4][64];   // [wave][c][lane]
    uint32_t acc = 0;
#pragma unroll 1
    for (int s = 0; s < PPT; s++) {
        const uint32_t p0 = base + s * 64;
        uint4 v[4];
#pragma unroll
        for (int c = 0; c < 4; c++) {
            uint32_t q = min(p0 + c * 16 + lane / 4, n - 1);
            v[c] = *(const uint4 *)(pk + (size_t)q * 64 + (lane & 3) * 16);
        }
#pragma unroll
        for (int c = 0; c < 4; c++) sh[wave][c][lane] = v[c];
        __builtin_amdgcn_s_waitcnt(0xC07F);
        // packet p0+lane's chunk k is at sh[wave][lane/16][(lane%16)*4 + k]
        const uint4 *row = &sh[wave][lane >> 4][(lane & 15) * 4];
        uint4 c0 = row[0], c1 = row[1], c2 = row[2];
        uint32_t i = p0 + lane;
        if (i < n) out[i] = mixw(c0.w, c1.z, c1.w, c2.x);
        acc += c0.x;
    }
    if (acc == 0xFFFFFFFFu) out[0] = acc;
}

template <int PPT>
__global__ __launch_bounds__(256) void kC(const uint8_t *__restrict__ pk, uint32_t *__restrict__ out, uint32_t n) {
    // LDS-DMA: per step each wave moves its 64 packets' 4 KiB into LDS
    // (linear copy), then each lane reads its 3 chunks with ds_read_b128.
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t base = blockIdx.x * 256 * PPT + wave * 64 * PPT;
    uint32_t *wl = lds + wave * 2 * 1024;   // 2 x 4 KiB per wave
    auto issue = [&](int s) {
        const uint32_t p0 = base + s * 64;
        uint32_t *dst = wl + (s & 1) * 1024;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            uint32_t byte = (c * 64 + lane) * 16;
            uint32_t q = min(p0 + byte / 64, n - 1);
            const uint8_t *src = pk + (size_t)q * 64 + (byte & 63);
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                             (__attribute__((address_space(3))) void *)(dst + c * 256), 16, 0, 0);
        }
    };
    issue(0);
#pragma unroll 1
    for (int s = 0; s < PPT; s++) {
        if (s + 1 < PPT) { issue(s + 1); asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); }
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t *buf = wl + (s & 1) * 1024;
        const uint4 *pkt = (const uint4 *)(buf + lane * 16);
        // rotate the chunk order by lane so 16-lane groups hit distinct banks
        uint4 r0 = pkt[(lane + 0) & 3], r1 = pkt[(lane + 1) & 3], r2 = pkt[(lane + 2) & 3], r3 = pkt[(lane + 3) & 3];
        const int rot = lane & 3;   // chunk k sits in r[(k - rot) & 3]
        uint4 c0 = rot == 0 ? r0 : rot == 1 ? r3 : rot == 2 ? r2 : r1;
        uint4 c1 = rot == 0 ? r1 : rot == 1 ? r0 : rot == 2 ? r3 : r2;
        uint4 c2 = rot == 0 ? r2 : rot == 1 ? r1 : rot == 2 ? r0 : r3;
        uint32_t i = base + s * 64 + lane;
        if (i < n) out[i] = mixw(c0.w, c1.z, c1.w, c2.x);
    }
}

__global__ __launch_bounds__(256) void kD(const uint4 *__restrict__ pk, uint32_t *__restrict__ out, uint64_t n16) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        uint4 v = pk[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
    const uint32_t n = 5u << 20;              // 5 Mi packets = 320 MiB
    uint8_t *pk; uint32_t *out;
    CHK(hipMalloc(&pk, (size_t)n * 64));
    CHK(hipMalloc(&out, (size_t)n * 8 + (1 << 24)));
    CHK(hipMemset(pk, 0x5A, (size_t)n * 64));
    hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, auto launch, double bytes) {
        std::vector<float> v;
        for (int r = 0; r < 12; r++) {
            CHK(hipEventRecord(e0)); launch(); CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
            float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); v.push_back(ms);
        }
        std::sort(v.begin(), v.end());
        float med = v[v.size() / 2];
        printf("%-28s %8.1f us  %7.0f GB/s (algorithmic %.0f B/pkt)\n", name, med * 1e3, bytes / (med * 1e-3) / 1e9, bytes / n);
    };
    const double alg = 64.0 * n + 4.0 * n;
    timeit("A strided ppt4", [&] { hipLaunchKernelGGL(kA<4>, dim3((n + 1023) / 1024), dim3(256), 0, 0, pk, out, n); }, alg);
    timeit("A strided ppt8", [&] { hipLaunchKernelGGL(kA<8>, dim3((n + 2047) / 2048), dim3(256), 0, 0, pk, out, n); }, alg);
    timeit("A strided ppt16", [&] { hipLaunchKernelGGL(kA<16>, dim3((n + 4095) / 4096), dim3(256), 0, 0, pk, out, n); }, alg);
    timeit("E interleaved ppt8", [&] { hipLaunchKernelGGL(kE<8>, dim3((n + 2047) / 2048), dim3(256), 0, 0, pk, out, n); }, alg);
    timeit("E interleaved ppt4", [&] { hipLaunchKernelGGL(kE<4>, dim3((n + 1023) / 1024), dim3(256), 0, 0, pk, out, n); }, alg);
    timeit("F strided+8B rec ppt8", [&] { hipLaunchKernelGGL(kF<8>, dim3((n + 2047) / 2048), dim3(256), 0, 0, pk, (uint2 *)out, n); }, 72.0 * n);
    timeit("B coalesced+lds ppt4", [&] { hipLaunchKernelGGL(kB<4>, dim3((n + 1023) / 1024), dim3(256), 0, 0, pk, out, n); }, alg);
    timeit("B coalesced+lds ppt8", [&] { hipLaunchKernelGGL(kB<8>, dim3((n + 2047) / 2048), dim3(256), 0, 0, pk, out, n); }, alg);
    timeit("C glds ppt4", [&] { hipLaunchKernelGGL(kC<4>, dim3((n + 1023) / 1024), dim3(256), 32768, 0, pk, out, n); }, alg);
    timeit("C glds ppt8", [&] { hipLaunchKernelGGL(kC<8>, dim3((n + 2047) / 2048), dim3(256), 32768, 0, pk, out, n); }, alg);
    timeit("C glds ppt16", [&] { hipLaunchKernelGGL(kC<16>, dim3((n + 4095) / 4096), dim3(256), 32768, 0, pk, out, n); }, alg);
    timeit("D stream dwordx4 g=2048", [&] { hipLaunchKernelGGL(kD, dim3(2048), dim3(256), 0, 0, (const uint4 *)pk, out, (uint64_t)n * 4); }, 64.0 * n);
    timeit("D stream dwordx4 g=8192", [&] { hipLaunchKernelGGL(kD, dim3(8192), dim3(256), 0, 0, (const uint4 *)pk, out, (uint64_t)n * 4); }, 64.0 * n);
    // a 1M-packet slice (the bench's per-launch size) for the best patterns
    const uint32_t m = 1u << 20;
    auto timeit_m = [&](const char *name, auto launch) {
        std::vector<float> v;
        for (int r = 0; r < 12; r++) {
            CHK(hipEventRecord(e0)); launch(); CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
            float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); v.push_back(ms);
        }
        std::sort(v.begin(), v.end());
        float med = v[v.size() / 2];
        printf("%-28s %8.1f us  %7.0f GB/s  (1 Mi pkts)\n", name, med * 1e3, 68.0 * m / (med * 1e-3) / 1e9);
    };
    for (int rep = 0; rep < 2; rep++) {
        uint8_t *src = pk + (size_t)rep * m * 64 * 2;
        timeit_m("A strided ppt8 1M", [&] { hipLaunchKernelGGL(kA<8>, dim3(m / 2048), dim3(256), 0, 0, src, out, m); });
        timeit_m("C glds ppt8 1M", [&] { hipLaunchKernelGGL(kC<8>, dim3(m / 2048), dim3(256), 32768, 0, src, out, m); });
        timeit_m("C glds ppt4 1M", [&] { hipLaunchKernelGGL(kC<4>, dim3(m / 1024), dim3(256), 32768, 0, src, out, m); });
    }
    return 0;
}
