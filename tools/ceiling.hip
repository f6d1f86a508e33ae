// ceiling.hip — the box's streaming ceiling for the pipeline's byte mix.
//
// Reads every 64-byte packet slot of a pool once and writes one 8-byte
// record per slot (non-temporal), in two access patterns (a grid-stride of
// 16-byte loads; per-wave LDS-DMA rings): the 72 B/packet of the bench's algorithmic bytes with no
// classification, no tables and no ordering. bench.py times it on the same
// pool, in the same process, right after the pipeline, so that the
// pipeline's roofline fraction can be read against what this box's HBM
// sustains for the identical access mix (boxes differ by up to 10 %).
// Measurement tooling only: not part of the product library.
//
// Build: make -C tools libceiling.so
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "probe_kernels.h"

namespace {

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void copy_mix(const u32x4 *__restrict__ pk, u32x2 *__restrict__ out, uint64_t n16)
{
    // lane i reads 16-byte chunk i of the pool; the slot's first lane (i % 4
    // == 0) writes its record, folded from the four chunks so no load is dead
    const uint64_t step = (uint64_t)gridDim.x * 256;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += step) {
        const u32x4 v = __builtin_nontemporal_load(&pk[i]);
        const uint32_t x = v.x ^ v.w;
        const uint32_t y = __shfl_xor(x, 1) + __shfl_xor(x, 2);
        if ((threadIdx.x & 3) == 0) {
            u32x2 r;
            r.x = x;
            r.y = y;
            __builtin_nontemporal_store(r, &out[i / 4]);
        }
    }
}

// The same byte mix through per-wave LDS-DMA rings (the fastest pattern in
// tools/membench2.hip): a persistent grid, each wave streams wave-tiles of
// 64 slots (4 KiB, four global_load_lds_dwordx4) through a 2-deep ring in
// LDS, keeps the next tile in flight with a counted vmcnt, reads its
// packet's header words from LDS and writes the 8-byte record.
__global__ __launch_bounds__(256) void ring_mix(const uint8_t *__restrict__ pk, u32x2 *__restrict__ out, uint64_t n)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    constexpr int D = 2;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t *ring = lds + wave * D * 1024;
    const uint64_t nwt = (n + 63) / 64;
    const uint64_t W = (uint64_t)gridDim.x * 4;
    const uint64_t w0 = blockIdx.x * 4ull + wave;
    auto issue = [&](uint64_t wt, int slot) {
        uint32_t *dst = ring + slot * 1024;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t byte = (c * 64 + lane) * 16;
            const uint64_t q = min(wt * 64 + byte / 64, n - 1);
            const uint8_t *src = pk + q * 64 + (byte & 63);
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                             (__attribute__((address_space(3))) void *)(dst + c * 256), 16, 0, 2);
        }
    };
    const uint64_t nmine = w0 < nwt ? (nwt - w0 + W - 1) / W : 0;
    if (nmine) issue(w0, 0);
    for (uint64_t i = 0; i < nmine; i++) {
        if (i + 1 < nmine) {
            issue(w0 + (i + 1) * W, (int)((i + 1) % D));
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");   // tile i landed, tile i+1 in flight
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const uint32_t *buf = ring + (i % D) * 1024 + lane * 16;
        const uint32_t w3 = buf[3], w6 = buf[6], w7 = buf[7], w8 = buf[8];
        const uint64_t q = (w0 + i * W) * 64 + lane;
        u32x2 r;
        r.x = w3 ^ (w6 * 3u);
        r.y = w7 + w8;
        if (q < n) __builtin_nontemporal_store(r, &out[q]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads done before the slot is refilled
    }
}

// Deeper LDS-DMA rings (MI355X_MICROARCH.md ldsdma-fill: 6.5-6.8 TB/s
// chip-wide for nt LDS-DMA streams with 8 x 16 KiB in flight per CU): the
// same per-wave tiles of 64 slots, D tiles in flight per wave.
template <int D>
__global__ __launch_bounds__(256) void ring_mix_deep(const uint8_t *__restrict__ pk, u32x2 *__restrict__ out,
                                                     uint64_t n)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t *ring = lds + wave * D * 1024;
    const uint64_t nwt = (n + 63) / 64;
    const uint64_t W = (uint64_t)gridDim.x * 4;
    const uint64_t w0 = blockIdx.x * 4ull + wave;
    auto issue = [&](uint64_t wt, int slot) {
        uint32_t *dst = ring + slot * 1024;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t byte = (c * 64 + lane) * 16;
            const uint64_t q = min(wt * 64 + byte / 64, n - 1);
            const uint8_t *src = pk + q * 64 + (byte & 63);
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                             (__attribute__((address_space(3))) void *)(dst + c * 256), 16, 0, 2);
        }
    };
    const uint64_t nmine = w0 < nwt ? (nwt - w0 + W - 1) / W : 0;
    for (int k = 0; k < D - 1; k++)
        if ((uint64_t)k < nmine) issue(w0 + k * W, k);
    for (uint64_t i = 0; i < nmine; i++) {
        const uint64_t nx = i + D - 1;
        if (nx < nmine) {
            issue(w0 + nx * W, (int)(nx % D));
            // tile i landed; D-1 tiles (4 loads each) still in flight; the
            // record stores in between count too, so wait for the loads by
            // draining to the in-flight load count plus this wave's stores
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (D - 1)) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const uint32_t *buf = ring + (i % D) * 1024 + lane * 16;
        const uint32_t w3 = buf[3], w6 = buf[6], w7 = buf[7], w8 = buf[8];
        const uint64_t q = (w0 + i * W) * 64 + lane;
        u32x2 r;
        r.x = w3 ^ (w6 * 3u);
        r.y = w7 + w8;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads done before the slot is refilled
        if (q < n) __builtin_nontemporal_store(r, &out[q]);
    }
}

// Grid-stride with four 16-byte non-temporal loads in flight per lane before
// any is used (the guide's float4 copy shape, 6.29 TB/s for a 1:1 copy)
__global__ __launch_bounds__(256) void copy_mix_x4(const u32x4 *__restrict__ pk, u32x2 *__restrict__ out, uint64_t n16)
{
    const uint64_t step = (uint64_t)gridDim.x * 256;
    for (uint64_t i0 = blockIdx.x * 256ull + threadIdx.x; i0 < n16; i0 += 4 * step) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint64_t i = i0 + u * step;
            v[u] = i < n16 ? __builtin_nontemporal_load(&pk[i]) : u32x4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint64_t i = i0 + u * step;
            const uint32_t x = v[u].x ^ v[u].w;
            const uint32_t y = __shfl_xor(x, 1) + __shfl_xor(x, 2);
            if ((threadIdx.x & 3) == 0 && i < n16) {
                u32x2 r;
                r.x = x;
                r.y = y;
                __builtin_nontemporal_store(r, &out[i / 4]);
            }
        }
    }
}

}  // namespace

// Median over `iters` launches of the copy over n_slots 64-byte slots at
// grid = CUs * grid_mult workgroups. Returns 0 and *ms_out, or -1.
// pattern 0: copy_mix (grid-stride 16-byte loads); 1: ring_mix (LDS-DMA rings);
// 2: ring_mix_deep<4>; 3: ring_mix_deep<8>; 4: copy_mix_x4 (4 loads in flight per lane)
extern "C" int ceiling_pattern(const void *pkts, uint64_t n_slots, void *out, int pattern, int grid_mult, int iters,
                               float *ms_out);

extern "C" int ceiling_copy_mix(const void *pkts, uint64_t n_slots, void *out, int grid_mult, int iters,
                                float *ms_out)
{
    return ceiling_pattern(pkts, n_slots, out, 0, grid_mult, iters, ms_out);
}

extern "C" int ceiling_pattern(const void *pkts, uint64_t n_slots, void *out, int pattern, int grid_mult, int iters,
                               float *ms_out)
{
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return -1;
    if (!pkts || !out || n_slots == 0 || iters < 1 || grid_mult < 1) return -1;
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return -1;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return -1;
    const uint32_t grid = (uint32_t)prop.multiProcessorCount * (uint32_t)grid_mult;
    std::vector<float> v;
    int rc = 0;
    for (int r = 0; r <= iters; r++) {
        (void)hipEventRecord(e0, s);
        if (pattern == 1)
            hipLaunchKernelGGL(ring_mix, dim3(grid), dim3(256), 4 * 2 * 4096, s, (const uint8_t *)pkts, (u32x2 *)out,
                               n_slots);
        else if (pattern == 2)
            hipLaunchKernelGGL(ring_mix_deep<4>, dim3(grid), dim3(256), 4 * 4 * 4096, s, (const uint8_t *)pkts,
                               (u32x2 *)out, n_slots);
        else if (pattern == 3)
            hipLaunchKernelGGL(ring_mix_deep<8>, dim3(grid), dim3(256), 4 * 8 * 4096, s, (const uint8_t *)pkts,
                               (u32x2 *)out, n_slots);
        else if (pattern == 4)
            hipLaunchKernelGGL(copy_mix_x4, dim3(grid), dim3(256), 0, s, (const u32x4 *)pkts, (u32x2 *)out,
                               n_slots * 4);
        else
            hipLaunchKernelGGL(copy_mix, dim3(grid), dim3(256), 0, s, (const u32x4 *)pkts, (u32x2 *)out, n_slots * 4);
        (void)hipEventRecord(e1, s);
        if (hipEventSynchronize(e1) != hipSuccess) {
            rc = -1;
            break;
        }
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (r > 0) v.push_back(ms);   // the first launch warms up
    }
    if (rc == 0 && hipGetLastError() != hipSuccess) rc = -1;
    if (rc == 0) {
        std::sort(v.begin(), v.end());
        *ms_out = v[v.size() / 2];
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipStreamDestroy(s);
    return rc;
}

// The box's random-probe ceiling for the pipeline's DIR-24-8 probe shape:
// uniformly random dword loads into `tables` tables of `entries` u32 each (the
// caller's buffers: the same sizes as the pipeline's tbl24s), 8 packets per
// lane with all their probes in flight (tools/probe_kernels.h). Median over
// `iters` launches; *gprobes_out = probes per second / 1e9. 0 or -1.
extern "C" int ceiling_probe(const void *t0, const void *t1, uint32_t entries, int tables, int iters,
                             float *gprobes_out)
{
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return -1;
    if (!t0 || (tables > 1 && !t1) || entries == 0 || (entries & (entries - 1)) || iters < 1) return -1;
    // shapes: 8 or 16 packets per lane in flight, 8 or 16 workgroups per
    // CU; the best is the ceiling
    const uint32_t ncu = (uint32_t)prop.multiProcessorCount;
    const int rounds = 4;
    uint32_t *out = nullptr;
    if (hipMalloc(&out, (size_t)ncu * 16 * 256 * 4) != hipSuccess) return -1;
    hipStream_t s;
    hipEvent_t e0, e1;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return -1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return -1;
    int rc = 0;
    float best = 0.f;
    for (int shape = 0; shape < 4 && rc == 0; shape++) {
        const int ppt = shape & 1 ? 16 : 8;
        const uint32_t grid = ncu * (shape & 2 ? 16u : 8u);
        std::vector<float> v;
        for (int r = 0; r <= iters; r++) {
            (void)hipEventRecord(e0, s);
            if (ppt == 16)
                hipLaunchKernelGGL(probek::probe_rand<16>, dim3(grid), dim3(256), 0, s, (const uint32_t *)t0,
                                   (const uint32_t *)(tables > 1 ? t1 : t0), entries, tables, rounds,
                                   (unsigned long long)r * 0x9E3779B97F4A7C15ull, out);
            else
                hipLaunchKernelGGL(probek::probe_rand<8>, dim3(grid), dim3(256), 0, s, (const uint32_t *)t0,
                                   (const uint32_t *)(tables > 1 ? t1 : t0), entries, tables, rounds,
                                   (unsigned long long)r * 0x9E3779B97F4A7C15ull, out);
            (void)hipEventRecord(e1, s);
            if (hipEventSynchronize(e1) != hipSuccess) {
                rc = -1;
                break;
            }
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (r > 0) v.push_back(ms);
        }
        if (rc == 0 && hipGetLastError() != hipSuccess) rc = -1;
        if (rc == 0) {
            std::sort(v.begin(), v.end());
            const double probes = (double)grid * 256 * ppt * (tables > 1 ? 2 : 1) * rounds;
            best = std::max(best, (float)(probes / (v[v.size() / 2] * 1e-3) / 1e9));
        }
    }
    if (rc == 0) *gprobes_out = best;
    (void)hipFree(out);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipStreamDestroy(s);
    return rc;
}
