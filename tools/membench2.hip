// membench2.hip — steady-state read patterns for the pipeline's byte mix
// (64 B packet slot read, 8 B record written per packet) at a size far
// beyond the Infinity Cache (24 Mi packets = 1.5 GiB), so launch ramp/tail
// and MALL hits do not flatter any variant.
//   A  one-shot grid, strided header loads per lane (the pipeline today)
//   P  persistent grid, static tile order, next tile's loads in registers
//      while the current tile is processed (compiler-counted waits)
//   L  persistent grid, per-wave LDS-DMA ring of D x 4 KiB (64 slots),
//      counted vmcnt, fields read from LDS
//   Q  persistent grid, coalesced dwordx4 (4 lanes per slot), quad DPP
//      gather of the fields into the slot's first lane, then bpermute
//   D  dwordx4 grid-stride read only (roofline reference)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/membench2 tools/membench2.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include <string.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x2 rec(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    u32x2 r; r.x = a ^ (b * 3u) ^ (c * 5u); r.y = d + a; return r;
}

template <bool NT>
__device__ __forceinline__ uint32_t ld32(const uint8_t *p) {
    if (NT) return __builtin_nontemporal_load((const uint32_t *)p);
    return *(const uint32_t *)p;
}
template <bool NT>
__device__ __forceinline__ u32x2 ld64(const uint8_t *p) {
    if (NT) return __builtin_nontemporal_load((const u32x2 *)p);
    return *(const u32x2 *)p;
}

__global__ void kFill(uint32_t *p, uint64_t nw) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nw; i += (uint64_t)gridDim.x * 256) {
        uint64_t x = i * 0x9E3779B97F4A7C15ull; x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32;
        p[i] = (uint32_t)x;
    }
}

template <int PPT, bool NT = false>
__global__ __launch_bounds__(256) void kA(const uint8_t *__restrict__ pk, u32x2 *__restrict__ out, uint32_t n) {
    const uint32_t base = blockIdx.x * 256 * PPT;
    uint32_t w3[PPT], w6[PPT], w7[PPT], w8[PPT];
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        uint32_t i = min(base + k * 256 + threadIdx.x, n - 1);
        const uint8_t *p = pk + (size_t)i * 64;
        w3[k] = ld32<NT>(p + 12);
        u32x2 v = ld64<NT>(p + 24);
        w6[k] = v.x; w7[k] = v.y;
        w8[k] = ld32<NT>(p + 32);
    }
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        uint32_t i = base + k * 256 + threadIdx.x;
        if (i < n) __builtin_nontemporal_store(rec(w3[k], w6[k], w7[k], w8[k]), &out[i]);
    }
}

// persistent, static tiles g, g+G, ...; tile = 256*PPT slots
template <int PPT, bool NT = false>
__global__ __launch_bounds__(256) void kP(const uint8_t *__restrict__ pk, u32x2 *__restrict__ out, uint32_t n) {
    const uint32_t ntiles = (n + 256 * PPT - 1) / (256 * PPT);
    uint32_t a3[PPT], a6[PPT], a7[PPT], a8[PPT];
    auto load = [&](uint32_t t) {
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            uint32_t i = min(t * 256 * PPT + k * 256 + threadIdx.x, n - 1);
            const uint8_t *p = pk + (size_t)i * 64;
            a3[k] = ld32<NT>(p + 12);
            u32x2 v = ld64<NT>(p + 24);
            a6[k] = v.x; a7[k] = v.y;
            a8[k] = ld32<NT>(p + 32);
        }
    };
    uint32_t t = blockIdx.x;
    if (t >= ntiles) return;
    load(t);
    for (;;) {
        uint32_t c3[PPT], c6[PPT], c7[PPT], c8[PPT];
#pragma unroll
        for (int k = 0; k < PPT; k++) { c3[k] = a3[k]; c6[k] = a6[k]; c7[k] = a7[k]; c8[k] = a8[k]; }
        const uint32_t tn = t + gridDim.x;
        if (tn < ntiles) load(tn);
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            uint32_t i = t * 256 * PPT + k * 256 + threadIdx.x;
            if (i < n) __builtin_nontemporal_store(rec(c3[k], c6[k], c7[k], c8[k]), &out[i]);
        }
        if (tn >= ntiles) break;
        t = tn;
    }
}

// persistent per-wave LDS-DMA ring: wave-tile = 64 slots (4 KiB, 4 glds),
// D buffers per wave; wave-tiles w, w+W, ... (W = total waves)
template <int D, int AUX>
__global__ __launch_bounds__(256) void kL(const uint8_t *__restrict__ pk, u32x2 *__restrict__ out, uint32_t n) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t *ring = lds + wave * D * 1024;
    const uint32_t nwt = (n + 63) / 64;
    const uint32_t W = gridDim.x * 4;
    const uint32_t w0 = blockIdx.x * 4 + wave;
    auto issue = [&](uint32_t wt, int slot) {
        uint32_t *dst = ring + slot * 1024;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t byte = (c * 64 + lane) * 16;
            const uint32_t q = min(wt * 64 + byte / 64, n - 1);
            const uint8_t *src = pk + (size_t)q * 64 + (byte & 63);
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                             (__attribute__((address_space(3))) void *)(dst + c * 256), 16, 0, AUX);
        }
    };
    // prologue: D-1 tiles in flight
    uint32_t nmine = w0 < nwt ? (nwt - w0 + W - 1) / W : 0;
#pragma unroll
    for (int s = 0; s < D - 1; s++)
        if ((uint32_t)s < nmine) issue(w0 + s * W, s);
    for (uint32_t i = 0; i < nmine; i++) {
        if (i + D - 1 < nmine) {
            issue(w0 + (i + D - 1) * W, (i + D - 1) % D);
            // wait for tile i: leave the later (D-1) tiles' glds in flight
            if (D == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            if (D == 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            if (D == 4) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
            if (D == 6) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
            if (D == 8) asm volatile("s_waitcnt vmcnt(28)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const uint32_t *buf = ring + (i % D) * 1024 + lane * 16;
        const uint32_t w3 = buf[3];
        const uint2 v67 = *(const uint2 *)(buf + 6);
        const uint32_t w8 = buf[8];
        const uint32_t q = (w0 + i * W) * 64 + lane;
        if (q < n) __builtin_nontemporal_store(rec(w3, v67.x, v67.y, w8), &out[q]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads done before the slot is refilled
    }
}

// persistent, coalesced: wave-tile = 64 slots read as 4 x dwordx4 per lane
// (instruction c: slot 16c + lane/4, chunk lane%4), fields moved to the
// slot's lane by ds_bpermute
template <int TPW, bool NT = false>
__global__ __launch_bounds__(256) void kQ(const uint8_t *__restrict__ pk, u32x2 *__restrict__ out, uint32_t n) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t nwt = (n + 63) / 64;
    const uint32_t W = gridDim.x * 4;
    const uint32_t w0 = blockIdx.x * 4 + wave;
    uint4 cur[TPW][4];
    auto load = [&](uint32_t wt, uint4 (&v)[4]) {
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t q = min(wt * 64 + c * 16 + lane / 4, n - 1);
            const u32x4 *a = (const u32x4 *)(pk + (size_t)q * 64 + (lane & 3) * 16);
            const u32x4 t = NT ? __builtin_nontemporal_load(a) : *a;
            v[c] = make_uint4(t.x, t.y, t.z, t.w);
        }
    };
    for (uint32_t wt = w0; wt < nwt; wt += W * TPW) {
#pragma unroll
        for (int u = 0; u < TPW; u++) load(min(wt + u * W, nwt - 1), cur[u]);
#pragma unroll
        for (int u = 0; u < TPW; u++) {
            // slot p = lane: source lanes 4*(p%16)+{0,1,2} of instruction p/16
            const int src0 = ((lane & 15) * 4) << 2;
            uint32_t f3 = 0, f6 = 0, f7 = 0, f8 = 0;
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const uint32_t a = __builtin_amdgcn_ds_bpermute(src0, cur[u][c].w);
                const uint32_t b = __builtin_amdgcn_ds_bpermute(src0 + 4, cur[u][c].z);
                const uint32_t d = __builtin_amdgcn_ds_bpermute(src0 + 4, cur[u][c].w);
                const uint32_t e = __builtin_amdgcn_ds_bpermute(src0 + 8, cur[u][c].x);
                if ((lane >> 4) == c) { f3 = a; f6 = b; f7 = d; f8 = e; }
            }
            const uint32_t q = (wt + u * W) * 64 + lane;
            if (wt + u * W < nwt && q < n) __builtin_nontemporal_store(rec(f3, f6, f7, f8), &out[q]);
        }
    }
}

template <bool NT = false>
__global__ __launch_bounds__(256) void kD(const u32x4 *__restrict__ pk, uint32_t *__restrict__ out, uint64_t n16) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        u32x4 v = NT ? __builtin_nontemporal_load(&pk[i]) : pk[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int U>
__global__ __launch_bounds__(256) void kS(const u32x4 *__restrict__ pk, u32x2 *__restrict__ out, uint32_t n) {
    // grid-stride over 16-byte chunks, U per lane in flight; lane%4==0 writes
    // the slot's 8 B record (the byte mix's ceiling, no field gathering)
    const uint64_t n16 = (uint64_t)n * 4;
    const uint64_t step = (uint64_t)gridDim.x * 256;
    for (uint64_t i0 = blockIdx.x * 256ull + threadIdx.x; i0 < n16; i0 += step * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = __builtin_nontemporal_load(&pk[min(i0 + u * step, n16 - 1)]);
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t x = v[u].x ^ v[u].w;
            const uint32_t y = __shfl_xor(x, 1) + __shfl_xor(x, 2);
            const uint64_t i = i0 + u * step;
            if ((threadIdx.x & 3) == 0 && i < n16) { u32x2 r; r.x = x; r.y = y; __builtin_nontemporal_store(r, &out[i / 4]); }
        }
    }
}

int main(int argc, char **argv) {
    const uint32_t n = 24u << 20;             // 24 Mi slots = 1.5 GiB
    int dev = 0; hipDeviceProp_t prop; CHK(hipGetDeviceProperties(&prop, dev));
    const int cus = prop.multiProcessorCount;
    printf("device %s, %d CUs\n", prop.name, cus);
    uint8_t *pk; u32x2 *out;
    CHK(hipMalloc(&pk, (size_t)n * 64));
    CHK(hipMalloc(&out, (size_t)n * 8 + (1 << 24)));
    hipLaunchKernelGGL(kFill, dim3(4096), dim3(256), 0, 0, (uint32_t *)pk, (uint64_t)n * 16);
    // a second buffer READ between runs to evict the Infinity Cache without
    // leaving dirty lines behind
    uint8_t *flush; const size_t fl = 512u << 20;
    CHK(hipMalloc(&flush, fl));
    CHK(hipMemset(flush, 1, fl));
    uint32_t *sink; CHK(hipMalloc(&sink, 4096 * 256 * 4));
    std::vector<u32x2> ref(n), got(n);
    hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    bool have_ref = false;
    auto timeit = [&](const char *name, auto launch, double bytes, bool check = true) {
        std::vector<float> v;
        for (int r = 0; r < 7; r++) {
            hipLaunchKernelGGL(kD<false>, dim3(2048), dim3(256), 0, 0, (const u32x4 *)flush, sink, (uint64_t)fl / 16);
            CHK(hipMemsetAsync(out, 0, (size_t)n * 8, 0));
            hipLaunchKernelGGL(kD<false>, dim3(2048), dim3(256), 0, 0, (const u32x4 *)flush, sink, (uint64_t)fl / 16);
            CHK(hipEventRecord(e0)); launch(); CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
            float ms; CHK(hipEventElapsedTime(&ms, e0, e1)); v.push_back(ms);
        }
        CHK(hipGetLastError());
        std::sort(v.begin(), v.end());
        float med = v[v.size() / 2];
        const char *ok = "";
        if (check) {
            CHK(hipMemcpy(have_ref ? got.data() : ref.data(), out, (size_t)n * 8, hipMemcpyDeviceToHost));
            if (!have_ref) { have_ref = true; ok = "(ref)"; }
            else ok = memcmp(ref.data(), got.data(), (size_t)n * 8) == 0 ? "ok" : "MISMATCH";
        }
        printf("%-34s %8.1f us  %7.0f GB/s  %s\n", name, med * 1e3, bytes / (med * 1e-3) / 1e9, ok);
        fflush(stdout);
    };
    const double alg = 72.0 * n;
    char nm[64];
    timeit("A one-shot strided ppt8", [&] { hipLaunchKernelGGL((kA<8>), dim3(n / 2048), dim3(256), 0, 0, pk, out, n); }, alg);
    timeit("L glds D2 nt grid 2xCU", [&] { hipLaunchKernelGGL((kL<2, 2>), dim3(cus * 2), dim3(256), 4 * 2 * 4096, 0, pk, out, n); }, alg);
    timeit("L glds D4 nt grid 2xCU", [&] { hipLaunchKernelGGL((kL<4, 2>), dim3(cus * 2), dim3(256), 4 * 4 * 4096, 0, pk, out, n); }, alg);
    timeit("L glds D2 nt grid 3xCU", [&] { hipLaunchKernelGGL((kL<2, 2>), dim3(cus * 3), dim3(256), 4 * 2 * 4096, 0, pk, out, n); }, alg);
    for (int m : {2, 4, 8, 16}) {
        snprintf(nm, sizeof nm, "Q nt tpw1 grid %dxCU", m);
        timeit(nm, [&] { hipLaunchKernelGGL((kQ<1, true>), dim3(cus * m), dim3(256), 0, 0, pk, out, n); }, alg);
        snprintf(nm, sizeof nm, "Q nt tpw2 grid %dxCU", m);
        timeit(nm, [&] { hipLaunchKernelGGL((kQ<2, true>), dim3(cus * m), dim3(256), 0, 0, pk, out, n); }, alg);
        snprintf(nm, sizeof nm, "Q nt tpw4 grid %dxCU", m);
        timeit(nm, [&] { hipLaunchKernelGGL((kQ<4, true>), dim3(cus * m), dim3(256), 0, 0, pk, out, n); }, alg);
    }
    for (int m : {4, 8, 16}) {
        snprintf(nm, sizeof nm, "S stream+rec U1 grid %dxCU", m);
        timeit(nm, [&] { hipLaunchKernelGGL((kS<1>), dim3(cus * m), dim3(256), 0, 0, (const u32x4 *)pk, out, n); }, alg, false);
        snprintf(nm, sizeof nm, "S stream+rec U4 grid %dxCU", m);
        timeit(nm, [&] { hipLaunchKernelGGL((kS<4>), dim3(cus * m), dim3(256), 0, 0, (const u32x4 *)pk, out, n); }, alg, false);
    }
    for (int g : {2048}) {
        snprintf(nm, sizeof nm, "D stream dwordx4 nt read g=%d", g);
        timeit(nm, [&] { hipLaunchKernelGGL(kD<true>, dim3(g), dim3(256), 0, 0, (const u32x4 *)pk, (uint32_t *)out, (uint64_t)n * 4); }, 64.0 * n, false);
    }
    return 0;
}
