// burst.hip — the floor of the driver's 20-step poll-mode post, without the
// pipeline (measurement tooling, not the product).
//
// 1280 resident workers (5 per CU, 256 threads, the poll-mode kernel's
// geometry) wait on a device flag raised by the last worker to arrive, then
// together read 20 batches of 65536 64-byte slots (80 MiB) with the
// pipeline's step loads (three 16-byte non-temporal loads per lane per 64
// packets, cop_device.h load_step), fold the header words, and write an
// 8-byte record per slot (write-through, as the poll-mode kernel does).
// Each worker drains its stores and stamps s_memrealtime; the span from the
// flag to the last stamp is the burst's floor for that work mapping:
//   mode 0  worker w reads its own contiguous 64 KiB tile (4 steps of 256
//           packets: the poll-mode kernel's tile mapping today)
//   mode 1  step k of worker w is the 256-packet segment k*G + w: the whole
//           grid sweeps the pool in address order, step by step
//   mode 2  mode 0 without records (loads only)
//   mode 3  mode 1 without records
//   mode 4  mode 0 with a workgroup barrier after every step (tile_steps' per-step barrier)
//   mode 5  mode 0, and a finished worker polls one of 8 relay lines 128 B apart plus one
//           word shared by all (agent-scope loads, the poll-mode kernel's waiting loop today:
//           ~0.4 us apart) until the last finisher raises the lines
//   mode 6  mode 5 without the shared word
//   mode 7  mode 6 with 64 relay lines 4160 B apart
//   mode 8  XCD-local relay lines (one per XCD, raised by a plain store from that XCD once
//           every worker has finished) polled with non-temporal loads
//   mode 9  the same with sc0 buffer loads; mode 10: buffer_inv sc0, then a plain load
//   modes 11/12/13: mode 6 polling every ~1 / ~2 / ~4 us
//   mode 14 mode 0 + one returning atomic add per worker on one word, after the drain
//   mode 15 the same on 20 words (one per batch: 64 adds each) 8 bytes apart (two lines)
//   mode 16 mode 15 with the words 4160 bytes apart; mode 17: mode 16 without the return
//   mode 18 mode 0 + the pipeline's counter flush (9 non-returning u64 adds into 256 packed shard lines)
// Prints per mode the median over 15 bursts of: span (us), the p50 and p90
// worker finish (us after the flag), and the finish by worker slot on the
// CU (blockIdx / 256).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CHK(x)                                                                   \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            printf("%s: %s\n", #x, hipGetErrorString(e));                        \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int G = 1280, STEPS = 4, SEG = 256, NB = 20, B = 65536;

__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memrealtime(); }

template <int MODE>
__global__ __launch_bounds__(256, 5) void burst(const uint8_t *__restrict__ pool, unsigned long long *__restrict__ rec,
                                               uint32_t *ctl, unsigned long long *stamps)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ uint32_t go;
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 7u;
    if (tid == 0) {
        atomicAdd(&ctl[16 + xcc], 1u);   // workers per XCD
        // census: the last arriver raises the flag (and stamps it)
        if (atomicAdd(&ctl[0], 1u) == G - 1) {
            stamps[G] = now();
            __hip_atomic_store(&ctl[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // bounded: a worker that never became resident must not hang the grid
        for (uint32_t spins = 0; !__hip_atomic_load(&ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); spins++) {
            if (spins > (1u << 22)) {
                atomicOr(&ctl[2], 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        go = 1;
    }
    __syncthreads();
    (void)go;
    uint32_t lpk[3], lch[3];
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const uint32_t q = (uint32_t)(c * 64 + lane);
        lpk[c] = q / 3u;
        lch[c] = (q % 3u) * 16u;
    }
    u32x4 v[STEPS][3];
    uint32_t segs[STEPS];
#pragma unroll
    for (int k = 0; k < STEPS; k++) {
        const uint32_t s = (MODE & 1) ? (uint32_t)(k * G + blockIdx.x) : (uint32_t)(blockIdx.x * STEPS + k);
        segs[k] = s;
        const uint8_t *base = pool + ((size_t)s * SEG + wave * 64) * 64;
#pragma unroll
        for (int c = 0; c < 3; c++) v[k][c] = __builtin_nontemporal_load((const u32x4 *)(base + lpk[c] * 64 + lch[c]));
    }
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < STEPS; k++) {
        uint32_t x = 0;
#pragma unroll
        for (int c = 0; c < 3; c++) x ^= v[k][c].x ^ v[k][c].y ^ v[k][c].z ^ v[k][c].w;
        if (MODE < 2 || MODE >= 4) {   // records
            const size_t i = (size_t)segs[k] * SEG + tid;
            __hip_atomic_store(&rec[i], ((unsigned long long)x << 32) | i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            acc ^= x;
        }
        if (MODE == 4) __syncthreads();
    }
    if (MODE >= 2 && acc == 0x9E3779B9u) rec[tid] = acc;   // keeps the loads
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (MODE == 18 && tid < 9) {
        // the pipeline's counter flush: nine non-returning u64 adds into one
        // of 256 counter shards, 128-byte lines packed one after another
        unsigned long long *sh = (unsigned long long *)(ctl + 65536);
        __hip_atomic_fetch_add(&sh[(blockIdx.x % 256) * 16 + tid], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (MODE >= 14 && MODE <= 17 && tid == 0) {
        // completion counting after the drain, as the poll-mode kernel's tiles do
        uint32_t *w = MODE == 14 ? &ctl[3] : MODE == 15 ? &ctl[64 + 2 * (blockIdx.x / 64)] : &ctl[2048 + 1040 * (blockIdx.x / 64)];
        if (MODE == 17) __hip_atomic_fetch_add(w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else if (atomicAdd(w, 1u) == 0xFFFFFFFFu) rec[0] = 0;
    }
    if (tid == 0) stamps[blockIdx.x] = now();
    if (((MODE >= 5 && MODE <= 7) || (MODE >= 11 && MODE <= 13)) && tid == 0) {
        // the last finisher raises every relay line; the others poll theirs
        // (plus, mode 5, one word shared by every poller, as the poll-mode
        // kernel's exit word) with the waiting loop's backoff
        const uint32_t nl = MODE == 7 ? 64u : 8u, gap = MODE == 7 ? 1040u : 32u;   // u32 words apart
        const int backoff = MODE == 11 ? 9 : MODE == 12 ? 18 : MODE == 13 ? 36 : 3;   // s_sleep(4) ~0.107 us each
        uint32_t *lines = ctl + 1024;
        if (atomicAdd(&ctl[3], 1u) == G - 1) {
            for (uint32_t l = 0; l < nl; l++) __hip_atomic_store(&lines[l * gap], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        uint32_t *line = lines + (blockIdx.x % nl) * gap;
        for (uint32_t spins = 0;; spins++) {
            const uint32_t a = __hip_atomic_load(line, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t d = MODE == 5 ? __hip_atomic_load(&ctl[4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
            if (a + d) break;
            if (spins > (1u << 18)) {
                atomicOr(&ctl[2], 2u);
                break;
            }
            for (int k = spins < 16 ? 0 : backoff; k; k--) __builtin_amdgcn_s_sleep(4);
            __builtin_amdgcn_s_sleep(2);
        }
    }
    if (MODE >= 8 && MODE <= 10 && tid == 0) {
        // XCD-local relays: the last finisher on each XCD waits (agent-scope
        // loads, one poller per XCD) for every worker, then raises its XCD's
        // line with a plain store (into that XCD's L2); the others poll their
        // XCD's line with loads that miss L1 but may hit L2:
        //   mode 8: non-temporal loads; 9: sc0 buffer loads; 10: buffer_inv sc0 + plain load
        uint32_t *line = ctl + 1024 + xcc * 1040u;
        atomicAdd(&ctl[3], 1u);
        const bool last = atomicAdd(&ctl[32 + xcc], 1u) + 1u == __hip_atomic_load(&ctl[16 + xcc], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (uint32_t spins = 0;; spins++) {
            uint32_t a;
            if (last) a = __hip_atomic_load(&ctl[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= G;
            else if (MODE == 8) a = __builtin_nontemporal_load(line);
            else if (MODE == 9) a = __builtin_amdgcn_raw_buffer_load_b32(__builtin_amdgcn_make_buffer_rsrc(line, 0, 0x7FFFFFFF, 0x00020000), 0, 0, 1);
            else {
                asm volatile("buffer_inv sc0" ::: "memory");
                a = *(const uint32_t *)line;
                asm volatile("" ::: "memory");
            }
            if (a) {
                if (last) *line = 1u;
                break;
            }
            if (spins > (1u << 18)) {
                atomicOr(&ctl[2], 2u);
                break;
            }
            for (int k = spins < 16 ? 0 : 3; k; k--) __builtin_amdgcn_s_sleep(4);
            __builtin_amdgcn_s_sleep(2);
        }
    }
}

int main()
{
    int per_cu = 0;
    CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, burst<0>, 256, 0));
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    printf("CUs %d, workers per CU admitted %d (need 5)\n", prop.multiProcessorCount, per_cu);
    if (per_cu < 5 || prop.multiProcessorCount * 5 < G) return 1;
    const size_t pool_bytes = (size_t)NB * B * 64;
    const size_t pool_n = 8;   // rotate over 8 pools (640 MiB > Infinity Cache)
    uint8_t *pool;
    unsigned long long *rec, *stamps;
    uint32_t *ctl;
    CHK(hipMalloc(&pool, pool_bytes * pool_n));
    CHK(hipMemset(pool, 0x5A, pool_bytes * pool_n));
    CHK(hipMalloc(&rec, (size_t)NB * B * 8));
    CHK(hipMalloc(&stamps, (G + 1) * 8));
    CHK(hipMalloc(&ctl, 1 << 20));
    std::vector<unsigned long long> h(G + 1);
    for (int mode = 0; mode < 19; mode++) {
        if (mode == 5 || (mode >= 7 && mode <= 13) || mode == 1 || mode == 3 || mode == 4) continue;   // measured: profiles/r03/burst
        std::vector<double> span, p50, p90, slot[5];
        for (int it = 0; it < 17; it++) {
            CHK(hipMemset(ctl, 0, 1 << 20));
            const uint8_t *pp = pool + (size_t)(it % pool_n) * pool_bytes;
            if (mode == 0) hipLaunchKernelGGL(burst<0>, dim3(G), dim3(256), 0, 0, pp, rec, ctl, stamps);
            if (mode == 1) hipLaunchKernelGGL(burst<1>, dim3(G), dim3(256), 0, 0, pp, rec, ctl, stamps);
            if (mode == 2) hipLaunchKernelGGL(burst<2>, dim3(G), dim3(256), 0, 0, pp, rec, ctl, stamps);
            if (mode == 3) hipLaunchKernelGGL(burst<3>, dim3(G), dim3(256), 0, 0, pp, rec, ctl, stamps);
            if (mode == 4) hipLaunchKernelGGL(burst<4>, dim3(G), dim3(256), 0, 0, pp, rec, ctl, stamps);
            if (mode == 5) hipLaunchKernelGGL(burst<5>, dim3(G), dim3(256), 0, 0, pp, rec, ctl, stamps);
            if (mode == 6) hipLaunchKernelGGL(burst<6>, dim3(G), dim3(256), 0, 0, pp, rec, ctl, stamps);
            if (mode == 7) hipLaunchKernelGGL(burst<7>, dim3(G), dim3(256), 0, 0, pp, rec, ctl, stamps);
            if (mode == 8) hipLaunchKernelGGL(burst<8>, dim3(G), dim3(256), 0, 0, pp, rec, ctl, stamps);
            if (mode == 9) hipLaunchKernelGGL(burst<9>, dim3(G), dim3(256), 0, 0, pp, rec, ctl, stamps);
            if (mode == 10) hipLaunchKernelGGL(burst<10>, dim3(G), dim3(256), 0, 0, pp, rec, ctl, stamps);
            if (mode == 11) hipLaunchKernelGGL(burst<11>, dim3(G), dim3(256), 0, 0, pp, rec, ctl, stamps);
            if (mode == 12) hipLaunchKernelGGL(burst<12>, dim3(G), dim3(256), 0, 0, pp, rec, ctl, stamps);
            if (mode == 13) hipLaunchKernelGGL(burst<13>, dim3(G), dim3(256), 0, 0, pp, rec, ctl, stamps);
            if (mode == 14) hipLaunchKernelGGL(burst<14>, dim3(G), dim3(256), 0, 0, pp, rec, ctl, stamps);
            if (mode == 15) hipLaunchKernelGGL(burst<15>, dim3(G), dim3(256), 0, 0, pp, rec, ctl, stamps);
            if (mode == 16) hipLaunchKernelGGL(burst<16>, dim3(G), dim3(256), 0, 0, pp, rec, ctl, stamps);
            if (mode == 17) hipLaunchKernelGGL(burst<17>, dim3(G), dim3(256), 0, 0, pp, rec, ctl, stamps);
            if (mode == 18) hipLaunchKernelGGL(burst<18>, dim3(G), dim3(256), 0, 0, pp, rec, ctl, stamps);
            CHK(hipGetLastError());
            CHK(hipDeviceSynchronize());
            CHK(hipMemcpy(h.data(), stamps, (G + 1) * 8, hipMemcpyDeviceToHost));
            uint32_t hc[4];
            CHK(hipMemcpy(hc, ctl, 16, hipMemcpyDeviceToHost));
            if (hc[2] & 1u) {
                printf("census timed out: not every worker resident\n");
                return 1;
            }
            if (hc[2] & 2u) {
                printf("mode %d: a relay poll never saw its line (stale cache): timed out\n", mode);
                break;
            }
            if (it < 2) continue;
            std::vector<double> fin(G);
            for (int w = 0; w < G; w++) fin[w] = (double)(long long)(h[w] - h[G]) / 100.0;   // 100 MHz
            std::vector<double> s = fin;
            std::sort(s.begin(), s.end());
            span.push_back(s[G - 1]);
            p50.push_back(s[G / 2]);
            p90.push_back(s[G * 9 / 10]);
            for (int r = 0; r < 5; r++) {
                std::vector<double> t(fin.begin() + r * 256, fin.begin() + (r + 1) * 256);
                std::sort(t.begin(), t.end());
                slot[r].push_back(t[128]);
            }
        }
        if (span.empty()) continue;
        auto med = [](std::vector<double> x) {
            std::sort(x.begin(), x.end());
            return x[x.size() / 2];
        };
        printf("mode %d: span %.2f us (%.2f TB/s of slot bytes), p50 %.2f, p90 %.2f; by CU slot:", mode, med(span),
               pool_bytes / med(span) / 1e6, med(p50), med(p90));
        for (int r = 0; r < 5; r++) printf(" %.2f", med(slot[r]));
        printf("\n");
    }
    return 0;
}
