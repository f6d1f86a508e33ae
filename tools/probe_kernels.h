// probe_kernels.h — random 4-byte table probes with a known probe count
// (measurement tooling, not the product). Shared by tools/ceiling.hip
// (bench.py's same-box random-probe ceiling) and tools/probebench.hip (the
// FETCH_SIZE calibration of isolated dword probes, SURVEY.md §8d: LPM probes
// are reported per packet beside the streaming bytes).
#ifndef PROBE_KERNELS_H
#define PROBE_KERNELS_H

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace probek {

__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// The pipeline's probe shape (DIR-24-8 tbl24 lookups of config 5): each lane
// handles PPT packets and issues, per packet, one dword load into each of
// `tables` tables of `entries` u32 (a power of two) at uniformly random
// indices, all PPT*tables loads in flight before any is used. Probes per
// launch = grid * 256 * PPT * tables * rounds. One u32 per lane is written.
template <int PPT>
__global__ __launch_bounds__(256) void probe_rand(const uint32_t *__restrict__ t0, const uint32_t *__restrict__ t1,
                                                  uint32_t entries, int tables, int rounds, uint64_t seed,
                                                  uint32_t *__restrict__ out)
{
    const uint64_t gid = blockIdx.x * 256ull + threadIdx.x;
    uint32_t acc = 0;
    for (int r = 0; r < rounds; r++) {
        uint32_t v0[PPT], v1[PPT];
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            const uint64_t h = mix64(seed ^ (gid * 64 + (uint64_t)r * PPT + k));
            v0[k] = t0[(uint32_t)h & (entries - 1)];
            v1[k] = tables > 1 ? t1[(uint32_t)(h >> 32) & (entries - 1)] : 0u;
        }
#pragma unroll
        for (int k = 0; k < PPT; k++) acc ^= v0[k] + v1[k];
    }
    out[gid] = acc;
}

// Request-size probe: each lane picks a random 128-byte line, loads one dword
// at byte `a` of it, waits for it, then loads one dword at byte `b` of the
// same line. With (a, b) = (0, 64) the second load hits in L2 only if the
// first miss filled the whole 128-byte line; with (0, 32) it always hits (the
// same 64-byte half). Fabric read requests per lane (TCC_EA0_RDREQ) then tell
// the fill granularity of an isolated probe.
__global__ __launch_bounds__(256) void probe_pair(const uint32_t *__restrict__ t, uint32_t lines, uint32_t a,
                                                  uint32_t b, uint64_t seed, uint32_t *__restrict__ out)
{
    const uint64_t gid = blockIdx.x * 256ull + threadIdx.x;
    const uint32_t line = (uint32_t)mix64(seed ^ gid) & (lines - 1);
    const uint32_t *p = t + (size_t)line * 32;
    const uint32_t x = p[a / 4];   // a plain load, as the pipeline's tbl24 probe
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // an L1-bypassing (sc1) load: answered by L2, or by the fabric on a miss
    const uint32_t y = __hip_atomic_load(p + b / 4 + (x & 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    out[gid] = x ^ y;
}

// Both loads of the pair issued back to back (plain loads, as the
// pipeline's probes), then used: a second load into the same line while the
// first miss is outstanding merges with it if the fill covers both offsets.
__global__ __launch_bounds__(256) void probe_pair_sim(const uint32_t *__restrict__ t, uint32_t lines, uint32_t a,
                                                      uint32_t b, uint64_t seed, uint32_t *__restrict__ out)
{
    const uint64_t gid = blockIdx.x * 256ull + threadIdx.x;
    const uint32_t line = (uint32_t)mix64(seed ^ gid) & (lines - 1);
    const uint32_t *p = t + (size_t)line * 32;
    const uint32_t x = p[a / 4], y = p[b / 4];
    out[gid] = x ^ y;
}

}  // namespace probek

#endif
