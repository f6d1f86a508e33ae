// ceiling.hip — the box's streaming ceiling for the pipeline's byte mix.
//
// Reads every 64-byte packet slot of a pool once (coalesced non-temporal
// 16-byte loads, grid-stride) and writes one 8-byte record per slot
// (non-temporal): the 72 B/packet of the bench's algorithmic bytes with no
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

}  // namespace

// Median over `iters` launches of the copy over n_slots 64-byte slots at
// grid = CUs * grid_mult workgroups. Returns 0 and *ms_out, or -1.
extern "C" int ceiling_copy_mix(const void *pkts, uint64_t n_slots, void *out, int grid_mult, int iters,
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
