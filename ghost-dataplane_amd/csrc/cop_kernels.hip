// cop_kernels.hip — the coprocessor NF pipeline, one tile per workgroup.
//
// One lane handles PPT packets, one workgroup one tile of 256*PPT packets.
// Per packet the kernel restates the SURVEY.md §8a contract (cop_device.h:
// get_next_hop switch.c:93-136, fw_packet_handler firewall.c:170-213 with
// rte_lpm_lookup firewall.c:194, the route LPM stage, and the ordered
// forward list of coprocessor() switch.c:464-470).
//
// Data layout (HBM): packets at 16-byte aligned starts (64-byte slots or an
// IMIX slab + u32 offsets). Tables: the vport routing table as a two-level
// image (256-entry top + 256-entry u16 leaves); the firewall table keyed by
// matching rule id (entry = rule | hit<<24 | (action != 0)<<26, so the
// verdict and the per-rule hit counter come from one probe) and the route
// table keyed by next hop; LPM tables either as a
// flattened interval array (binary search in LDS) or as a DPDK-layout
// DIR-24-8 image (tbl24 64 MiB + tbl8 groups, HBM / Infinity Cache). Small
// tables are staged into LDS by LDS-DMA at workgroup start, overlapped with
// the ticket atomic and the packet loads.
//
// Ordered compaction across workgroups: wave64 ballot + mbcnt inside a
// tile, an LDS scan over (step, wave), then decoupled look-back over the
// tiles of the batch, 64 predecessors per round. Workgroups are assigned to
// batches statically (blockIdx ranges) but draw their tile index inside the
// batch from that batch's own ticket counter, so every predecessor a tile
// waits on is held by a workgroup that is already running (no residency
// assumption), and ticket atomics are spread over one counter per batch.
// Look-back words are 8-byte {epoch, flag, value} granules written and
// polled with agent-scope relaxed atomics (sc1): the data is the flag.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cop_device.h"
#include "cop_kernels.h"
#include "cop_tile.h"

namespace {

using namespace copd;

// experiment builds may raise the occupancy target (KDEFS=-DCOPK_WAVES_PER_EU=8)
#ifndef COPK_WAVES_PER_EU
#define COPK_WAVES_PER_EU 1
#endif
// LAY: COPK_LAY_SLOTS (per-lane header loads at any stride), COPK_LAY_IMIX
// (slab + offsets), COPK_LAY_COALESCED (strides >= 48: a wave's 64
// consecutive packets by three 16-byte non-temporal loads per lane,
// cop_device.h load_step / gather_step), COPK_LAY_HDR16 (packed 16-byte
// header records, one 16-byte load per packet: the end-to-end host path)
// EXT: the launch uses an optional feature (demux, port stats, per-rule
// counters, $COP_DBG ablations); without, their code is compiled out.
// The batch's ticket: a returning device-scope add, waited for inside the
// same asm block. As a plain atomicAdd its pending result register made the
// compiler put an s_waitcnt vmcnt(0) in front of the header loads on the
// ticket-free path too (one merged wait state for both paths), so every
// small launch's workgroups waited for their LDS-DMA table staging before
// loading a packet.
__device__ __forceinline__ __attribute__((unused)) unsigned long long ticket_take(unsigned long long *p)
{
    unsigned long long old;
    asm volatile("global_atomic_add_x2 %0, %1, %2, off sc0\n\ts_waitcnt vmcnt(0)"
                 : "=v"(old)
                 : "v"(p), "v"(1ull)
                 : "memory");
    return old;
}

// the bucketed route form at 4 packets per lane sits just above 96 VGPRs:
// held to 96, it runs 5 waves per SIMD instead of 4. Not with the bucketed
// firewall: held to 96 those parts spill (44-144 bytes per lane of scratch,
// -Rpass-analysis=kernel-resource-usage), so they keep 4 waves (103-123 VGPRs)
template <int FW, int LPM, int LAY, int PPT, bool EXT>
__global__ __launch_bounds__(BLOCK, EXT ? 4 : (LPM == COPK_TBL_BKT && FW != COPK_TBL_BKT && PPT == 4) ? 5 : COPK_WAVES_PER_EU) void
cop_pipeline(const CopKParams p)
{
    const Opt o = EXT ? opt_all(p) : Opt{0u, 0u, 0u, nullptr};
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const LdsCarve lc = lds_carve<PPT>(p, lds);

    STAMP(0);
    // ---- batch of this workgroup: static blockIdx ranges ----
    // Equal-size batches are interleaved over blockIdx (b = g mod nb), so
    // consecutive tiles of one batch are dispatched nb workgroups apart and a
    // tile's predecessors have normally published their counts by the time
    // its look-back reads them. Unequal batches: blockIdx ranges.
    const uint32_t g = blockIdx.x;
    // ---- stage tables into LDS by LDS-DMA first: the loads go out before
    // anything else is in flight (no wait in front of them), and land while
    // the ticket and the header loads are in flight ----
    if (!(o.dbg & 4u)) stage_tables<FW, LPM>(p, lc.tb, lane, wave);
    const bool ilv = p.uniform_ntiles != 0 && !(o.dbg & 256u);
    const uint32_t b = ilv ? __builtin_amdgcn_readfirstlane(g % p.nb) : batch_of_tile(p, g);
    uint32_t look_off;
    const CopKBatch B = batch_desc(p, b, &look_off);

    // ---- zero the lane's other ticket buffer for the next launch on this
    // lane (stream order puts that launch after this one completes) ----
    for (uint32_t line = g; line < p.zero_lines; line += gridDim.x)
        if (tid < 16) p.zero_tickets[line * 16 + tid] = 0ull;

    // ---- per-rule hit binning: zero the tile's bucket counts (ordered
    // before the first add by the barrier below or tile_body's) ----
    if (EXT && p.hit_region)
        for (uint32_t i = (uint32_t)tid; i < p.hit_nb; i += BLOCK) lds[p.lds_hit_off + i] = 0u;

    // ---- tile index inside the batch: this batch's ticket counter (or the
    // static order when no look-back runs: p.compact == 0) ----
    // (segmented lists need no cross-tile order: static too)
    const bool dyn = p.compact != 0 && !p.seg && !(o.dbg & 2u) && !p.static_order;
    unsigned long long tk = 0;
    if (dyn && tid == 0) tk = ticket_take(&p.tickets[b * 16]);

    uint32_t j;
    if (dyn) {
        if (tid == 0) *lc.s_tile = (uint32_t)tk;
        __syncthreads();
        j = __builtin_amdgcn_readfirstlane(*lc.s_tile);
    } else {
        j = ilv ? g / p.nb : p.uniform_ntiles ? g - b * p.uniform_ntiles : g - p.tile_begin[b];
    }
    STAMP(1);

    tile_body<FW, LPM, LAY, PPT, EXT, false>(p, o, lc, B, look_off, j, LookCtx{p.look, p.epoch, p.err}, tid, lane,
                                             wave, !dyn, blockIdx.x);
}

template <int FW, int LPM, int LAY, int PPT>
hipError_t launch_one(const CopKParams &p, uint32_t grid, uint32_t lds_bytes, hipStream_t s)
{
    const bool ext = p.demux || p.port_stats || p.rule_hits || p.dbg;
    if (ext) hipLaunchKernelGGL((cop_pipeline<FW, LPM, LAY, PPT, true>), dim3(grid), dim3(BLOCK), lds_bytes, s, p);
    else hipLaunchKernelGGL((cop_pipeline<FW, LPM, LAY, PPT, false>), dim3(grid), dim3(BLOCK), lds_bytes, s, p);
    return hipGetLastError();
}

template <int FW, int LPM, int LAY>
hipError_t launch_ppt(const CopKParams &p, int ppt, uint32_t grid, uint32_t lds, hipStream_t s)
{
    if (ppt == 8) return launch_one<FW, LPM, LAY, 8>(p, grid, lds, s);
    if (ppt == 4) return launch_one<FW, LPM, LAY, 4>(p, grid, lds, s);
    return launch_one<FW, LPM, LAY, 1>(p, grid, lds, s);
}

template <int FW, int LPM>
hipError_t launch_imix(const CopKParams &p, int lay, int ppt, uint32_t grid, uint32_t lds, hipStream_t s)
{
    if (lay == COPK_LAY_IMIX) return launch_ppt<FW, LPM, COPK_LAY_IMIX>(p, ppt, grid, lds, s);
    if (lay == COPK_LAY_COALESCED) return launch_ppt<FW, LPM, COPK_LAY_COALESCED>(p, ppt, grid, lds, s);
    if (lay == COPK_LAY_HDR16) return launch_ppt<FW, LPM, COPK_LAY_HDR16>(p, ppt, grid, lds, s);
    return launch_ppt<FW, LPM, COPK_LAY_SLOTS>(p, ppt, grid, lds, s);
}

template <int FW>
hipError_t launch_lpm(const CopKParams &p, int lpm, int imix, int ppt, uint32_t grid, uint32_t lds,
                      hipStream_t s)
{
    if constexpr (FW == COPK_TBL_BKT) {
        // the bucketed firewall (1M-rule tables) beside the large route forms
        // only: a route table small enough for LDS goes with a small firewall
        if (lpm == COPK_TBL_DIR) return launch_imix<FW, COPK_TBL_DIR>(p, imix, ppt, grid, lds, s);
        if (lpm == COPK_TBL_BKT) return launch_imix<FW, COPK_TBL_BKT>(p, imix, ppt, grid, lds, s);
        if (lpm == COPK_TBL_OFF) return launch_imix<FW, COPK_TBL_OFF>(p, imix, ppt, grid, lds, s);
        return hipErrorInvalidValue;   // fill_launch maps IVT / TRIE routes to DIR-24-8 here
    } else {
        if (lpm == COPK_TBL_IVT) return launch_imix<FW, COPK_TBL_IVT>(p, imix, ppt, grid, lds, s);
        if (lpm == COPK_TBL_DIR) return launch_imix<FW, COPK_TBL_DIR>(p, imix, ppt, grid, lds, s);
        if (lpm == COPK_TBL_TRIE) return launch_imix<FW, COPK_TBL_TRIE>(p, imix, ppt, grid, lds, s);
        if (lpm == COPK_TBL_BKT) return launch_imix<FW, COPK_TBL_BKT>(p, imix, ppt, grid, lds, s);
        return launch_imix<FW, COPK_TBL_OFF>(p, imix, ppt, grid, lds, s);
    }
}

} // namespace

// The kernel's instantiations are compiled in three parts, one per firewall
// table mode (COPK_FW_PART = 0, 1, 2: this file built three more times), so
// the build runs in parallel; the part-less build holds the dispatcher and
// the small kernels.
#define COPK_LAUNCH_ARGS const CopKParams *p, int lpm_mode, int imix, int ppt, uint32_t grid, uint32_t lds_bytes, \
                         hipStream_t stream
extern "C" hipError_t copk_launch_fw0(COPK_LAUNCH_ARGS);
extern "C" hipError_t copk_launch_fw1(COPK_LAUNCH_ARGS);
extern "C" hipError_t copk_launch_fw2(COPK_LAUNCH_ARGS);
extern "C" hipError_t copk_launch_fw4(COPK_LAUNCH_ARGS);
#if defined(COPK_FW_PART)
#define COPK_CAT2(a, b) a##b
#define COPK_CAT(a, b) COPK_CAT2(a, b)
extern "C" hipError_t COPK_CAT(copk_launch_fw, COPK_FW_PART)(COPK_LAUNCH_ARGS)
{
    return launch_lpm<COPK_FW_PART>(*p, lpm_mode, imix, ppt, grid, lds_bytes, stream);
}
#else
static_assert(COPK_TBL_OFF == 0 && COPK_TBL_IVT == 1 && COPK_TBL_DIR == 2 && COPK_TBL_BKT == 4, "part numbering");
extern "C" hipError_t copk_launch(const CopKParams *p, int fw_mode, int lpm_mode, int imix, int ppt,
                                  uint32_t grid, uint32_t lds_bytes, hipStream_t stream)
{
    if (fw_mode == COPK_TBL_IVT) return copk_launch_fw1(p, lpm_mode, imix, ppt, grid, lds_bytes, stream);
    if (fw_mode == COPK_TBL_DIR) return copk_launch_fw2(p, lpm_mode, imix, ppt, grid, lds_bytes, stream);
    if (fw_mode == COPK_TBL_BKT) return copk_launch_fw4(p, lpm_mode, imix, ppt, grid, lds_bytes, stream);
    return copk_launch_fw0(p, lpm_mode, imix, ppt, grid, lds_bytes, stream);
}

namespace {
// Per-rule hit counters from binned ids (CopKParams::hit_region): workgroup
// (q, s) counts bucket q's runs of the tiles in slice s into LDS counters,
// then adds every non-zero counter to rule_hits (contiguous adds, one per
// rule and slice). A lane's task is one chunk of up to HIT_CHUNK ids of one
// tile's run (chunks per run: `chunks`), loaded four 16-byte loads at a time;
// repeats of one id within a lane's loads are merged before the LDS add.
constexpr uint32_t HIT_R = 1u << COPK_HIT_SHIFT;
constexpr uint32_t HIT_CHUNK = 64;
__global__ __launch_bounds__(256) void cop_hit_count(const CopKParams p, uint32_t n_tiles, uint32_t slices,
                                                     uint32_t chunks)
{
    __shared__ uint32_t cnt[HIT_R];
    const uint32_t tid = threadIdx.x;
    const uint32_t q = blockIdx.x / slices, s = blockIdx.x % slices, nb = p.hit_nb;
    for (uint32_t i = tid; i < HIT_R; i += 256) cnt[i] = 0u;
    __syncthreads();
    const uint32_t per = (n_tiles + slices - 1) / slices;
    const uint32_t t0 = s * per, t1 = min(n_tiles, t0 + per);
    const uint32_t tasks = (t1 > t0 ? t1 - t0 : 0u) * chunks;
    for (uint32_t k = tid; k < tasks; k += 256) {
        const uint32_t t = t0 + k / chunks, c = k % chunks;
        const uint32_t *ob = p.hit_off + (size_t)t * (nb + 1) + q;
        const uint32_t a = ob[0] + c * HIT_CHUNK;
        // the last chunk also takes whatever a run holds beyond chunks * HIT_CHUNK ids
        const uint32_t end = c + 1 == chunks ? ob[1] : min(ob[1], a + HIT_CHUNK);
        const uint32_t *reg = p.hit_region + (size_t)t * p.hit_reg_words;
        uint32_t cur = 0xFFFFFFFFu, n = 0;
        for (uint32_t i = a; i < end; i += 16) {
            u32x4 v[4];
#pragma unroll
            for (int u = 0; u < 4; u++)
                v[u] = i + 4 * u < end ? __builtin_nontemporal_load((const u32x4 *)&reg[i + 4 * u])
                                       : u32x4{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t x[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                for (int cc = 0; cc < 4; cc++) {
                    if (x[cc] == 0xFFFFFFFFu) continue;
                    if (x[cc] == cur) {
                        n++;
                    } else {
                        if (n) atomicAdd(&cnt[cur & (HIT_R - 1)], n);
                        cur = x[cc];
                        n = 1;
                    }
                }
            }
        }
        if (n) atomicAdd(&cnt[cur & (HIT_R - 1)], n);
    }
    __syncthreads();
    for (uint32_t i = tid; i < HIT_R; i += 256)
        if (cnt[i])
            __hip_atomic_fetch_add(&p.rule_hits[(size_t)q * HIT_R + i], (unsigned long long)cnt[i], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void cop_snapshot(unsigned long long *src, uint32_t n, unsigned long long *dst, int reset)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    dst[i] = reset ? __hip_atomic_exchange(&src[i], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                   : __hip_atomic_load(&src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
} // namespace

extern "C" hipError_t copk_hit_count(const CopKParams *p, uint32_t n_tiles, uint32_t tile_pkts, hipStream_t stream)
{
    const uint32_t nb = max(1u, p->hit_nb);
    // chunks per run: enough for a bucket's share of a whole tile
    const uint32_t chunks = min(32u, max(1u, (tile_pkts / nb + HIT_CHUNK - 1) / HIT_CHUNK));
    // about eight tasks per lane, at most ~two workgroups per CU (64 KiB of
    // LDS each) over all buckets: every slice adds its non-zero counters to
    // rule_hits, so more slices also mean more atomics
    const uint32_t want = (uint32_t)(((uint64_t)n_tiles * chunks + 2047) / 2048);
    const uint32_t slices = max(1u, min(want, 512u / nb));
    hipLaunchKernelGGL(cop_hit_count, dim3(nb * slices), dim3(256), 0, stream, *p, n_tiles, slices, chunks);
    return hipGetLastError();
}

extern "C" hipError_t copk_snapshot(unsigned long long *src, uint32_t n_words, unsigned long long *dst, int reset,
                                    hipStream_t stream)
{
    hipLaunchKernelGGL(cop_snapshot, dim3((n_words + 255) / 256), dim3(256), 0, stream, src, n_words, dst, reset);
    return hipGetLastError();
}
#endif  // COPK_FW_PART
