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

namespace {

using namespace copd;

// diagnostic-only phase stamps (p.dbg bit 8): wave 0 lane 0 writes
// s_memrealtime (100 MHz) per phase into a buffer nothing else reads
#define STAMP(ph)                                                                          \
    do {                                                                                   \
        if ((o.dbg & 8u) && tid == 0) {                                                    \
            __builtin_amdgcn_sched_barrier(0);                                             \
            p.stamps[blockIdx.x * 8 + (ph)] = __builtin_amdgcn_s_memrealtime();            \
            __builtin_amdgcn_sched_barrier(0);                                             \
        }                                                                                  \
    } while (0)

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
template <int FW, int LPM, int LAY, int PPT, bool EXT>
__global__ __launch_bounds__(BLOCK, COPK_WAVES_PER_EU) void cop_pipeline(const CopKParams p)
{
    constexpr bool IMIX = LAY == COPK_LAY_IMIX;
    const Opt o = EXT ? opt_all(p) : Opt{0u, 0u, 0u, nullptr};
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    constexpr int TILE = BLOCK * PPT;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;

    // ---- LDS carve (offsets in u32 words, all multiples of 4) ----
    Tables tb;
    uint32_t *rt_top = lds;                                  // 256
    uint16_t *rt_leaf = (uint16_t *)(lds + 256);             // nleaf*256 u16
    uint32_t *fw_s = lds + p.lds_fw_off;
    uint32_t *fw_v = fw_s + p.fw_m;
    uint32_t *lp_s = lds + p.lds_lpm_off;
    uint32_t *lp_v = lp_s + p.lpm_m;
    tb.rt_top = rt_top;
    tb.rt_leaf = rt_leaf;
    tb.fw_s = fw_s;
    tb.fw_v = fw_v;
    tb.lp_s = lp_s;
    tb.lp_v = lp_v;
    uint32_t *misc = lds + p.lds_misc_off;
    uint32_t *s_tile = misc + 32;
    uint32_t *s_red = misc + 40;                              // [WAVES][8]
    CompactLds cl;
    cl.cnt = misc;                                            // [PPT*WAVES]
    cl.pref = misc + 33;
    cl.dq = misc + COPK_LDS_MISC_WORDS;                       // [K][PPT*WAVES]
    cl.dpref = cl.dq + COPK_MAX_DEMUX_PORTS * PPT * WAVES;    // [K]
    uint32_t *s_ps = cl.dpref + 8;                   // [WAVES][16]
    cl.stage = p.lds_stage_off ? lds + p.lds_stage_off : nullptr;   // [TILE]

    STAMP(0);
    // ---- batch of this workgroup: static blockIdx ranges ----
    // Equal-size batches are interleaved over blockIdx (b = g mod nb), so
    // consecutive tiles of one batch are dispatched nb workgroups apart and a
    // tile's predecessors have normally published their counts by the time
    // its look-back reads them. Unequal batches: blockIdx ranges.
    const uint32_t g = blockIdx.x;
    const bool ilv = p.uniform_ntiles != 0 && !(o.dbg & 256u);
    const uint32_t b = ilv ? __builtin_amdgcn_readfirstlane(g % p.nb) : batch_of_tile(p, g);
    uint32_t look_off;
    const CopKBatch B = batch_desc(p, b, &look_off);

    // ---- zero the lane's other ticket buffer for the next launch on this
    // lane (stream order puts that launch after this one completes) ----
    for (uint32_t line = g; line < p.zero_lines; line += gridDim.x)
        if (tid < 16) p.zero_tickets[line * 16 + tid] = 0ull;

    // ---- tile index inside the batch: this batch's ticket counter (or the
    // static order when no look-back runs: p.compact == 0) ----
    const bool dyn = p.compact != 0 && !(o.dbg & 2u);
    unsigned long long tk = 0;
    if (dyn && tid == 0) tk = atomicAdd(&p.tickets[b * 16], 1ull);

    // ---- stage tables into LDS by LDS-DMA while the ticket is in flight ----
    if (!(o.dbg & 4u)) {
        lds_stage(rt_top, p.rt_top, 64, lane, wave);
        lds_stage((uint32_t *)rt_leaf, p.rt_leaf, p.rt_nleaf * 32u, lane, wave);
        if (FW == COPK_TBL_IVT) {
            lds_stage(fw_s, p.fw_starts, p.fw_m >> 2, lane, wave);
            lds_stage(fw_v, p.fw_vals, p.fw_m >> 2, lane, wave);
        }
        if (LPM == COPK_TBL_IVT) {
            lds_stage(lp_s, p.lpm_starts, p.lpm_m >> 2, lane, wave);
            lds_stage(lp_v, p.lpm_vals, p.lpm_m >> 2, lane, wave);
        }
    }
    uint32_t j;
    if (dyn) {
        if (tid == 0) *s_tile = (uint32_t)tk;
        __syncthreads();
        j = __builtin_amdgcn_readfirstlane(*s_tile);
    } else {
        j = ilv ? g / p.nb : p.uniform_ntiles ? g - b * p.uniform_ntiles : g - p.tile_begin[b];
    }
    const uint32_t base = j * TILE;
    STAMP(1);

    // ---- packet header loads (all PPT packets, no branches). Lanes past
    // the end of the batch re-read the last packet and are masked out of
    // every store and count. ----
    uint32_t w3[PPT], w6[PPT], w7[PPT], w8[PPT];
    bool valid[PPT];
    const uint32_t last = B.n ? B.n - 1 : 0u;
    if (LAY == COPK_LAY_COALESCED && B.n) {
        const StepGeom sg = step_geom(lane);
        u32x4 v[PPT][3];
#pragma unroll
        for (int k = 0; k < PPT; k++) load_step(sg, B.pkts + B.data_off, B.stride, base + k * BLOCK + wave * 64, last, v[k]);
#pragma unroll
        for (int k = 0; k < PPT; k++) gather_step(sg, v[k], w3[k], w6[k], w7[k], w8[k]);
    } else if (LAY == COPK_LAY_HDR16 && B.n) {
        // one 16-byte record per packet: frame bytes 12..15 then 24..35
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            const uint32_t ic = min(base + k * BLOCK + tid, last);
            const u32x4 v = __builtin_nontemporal_load((const u32x4 *)(B.pkts + B.data_off + (size_t)ic * 16u));
            w3[k] = v.x;
            w6[k] = v.y;
            w7[k] = v.z;
            w8[k] = v.w;
        }
    } else if (B.n) {
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            const uint32_t ic = min(base + k * BLOCK + tid, last);
            const uint8_t *pk;
            if (IMIX) pk = B.pkts + B.offsets[ic] + B.data_off;
            else pk = B.pkts + (size_t)ic * B.stride + B.data_off;
            // two loads: bytes 12..27 (dwordx4 at a 4-byte-aligned address;
            // w3 and w6) and 28..35 (w7, w8)
            const u32x4a a = *(const u32x4a *)(pk + 12);
            const u32x2a b = *(const u32x2a *)(pk + 28);
            w3[k] = a.x;
            w6[k] = a.w;
            w7[k] = b.x;
            w8[k] = b.y;
        }
    } else {
#pragma unroll
        for (int k = 0; k < PPT; k++) w3[k] = w6[k] = w7[k] = w8[k] = 0;
    }
#pragma unroll
    for (int k = 0; k < PPT; k++) valid[k] = base + k * BLOCK + tid < B.n;
    if (!dyn) __syncthreads();   // LDS tables (the dynamic path synced above)

    // ---- pass 1 (parse, route, LDS searches, tbl24 loads issued) ----
    uint32_t verdict[PPT], port[PPT], flags[PPT], rnh[PPT], fwe[PPT], lpe[PPT], src[PPT], dst[PPT];
    pass1<FW, LPM, PPT>(p, tb, w3, w6, w7, w8, verdict, port, src, dst, fwe, lpe);
    if (o.dbg & 8u) {
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < PPT; k++) x ^= verdict[k] ^ src[k];
        asm volatile("" ::"v"(x));
    }
    STAMP(2);

    // ---- pass 2 (tbl8 step) and the verdicts ----
    Counts cn;
    pass2<FW, LPM, PPT>(p, w3, src, dst, valid, fwe, lpe, verdict, flags, rnh, cn.total, cn.notv4);
    rule_hit_atomics<FW, PPT>(o, valid, flags, fwe);
    if (o.dbg & 8u) {
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < PPT; k++) x ^= verdict[k] ^ rnh[k];
        asm volatile("" ::"v"(x));
    }
    STAMP(3);
    // ---- ordered compaction (one list per batch, or per vport), with the
    // result records (8 B per packet, coalesced) stored during its look-back
    bool fwd[PPT];
#pragma unroll
    for (int k = 0; k < PPT; k++) fwd[k] = valid[k] && verdict[k] == COPK_FORWARD;
    auto records = [&] { store_records<PPT>(B, base, tid, valid, verdict, flags, port, rnh, fwd, cn); };
    if (p.compact) compact_tile<PPT>(p, o, B, look_off, j, base, fwd, port, cl, tid, lane, wave, records);
    else records();
    STAMP(5);

    // ---- counters (one flush per workgroup) ----
    uint32_t prx[COPK_MAX_DEMUX_PORTS] = {}, ptx[COPK_MAX_DEMUX_PORTS] = {};
    if (o.port_stats) port_counts<PPT>(o.port_stats, valid, fwd, port, prx, ptx);
    flush_counters(p, o, cn, prx, ptx, s_red, s_ps, tid, lane, wave);
    STAMP(6);
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
    if (lpm == COPK_TBL_IVT) return launch_imix<FW, COPK_TBL_IVT>(p, imix, ppt, grid, lds, s);
    if (lpm == COPK_TBL_DIR) return launch_imix<FW, COPK_TBL_DIR>(p, imix, ppt, grid, lds, s);
    return launch_imix<FW, COPK_TBL_OFF>(p, imix, ppt, grid, lds, s);
}

} // namespace

extern "C" hipError_t copk_launch(const CopKParams *p, int fw_mode, int lpm_mode, int imix, int ppt,
                                  uint32_t grid, uint32_t lds_bytes, hipStream_t stream)
{
    if (fw_mode == COPK_TBL_IVT) return launch_lpm<COPK_TBL_IVT>(*p, lpm_mode, imix, ppt, grid, lds_bytes, stream);
    if (fw_mode == COPK_TBL_DIR) return launch_lpm<COPK_TBL_DIR>(*p, lpm_mode, imix, ppt, grid, lds_bytes, stream);
    return launch_lpm<COPK_TBL_OFF>(*p, lpm_mode, imix, ppt, grid, lds_bytes, stream);
}

namespace {
__global__ void cop_snapshot(unsigned long long *src, uint32_t n, unsigned long long *dst, int reset)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    dst[i] = reset ? __hip_atomic_exchange(&src[i], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                   : __hip_atomic_load(&src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
} // namespace

extern "C" hipError_t copk_snapshot(unsigned long long *src, uint32_t n_words, unsigned long long *dst, int reset,
                                    hipStream_t stream)
{
    hipLaunchKernelGGL(cop_snapshot, dim3((n_words + 255) / 256), dim3(256), 0, stream, src, n_words, dst, reset);
    return hipGetLastError();
}
