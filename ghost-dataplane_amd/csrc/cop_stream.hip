// cop_stream.hip — the coprocessor NF pipeline, persistent batch-sweep form.
//
// For launches of many equal 64-byte-slot batches (the bench's batch rings;
// cop_kernels.hip handles everything else: few or ragged batches, IMIX,
// strides < 48). Same per-packet contract (cop_device.h), same
// records, forward lists and counters as the one-shot kernel; what differs
// is how packet bytes move and how work is scheduled:
//
//  * One workgroup sweeps a whole batch, front to back, in tiles of 256*PPT
//    packets; a persistent grid of G workgroups (<= co-resident) takes
//    batches b = blockIdx, blockIdx + G, ... The ordered forward list of a
//    batch (coprocessor() forwards in ring order, switch.c:443-474) then
//    needs no cross-workgroup look-back: the workgroup keeps the list's
//    length as a running count, and each tile's order comes from wave
//    ballots plus one LDS scan (one workgroup barrier per tile). A single
//    pass with decoupled look-back needs either an in-order wait on loads
//    that were prefetched (vmcnt retires in order) or a lockstep of the
//    tiles of a batch; both measured slower than this.
//  * Software pipelining: the next tile's loads (the first tile of the next
//    batch at a batch's end) are issued before this tile is classified, or
//    right after its DIR-24-8 probes when a stage uses the HBM table (a
//    wait on a probe is a wait on every older load).
//  * Coalesced non-temporal loads (cop_device.h load_step / gather_step):
//    a wave moves the first 48 bytes of 64 consecutive packets with three
//    16-byte loads per lane and regroups the fields with four ds_bpermute;
//    non-temporal, so the packet stream does not evict LPM tables from the
//    Infinity Cache. A workgroup reads its batch sequentially (4 MiB per
//    64k batch), which keeps DRAM pages open.
//  * LDS tables are staged once per workgroup; counters are flushed once.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cop_device.h"
#include "cop_kernels.h"

namespace {

using namespace copd;

// stream-kernel LDS misc area (u32 words after the tables)
constexpr uint32_t SM_RED = 0;      // [WAVES][8] counter reduction
constexpr uint32_t SM_PS = 32;      // [WAVES][16] per-port counts
constexpr uint32_t SM_CNT = 96;     // [2][K=8][PPT*WAVES <= 32] tile counts (tile parity)
static_assert(SM_CNT + 2 * COPK_MAX_DEMUX_PORTS * 32 <= COPK_LDS_STREAM_MISC_WORDS, "stream misc area");

template <int PPT>
struct Slots {
    u32x4 v[PPT][3];
};

template <int FW, int LPM, int PPT>
__global__ __launch_bounds__(BLOCK, 2) void cop_stream(const CopKParams p)
{
    static_assert(PPT * WAVES <= 32, "tile counts per chain");
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    constexpr int TILE = BLOCK * PPT;
    constexpr int NQ = PPT * WAVES;
    constexpr bool EARLY = FW != COPK_TBL_DIR && LPM != COPK_TBL_DIR;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;

    Tables tb;
    uint32_t *rt_top = lds;
    uint16_t *rt_leaf = (uint16_t *)(lds + 256);
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

    // the other ticket buffer of this lane: zeroed for the next one-shot
    // launch (this kernel draws no tickets)
    for (uint32_t line = blockIdx.x; line < p.zero_lines; line += gridDim.x)
        if (tid < 16) p.zero_tickets[line * 16 + tid] = 0ull;

    // tables into LDS once (LDS-DMA; the barrier below waits for it)
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

    const StepGeom sg = step_geom(lane);
    const Opt o = opt_all(p);
    const uint32_t K = p.demux ? p.demux : 1u;   // forward lists per batch
    const uint32_t G = gridDim.x;

    // (batch, tile) cursor: this workgroup's batches b = blockIdx + i*G
    auto ntiles_of = [&](const CopKBatch &B) { return (B.n + TILE - 1) / TILE; };
    auto load = [&](const CopKBatch &B, uint32_t t, Slots<PPT> &s) {
        const uint8_t *pk0 = B.pkts + B.data_off;
#pragma unroll
        for (int k = 0; k < PPT; k++) load_step(sg, pk0, B.stride, t * TILE + k * BLOCK + wave * 64, B.n - 1, s.v[k]);
    };

    uint32_t b = blockIdx.x, look_unused;
    CopKBatch B = batch_desc(p, b, &look_unused);
    uint32_t t = 0;
    // skip leading empty batches (their list lengths are written as 0)
    auto skip_empty = [&](uint32_t &bb, CopKBatch &BB) {
        while (bb < p.nb && BB.n == 0) {
            if (p.compact && BB.fwd_count && tid < (int)K) BB.fwd_count[tid] = 0;
            bb += G;
            if (bb < p.nb) BB = batch_desc(p, bb, &look_unused);
        }
    };
    skip_empty(b, B);
    // ping-pong tile buffers: the loop runs two tiles per trip, so the tile
    // in flight never has to be copied into the tile in hand (a copy waits
    // for the loads to land and ends the overlap)
    Slots<PPT> bufA, bufB;
    if (b < p.nb) load(B, 0, bufA);
    __syncthreads();   // LDS tables landed (the barrier waits for the DMA)

    Counts cn;
    uint32_t prx[COPK_MAX_DEMUX_PORTS] = {}, ptx[COPK_MAX_DEMUX_PORTS] = {};
    uint32_t run[COPK_MAX_DEMUX_PORTS] = {};   // forward-list lengths so far (wave-uniform)
    uint32_t par = 0;
    // one tile: classify `cur` while `nxt` loads; false after the last tile
    auto step = [&](Slots<PPT> &cur, Slots<PPT> &nxt) -> bool {
        // ---- the next tile: this batch's, or the first of the next batch ----
        uint32_t bn = b, tn = t + 1;
        CopKBatch Bn = B;
        if (tn >= ntiles_of(B)) {
            bn = b + G;
            tn = 0;
            if (bn < p.nb) {
                Bn = batch_desc(p, bn, &look_unused);
                skip_empty(bn, Bn);
            }
        }
        const bool more = bn < p.nb;
        if (EARLY && more) load(Bn, tn, nxt);
        // keep the prefetch ahead of this tile's gathers: without the fence
        // the scheduler sinks the loads below the ds_bpermutes, which wait
        // for this tile's data, and nothing is in flight while it is used
        __builtin_amdgcn_sched_barrier(0);

        // ---- fields to the packet's lane ----
        uint32_t w3[PPT], w6[PPT], w7[PPT], w8[PPT];
#pragma unroll
        for (int k = 0; k < PPT; k++) gather_step(sg, cur.v[k], w3[k], w6[k], w7[k], w8[k]);
        const uint32_t base = t * TILE;
        bool valid[PPT];
#pragma unroll
        for (int k = 0; k < PPT; k++) valid[k] = base + k * BLOCK + tid < B.n;

        uint32_t verdict[PPT], port[PPT], flags[PPT], rnh[PPT], fwe[PPT], lpe[PPT], src[PPT], dst[PPT];
        pass1<FW, LPM, PPT>(p, tb, w3, w6, w7, w8, verdict, port, src, dst, fwe, lpe);
        pass2<FW, LPM, PPT>(p, w3, src, dst, valid, fwe, lpe, verdict, flags, rnh, cn.total, cn.notv4);
        if (!EARLY && more) load(Bn, tn, nxt);
        __builtin_amdgcn_sched_barrier(0);
        rule_hit_atomics<FW, PPT>(o, valid, flags, fwe);
        bool fwd[PPT];
        store_records<PPT>(B, base, tid, valid, verdict, flags, port, rnh, fwd, cn);
        if (p.port_stats) port_counts<PPT>(p.port_stats, valid, fwd, port, prx, ptx);

        // ---- ordered compaction: tile-local ballots + LDS scan, appended
        // at the batch's running list lengths ----
        if (p.compact) {
            uint32_t *cnt = misc + SM_CNT + par * (COPK_MAX_DEMUX_PORTS * 32);
#pragma unroll
            for (int q = 0; q < COPK_MAX_DEMUX_PORTS; q++) {
                if ((uint32_t)q >= K) break;
#pragma unroll
                for (int k = 0; k < PPT; k++) {
                    const unsigned long long bl = __ballot(fwd[k] && (K == 1 || port[k] == (uint32_t)q));
                    if (lane == 0) cnt[q * 32 + k * WAVES + wave] = (uint32_t)__popcll(bl);
                }
            }
            lds_barrier();
            uint32_t off[PPT] = {};
#pragma unroll
            for (int q = 0; q < COPK_MAX_DEMUX_PORTS; q++) {
                if ((uint32_t)q >= K) break;
                uint32_t agg;
                const uint32_t ex = wave_excl_scan(lane < NQ ? cnt[q * 32 + lane] : 0u, NQ, lane, &agg);
#pragma unroll
                for (int k = 0; k < PPT; k++) {
                    const uint32_t o = (uint32_t)__shfl((int)ex, k * WAVES + wave);
                    const bool mine = fwd[k] && (K == 1 || port[k] == (uint32_t)q);
                    const unsigned long long bl = __ballot(mine);
                    if (mine)
                        off[k] = q * B.n + run[q] + o +
                                 __builtin_amdgcn_mbcnt_hi((uint32_t)(bl >> 32),
                                                           __builtin_amdgcn_mbcnt_lo((uint32_t)bl, 0u));
                }
                run[q] += agg;
            }
            if (B.fwd_idx) {
#pragma unroll
                for (int k = 0; k < PPT; k++)
                    if (fwd[k]) __builtin_nontemporal_store(base + k * BLOCK + tid, &B.fwd_idx[off[k]]);
            }
            par ^= 1u;
        }

        // ---- batch done: its list lengths ----
        if (bn != b || !more) {
            if (p.compact && B.fwd_count && wave == 0) {
#pragma unroll
                for (int q = 0; q < COPK_MAX_DEMUX_PORTS; q++)
                    if ((uint32_t)q < K && lane == q) B.fwd_count[q] = run[q];
            }
#pragma unroll
            for (int q = 0; q < COPK_MAX_DEMUX_PORTS; q++) run[q] = 0;
        }
        if (!more) return false;
        b = bn;
        t = tn;
        B = Bn;
        return true;
    };
    if (b < p.nb) {
        while (step(bufA, bufB) && step(bufB, bufA)) {
        }
    }
    flush_counters(p, o, cn, prx, ptx, misc + SM_RED, misc + SM_PS, tid, lane, wave);
}

template <int FW, int LPM, int PPT>
hipError_t launch_stream(const CopKParams &p, uint32_t grid, uint32_t lds_bytes, hipStream_t s)
{
    hipLaunchKernelGGL((cop_stream<FW, LPM, PPT>), dim3(grid), dim3(BLOCK), lds_bytes, s, p);
    return hipGetLastError();
}

template <int FW, int LPM>
hipError_t stream_ppt(const CopKParams *p, int ppt, uint32_t grid, uint32_t lds, hipStream_t s, int *occ)
{
    if (occ) {
        if (ppt == 4) return hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, cop_stream<FW, LPM, 4>, BLOCK, lds);
        if (ppt == 2) return hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, cop_stream<FW, LPM, 2>, BLOCK, lds);
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, cop_stream<FW, LPM, 1>, BLOCK, lds);
    }
    if (ppt == 4) return launch_stream<FW, LPM, 4>(*p, grid, lds, s);
    if (ppt == 2) return launch_stream<FW, LPM, 2>(*p, grid, lds, s);
    return launch_stream<FW, LPM, 1>(*p, grid, lds, s);
}

template <int FW>
hipError_t stream_lpm(const CopKParams *p, int lpm, int ppt, uint32_t grid, uint32_t lds, hipStream_t s, int *occ)
{
    if (lpm == COPK_TBL_IVT) return stream_ppt<FW, COPK_TBL_IVT>(p, ppt, grid, lds, s, occ);
    if (lpm == COPK_TBL_DIR) return stream_ppt<FW, COPK_TBL_DIR>(p, ppt, grid, lds, s, occ);
    return stream_ppt<FW, COPK_TBL_OFF>(p, ppt, grid, lds, s, occ);
}

hipError_t stream_dispatch(const CopKParams *p, int fw, int lpm, int ppt, uint32_t grid, uint32_t lds, hipStream_t s,
                           int *occ)
{
    if (fw == COPK_TBL_IVT) return stream_lpm<COPK_TBL_IVT>(p, lpm, ppt, grid, lds, s, occ);
    if (fw == COPK_TBL_DIR) return stream_lpm<COPK_TBL_DIR>(p, lpm, ppt, grid, lds, s, occ);
    return stream_lpm<COPK_TBL_OFF>(p, lpm, ppt, grid, lds, s, occ);
}

}  // namespace

extern "C" hipError_t copk_launch_stream(const CopKParams *p, int fw_mode, int lpm_mode, int ppt, uint32_t grid,
                                         uint32_t lds_bytes, hipStream_t stream)
{
    return stream_dispatch(p, fw_mode, lpm_mode, ppt, grid, lds_bytes, stream, nullptr);
}

extern "C" hipError_t copk_stream_occupancy(int fw_mode, int lpm_mode, int ppt, uint32_t lds_bytes, int *blocks_per_cu)
{
    *blocks_per_cu = 0;
    return stream_dispatch(nullptr, fw_mode, lpm_mode, ppt, 0, lds_bytes, nullptr, blocks_per_cu);
}
