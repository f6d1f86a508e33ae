// cop_sweep.hip — the coprocessor NF pipeline, persistent globally ordered
// form ("sweep").
//
// Same per-packet contract (cop_device.h), same records,
// forward lists and counters as the one-shot kernel (cop_kernels.hip); what
// differs is how work is scheduled:
//
//  * A persistent grid (a few workgroups per CU) claims tiles of 256*PPT
//    packets in GLOBAL order from one ticket counter, SW_CHUNK tiles per
//    atomic. The whole chip then sweeps the launch's packets front to back,
//    instead of one tile per short-lived workgroup.
//  * Each workgroup is 4 data waves plus 1 coordinator wave. The data waves
//    prefetch the next tile's packet bytes (coalesced non-temporal loads,
//    cop_device.h load_step) before they classify the current one. The
//    coordinator draws tickets and runs the decoupled look-back of the
//    ordered forward list (coprocessor() forwards in ring order,
//    switch.c:443-474). vmcnt retires in order within a wave, so a look-back
//    load issued by a data wave would wait for the prefetched tile; on a wave
//    of its own it waits for nothing but its granules.
//  * Deadlock freedom needs no residency assumption: a tile is claimed only
//    by a running workgroup, each workgroup processes its claims in claim
//    order, and a tile's look-back waits only on smaller tiles.
//
// Per tile (two workgroup barriers): data waves classify, store records,
// ballot their forward flags into LDS counts | A | coordinator: claim the
// tile after next, look back, publish the batch prefix; data waves: scan the
// counts, stage the tile's list in LDS | B | data waves: copy the list out.
// LDS buffers alternate by tile parity.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cop_device.h"
#include "cop_kernels.h"

namespace {

using namespace copd;

constexpr int SW_THREADS = BLOCK + 64;   // 4 data waves + 1 coordinator wave
constexpr int COORD = WAVES;             // the coordinator's wave index
constexpr uint32_t SW_CHUNK = 1;         // tiles claimed per ticket atomic (consecutive tiles must run concurrently)

// misc LDS area (u32 words after the tables)
constexpr uint32_t SW_TQ = 0;      // [4] claimed tile queue
constexpr uint32_t SW_PREF = 4;    // [2] batch prefix of the tile (by parity)
constexpr uint32_t SW_CNT = 8;     // [2][32] (step, wave) forward counts (by parity)
constexpr uint32_t SW_RED = 72;    // [WAVES][8] counter reduction
constexpr uint32_t SW_PS = 104;    // [WAVES][16] per-port counts
static_assert(SW_PS + WAVES * 16 <= COPK_LDS_SWEEP_MISC_WORDS, "sweep misc area");

template <int FW, int LPM, int PPT>
__global__ __launch_bounds__(SW_THREADS, 3) void cop_sweep(const CopKParams p)
{
    static_assert(PPT * WAVES <= 32, "tile counts");
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    constexpr int TILE = BLOCK * PPT;
    constexpr int NQ = PPT * WAVES;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const bool coord = wave == COORD;

    Tables tb;
    tb.rt_top = lds;
    tb.rt_leaf = (const uint16_t *)(lds + 256);
    tb.fw_s = lds + p.lds_fw_off;
    tb.fw_v = tb.fw_s + p.fw_m;
    tb.lp_s = lds + p.lds_lpm_off;
    tb.lp_v = tb.lp_s + p.lpm_m;
    uint32_t *misc = lds + p.lds_misc_off;
    uint32_t *tq = misc + SW_TQ;
    uint32_t *pref = misc + SW_PREF;
    uint32_t *cnt = misc + SW_CNT;
    uint32_t *stage = p.lds_stage_off ? lds + p.lds_stage_off : nullptr;   // [2][TILE]

    // the lane's other ticket buffer: zeroed for the next launch on this lane
    for (uint32_t line = blockIdx.x; line < p.zero_lines; line += gridDim.x)
        if (tid < 16) p.zero_tickets[line * 16 + tid] = 0ull;

    const uint32_t total = p.ntiles;
    // coordinator: tiles claimed SW_CHUNK at a time, handed out in order
    uint32_t cpos = 0, cend = 0;
    const bool stat = (p.dbg & 512u) != 0;   // experiment: static round-robin tiles (needs co-residency)
    uint32_t sidx = blockIdx.x;
    auto claim = [&]() -> uint32_t {
        if (stat) {
            const uint32_t t = sidx;
            sidx += gridDim.x;
            return t < total ? t : total;
        }
        if (cpos >= cend) {
            if (cend >= total && cend != 0) return total;   // the launch's tiles are all claimed
            unsigned long long t = 0;
            if (lane == 0) t = atomicAdd(&p.tickets[0], (unsigned long long)SW_CHUNK);
            const uint32_t t0 = (uint32_t)min(__shfl(t, 0), (unsigned long long)total);
            cpos = __builtin_amdgcn_readfirstlane(t0);
            cend = __builtin_amdgcn_readfirstlane(min(t0 + SW_CHUNK, total));
            if (cpos >= cend) {
                cend = total;
                return total;
            }
        }
        return cpos++;
    };
    if (coord) {
        const uint32_t a = claim();
        const uint32_t b = a < total ? claim() : total;
        if (lane == 0) {
            tq[0] = a;
            tq[1] = b;
        }
    } else {
        lds_stage((uint32_t *)tb.rt_top, p.rt_top, 64, lane, wave);
        lds_stage((uint32_t *)tb.rt_leaf, p.rt_leaf, p.rt_nleaf * 32u, lane, wave);
        if (FW == COPK_TBL_IVT) {
            lds_stage((uint32_t *)tb.fw_s, p.fw_starts, p.fw_m >> 2, lane, wave);
            lds_stage((uint32_t *)tb.fw_v, p.fw_vals, p.fw_m >> 2, lane, wave);
        }
        if (LPM == COPK_TBL_IVT) {
            lds_stage((uint32_t *)tb.lp_s, p.lpm_starts, p.lpm_m >> 2, lane, wave);
            lds_stage((uint32_t *)tb.lp_v, p.lpm_vals, p.lpm_m >> 2, lane, wave);
        }
    }
    __syncthreads();   // tables landed, first two claims visible

    const StepGeom sg = step_geom(lane);
    // tile T -> batch, its descriptor, the batch's first look-back granule,
    // the tile's index inside the batch
    auto locate = [&](uint32_t T, CopKBatch &B, uint32_t &look_off, uint32_t &j) {
        const uint32_t b = batch_of_tile(p, T);
        B = batch_desc(p, b, &look_off);
        j = T - (p.uniform_ntiles ? b * p.uniform_ntiles : p.tile_begin[b]);
    };
    auto load_tile = [&](const CopKBatch &B, uint32_t j, u32x4 (&v)[PPT][3]) {
        if (!B.n) return;   // an empty batch's one tile: nothing to read
        const uint8_t *pk0 = B.pkts + B.data_off;
#pragma unroll
        for (int k = 0; k < PPT; k++) load_step(sg, pk0, B.stride, j * TILE + k * BLOCK + wave * 64, B.n - 1, v[k]);
    };

    uint32_t T = __builtin_amdgcn_readfirstlane(tq[0]);
    u32x4 bufA[PPT][3], bufB[PPT][3];   // ping-pong: tile in hand / tile in flight
    if (!coord && T < total) {
        CopKBatch B0;
        uint32_t lo0, j0;
        locate(T, B0, lo0, j0);
        load_tile(B0, j0, bufA);
    }

    Counts cn;
    uint32_t prx[COPK_MAX_DEMUX_PORTS] = {}, ptx[COPK_MAX_DEMUX_PORTS] = {};
    uint32_t it = 0;
    // one tile: classify `cur` (tile T) while `nxt` (tile Tn) loads
    auto body = [&](u32x4 (&cur)[PPT][3], u32x4 (&nxt)[PPT][3]) {
        const uint32_t par = it & 1u;
        const uint32_t Tn = __builtin_amdgcn_readfirstlane(tq[(it + 1) & 3u]);
        CopKBatch B;
        uint32_t look_off, j;
        locate(T, B, look_off, j);
        const uint32_t base = j * TILE;
        bool fwd[PPT];
        unsigned long long bal[PPT];
        if (!coord) {
            // ---- the next tile's bytes in flight while this one is classified ----
            if (Tn < total) {
                CopKBatch Bn;
                uint32_t lon, jn;
                locate(Tn, Bn, lon, jn);
                load_tile(Bn, jn, nxt);
            }
            uint32_t w3[PPT], w6[PPT], w7[PPT], w8[PPT];
            bool valid[PPT];
            if (B.n) {
#pragma unroll
                for (int k = 0; k < PPT; k++) gather_step(sg, cur[k], w3[k], w6[k], w7[k], w8[k]);
            } else {
#pragma unroll
                for (int k = 0; k < PPT; k++) w3[k] = w6[k] = w7[k] = w8[k] = 0;
            }
#pragma unroll
            for (int k = 0; k < PPT; k++) valid[k] = base + k * BLOCK + tid < B.n;
            uint32_t verdict[PPT], port[PPT], flags[PPT], rnh[PPT], fwe[PPT], lpe[PPT], src[PPT], dst[PPT];
            pass1<FW, LPM, PPT>(p, tb, w3, w6, w7, w8, verdict, port, src, dst, fwe, lpe);
            pass2<FW, LPM, PPT>(p, w3, src, dst, valid, fwe, lpe, verdict, flags, rnh, cn.total, cn.notv4);
            rule_hit_atomics<FW, PPT>(p, valid, flags, fwe);
            store_records<PPT>(B, base, tid, valid, verdict, flags, port, rnh, fwd, cn);
            if (p.port_stats) port_counts<PPT>(p.port_stats, valid, fwd, port, prx, ptx);
            if (p.compact) {
#pragma unroll
                for (int k = 0; k < PPT; k++) {
                    bal[k] = __ballot(fwd[k]);
                    if (lane == 0) cnt[par * 32 + k * WAVES + wave] = (uint32_t)__popcll(bal[k]);
                }
            }
        }
        lds_barrier();   // A: counts of tile T
        uint32_t off[PPT] = {};
        if (coord) {
            const uint32_t T2 = Tn < total ? claim() : total;
            if (lane == 0) tq[(it + 2) & 3u] = T2;
            if (p.compact) {
                uint32_t agg;
                (void)wave_excl_scan(lane < NQ ? cnt[par * 32 + lane] : 0u, NQ, lane, &agg);
                const uint32_t excl = look_back(p.look + look_off, 1u, j, agg, p.epoch, p.err, lane);
                if (lane == 0) {
                    pref[par] = excl;
                    if (B.fwd_count && j == B.ntiles - 1) *B.fwd_count = excl + agg;
                }
            }
        } else if (p.compact) {
            uint32_t agg;
            const uint32_t ex = wave_excl_scan(lane < NQ ? cnt[par * 32 + lane] : 0u, NQ, lane, &agg);
#pragma unroll
            for (int k = 0; k < PPT; k++) off[k] = (uint32_t)__shfl((int)ex, k * WAVES + wave);
            if (stage && B.fwd_idx) {
                uint32_t *st = stage + par * TILE;
#pragma unroll
                for (int k = 0; k < PPT; k++)
                    if (fwd[k])
                        st[off[k] + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal[k] >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)bal[k], 0u))] =
                            base + k * BLOCK + tid;
            }
        }
        lds_barrier();   // B: the batch prefix of tile T
        if (!coord && p.compact && B.fwd_idx) {
            const uint32_t pr = pref[par];
            if (stage) {
                uint32_t agg = 0;
#pragma unroll
                for (int q = 0; q < NQ; q++) agg += cnt[par * 32 + q];
                copy_out_list(B.fwd_idx, pr, agg, stage + par * TILE, tid);
            } else {
#pragma unroll
                for (int k = 0; k < PPT; k++) {
                    if (fwd[k]) {
                        const uint32_t r = __builtin_amdgcn_mbcnt_hi(
                            (uint32_t)(bal[k] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal[k], 0u));
                        __builtin_nontemporal_store(base + k * BLOCK + tid, &B.fwd_idx[pr + off[k] + r]);
                    }
                }
            }
        }
        T = Tn;
        it++;
    };
    while (T < total) {
        body(bufA, bufB);
        if (T >= total) break;
        body(bufB, bufA);
    }
    flush_counters(p, cn, prx, ptx, misc + SW_RED, misc + SW_PS, tid, lane, wave);
}

template <int FW, int LPM, int PPT>
hipError_t sweep_one(const CopKParams *p, uint32_t grid, uint32_t lds, hipStream_t s, int *occ)
{
    if (occ) return hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, cop_sweep<FW, LPM, PPT>, SW_THREADS, lds);
    hipLaunchKernelGGL((cop_sweep<FW, LPM, PPT>), dim3(grid), dim3(SW_THREADS), lds, s, *p);
    return hipGetLastError();
}

template <int FW, int LPM>
hipError_t sweep_ppt(const CopKParams *p, int ppt, uint32_t grid, uint32_t lds, hipStream_t s, int *occ)
{
    if (ppt == 4) return sweep_one<FW, LPM, 4>(p, grid, lds, s, occ);
    if (ppt == 2) return sweep_one<FW, LPM, 2>(p, grid, lds, s, occ);
    return sweep_one<FW, LPM, 1>(p, grid, lds, s, occ);
}

template <int FW>
hipError_t sweep_lpm(const CopKParams *p, int lpm, int ppt, uint32_t grid, uint32_t lds, hipStream_t s, int *occ)
{
    if (lpm == COPK_TBL_IVT) return sweep_ppt<FW, COPK_TBL_IVT>(p, ppt, grid, lds, s, occ);
    if (lpm == COPK_TBL_DIR) return sweep_ppt<FW, COPK_TBL_DIR>(p, ppt, grid, lds, s, occ);
    return sweep_ppt<FW, COPK_TBL_OFF>(p, ppt, grid, lds, s, occ);
}

hipError_t sweep_dispatch(const CopKParams *p, int fw, int lpm, int ppt, uint32_t grid, uint32_t lds, hipStream_t s,
                          int *occ)
{
    if (fw == COPK_TBL_IVT) return sweep_lpm<COPK_TBL_IVT>(p, lpm, ppt, grid, lds, s, occ);
    if (fw == COPK_TBL_DIR) return sweep_lpm<COPK_TBL_DIR>(p, lpm, ppt, grid, lds, s, occ);
    return sweep_lpm<COPK_TBL_OFF>(p, lpm, ppt, grid, lds, s, occ);
}

}  // namespace

extern "C" hipError_t copk_launch_sweep(const CopKParams *p, int fw_mode, int lpm_mode, int ppt, uint32_t grid,
                                        uint32_t lds_bytes, hipStream_t stream)
{
    return sweep_dispatch(p, fw_mode, lpm_mode, ppt, grid, lds_bytes, stream, nullptr);
}

extern "C" hipError_t copk_sweep_occupancy(int fw_mode, int lpm_mode, int ppt, uint32_t lds_bytes, int *blocks_per_cu)
{
    *blocks_per_cu = 0;
    return sweep_dispatch(nullptr, fw_mode, lpm_mode, ppt, 0, lds_bytes, nullptr, blocks_per_cu);
}
