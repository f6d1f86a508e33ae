// cop_tile.h — the per-tile pipeline body shared by the one-shot kernel
// (cop_kernels.hip) and the poll-mode kernel (cop_pmd.hip). Internal.
#ifndef COP_TILE_H
#define COP_TILE_H

#include "cop_device.h"

namespace copd {

// diagnostic-only phase stamps (p.dbg bit 8): wave 0 lane 0 writes
// s_memrealtime (100 MHz) per phase into a buffer nothing else reads.
// Experiment builds with -DCOPK_PHASE_STAMPS=1 stamp whenever p.stamps is
// set, so the production (non-EXT) kernels can be stamped at their own
// occupancy.
#ifndef COPK_PHASE_STAMPS
#define COPK_PHASE_STAMPS 0
#endif
#define STAMP(ph)                                                                          \
    do {                                                                                   \
        if (((o.dbg & 8u) || (COPK_PHASE_STAMPS && p.stamps)) && tid == 0) {               \
            __builtin_amdgcn_sched_barrier(0);                                             \
            __hip_atomic_store(&p.stamps[blockIdx.x * 8 + (ph)], __builtin_amdgcn_s_memrealtime(), \
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);                     \
            __builtin_amdgcn_sched_barrier(0);                                             \
        }                                                                                  \
    } while (0)

// LDS carve of a launch (offsets in u32 words, all multiples of 4): the
// staged tables, then the misc scratch (compaction counts and prefixes, the
// ticket broadcast, counter reduction, per-port scratch), then the tile's
// staged forward list.
struct LdsCarve {
    Tables tb;
    CompactLds cl;
    uint32_t *s_tile;   // ticket broadcast
    uint32_t *s_red;    // [WAVES][8] counter reduction
    uint32_t *s_ps;     // [WAVES][16] per-port counter reduction
    uint32_t *s_misc;   // the misc area (poll-mode kernel: doorbell broadcast at +36)
};

template <int PPT>
__device__ __forceinline__ LdsCarve lds_carve(const CopKParams &p, uint32_t *lds)
{
    LdsCarve c;
    c.tb.rt_top = lds;                                  // 256
    c.tb.rt_leaf = (uint16_t *)(lds + 256);       // nleaf*256 u16
    c.tb.fw_s = lds + p.lds_fw_off;                 // sorted starts, then the bucket index
    c.tb.fw_v = c.tb.fw_s + p.fw_m + p.fw_iw;
    c.tb.lp_s = lds + p.lds_lpm_off;
    c.tb.lp_v = c.tb.lp_s + p.lpm_m + p.lpm_iw;
    uint32_t *misc = lds + p.lds_misc_off;
    c.s_misc = misc;
    c.s_tile = misc + 32;
    c.s_red = misc + 40;                                            // [WAVES][8]
    c.cl.cnt = misc;                                                // [PPT*WAVES]
    c.cl.pref = misc + 33;
    c.cl.dq = misc + COPK_LDS_MISC_WORDS;                           // [K][PPT*WAVES]
    c.cl.dpref = c.cl.dq + COPK_MAX_DEMUX_PORTS * PPT * WAVES;      // [K]
    c.s_ps = c.cl.dpref + 8;                                        // [WAVES][16]
    c.cl.stage = p.lds_stage_off ? lds + p.lds_stage_off : nullptr; // [TILE]
    return c;
}

// Stage the vport route image and the interval tables into LDS by LDS-DMA
// (completion: the caller's __syncthreads()).
// (one LDS-DMA loop for all of them: lds_stage_all)
template <int FW, int LPM>
__device__ __forceinline__ void stage_tables(const CopKParams &p, const Tables &tb, int lane, int wave)
{
    constexpr bool fw = FW == COPK_TBL_IVT, lpm = LPM == COPK_TBL_IVT, trie = LPM == COPK_TBL_TRIE;
    const StageSeg none{nullptr, nullptr, 0u};
    lds_stage_all(StageSeg{p.rt_top, tb.rt_top, 64u}, StageSeg{p.rt_leaf, (uint32_t *)tb.rt_leaf, p.rt_nleaf * 32u},
                  fw ? StageSeg{p.fw_starts, tb.fw_s, (p.fw_m + p.fw_iw) >> 2} : none,
                  fw ? StageSeg{p.fw_vals, tb.fw_v, p.fw_m >> 2} : none,
                  lpm ? StageSeg{p.lpm_starts, tb.lp_s, (p.lpm_m + p.lpm_iw) >> 2}
                      : trie ? StageSeg{p.lpm_tl0, tb.lp_s, COPK_TRIE_L0 / 4u} : none,
                  lpm ? StageSeg{p.lpm_vals, tb.lp_v, p.lpm_m >> 2} : none, lane, wave);
}

// Per-rule hit binning (CopKParams::hit_region): the LDS of the tile's sort
struct HitLds {
    uint32_t *cnt;    // [nb] hits per bucket
    uint32_t *cur;    // [nb] write cursor per bucket
    uint32_t *wsum;   // [4] per-wave scan totals
    uint32_t *off;    // [nb + 1] run starts, then the end
    uint32_t *tmp;    // [TILE] each packet's hit rule id or ~0u, in tile order
    uint32_t *ids;    // [hit_reg_words] the tile's ids, bucket by bucket
};

template <int PPT>
__device__ __forceinline__ HitLds hit_lds(const CopKParams &p, uint32_t *lds)
{
    HitLds h;
    const uint32_t nb = p.hit_nb;
    h.cnt = lds + p.lds_hit_off;
    h.cur = h.cnt + nb;
    h.wsum = h.cur + nb;
    h.off = h.wsum + 4;
    h.tmp = h.cnt + ((3u * nb + 5u + 3u) & ~3u);   // 16-byte aligned
    h.ids = h.tmp + BLOCK * PPT;
    return h;
}

// the tile's FW hits: per-bucket counts (LDS adds; cnt zeroed before the
// tile) and each packet's rule id parked in LDS, so nothing stays in
// registers until the sort
template <int PPT>
__device__ __forceinline__ void hit_hist(const HitLds &h, const bool (&valid)[PPT], const uint32_t (&flags)[PPT],
                                         const uint32_t (&fwe)[PPT], int tid, bool one)
{
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        const bool hit = valid[k] && (flags[k] & COPK_FLAG_FW_HIT);
        const uint32_t id = fwe[k] & 0x00FFFFFFu;
        if (hit && !one) atomicAdd(&h.cnt[id >> COPK_HIT_SHIFT], 1u);
        h.tmp[k * BLOCK + tid] = hit ? id : 0xFFFFFFFFu;
    }
}

// After a barrier that follows hit_hist: scan the bucket counts (each run
// padded to 4 ids), place every hit's rule id in its bucket's run, and write
// the runs (16-byte stores) and their offsets to the tile's region.
template <int PPT, bool WT>
__device__ __forceinline__ void hit_sort_out(const CopKParams &p, const HitLds &h, int tid, int lane, int wave,
                                             size_t tile)
{
    const uint32_t nb = p.hit_nb;
    uint32_t total;
    if (nb == 1) {
        // one bucket: no sort, the hits in tile order by a block-wide scan
        // of each lane's hit count (no LDS atomics on one word)
        uint32_t mine = 0;
#pragma unroll
        for (int k = 0; k < PPT; k++) mine += h.tmp[k * BLOCK + tid] != 0xFFFFFFFFu;
        uint32_t agg;
        const uint32_t ex = wave_excl_scan(mine, 64, lane, &agg);
        if (lane == 0) h.wsum[wave] = agg;
        lds_barrier();
        uint32_t pos = ex, all = 0;
        for (int w = 0; w < WAVES; w++) {
            pos += w < wave ? h.wsum[w] : 0u;
            all += h.wsum[w];
        }
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            const uint32_t id = h.tmp[k * BLOCK + tid];
            if (id != 0xFFFFFFFFu) h.ids[pos++] = id;
        }
        total = (all + 3u) & ~3u;
        if ((uint32_t)tid < total - all) h.ids[all + tid] = 0xFFFFFFFFu;
        if (tid == 0) {
            h.off[0] = 0;
            h.off[1] = total;
        }
        lds_barrier();
    } else {
        const uint32_t c = (uint32_t)tid < nb ? h.cnt[tid] : 0u;
        const uint32_t v = (c + 3u) & ~3u;
        uint32_t agg;
        const uint32_t ex = wave_excl_scan(v, 64, lane, &agg);
        if (lane == 0) h.wsum[wave] = agg;
        lds_barrier();
        uint32_t start = ex;
        for (int w = 0; w < wave; w++) start += h.wsum[w];
        if ((uint32_t)tid < nb) {
            h.off[tid] = start;
            h.cur[tid] = start;
            for (uint32_t i = c; i < v; i++) h.ids[start + i] = 0xFFFFFFFFu;
            if ((uint32_t)tid == nb - 1) h.off[nb] = start + v;
        }
        lds_barrier();
        for (int k = 0; k < PPT; k++) {
            const uint32_t id = h.tmp[k * BLOCK + tid];
            if (id != 0xFFFFFFFFu) h.ids[atomicAdd(&h.cur[id >> COPK_HIT_SHIFT], 1u)] = id;
        }
        lds_barrier();
        total = h.off[nb];
    }
    uint32_t *reg = p.hit_region + tile * p.hit_reg_words;
    for (uint32_t c4 = (uint32_t)tid; c4 < total / 4u; c4 += BLOCK)
        st_u32x4<WT>(*(const u32x4 *)&h.ids[4 * c4], reg, 4 * (long)c4);
    for (uint32_t q = (uint32_t)tid; q <= nb; q += BLOCK) st_u32<WT>(h.off[q], &p.hit_off[tile * (nb + 1) + q]);
}

// IMIX header loads: three cooperative 16-byte loads per lane and step at
// the packets' offsets (load_step_imix), or (0) per-lane loads of bytes
// 12..27 and 28..35. FW + LPM 100k IMIX at the driver's 20 steps: 36,664 /
// 36,881 / 37,028 against 31,232 / 33,901 / 31,254 Mpkt/s, the one-shot
// kernel's frac 0.479-0.482 against 0.449-0.486 (profiles/r06/check4/abx_*)
#ifndef COPK_IMIX_COOP
#define COPK_IMIX_COOP 1
#endif
// IMIX with the route's DIR-24-8 on the poll-mode step path (tile_steps_v):
// the offsets, header loads, tbl24 and tbl8 probes of successive steps
// pipelined (1), or the whole-tile body (0)
#ifndef COPK_IMIX_STEPS
#define COPK_IMIX_STEPS 1
#endif
// The bucketed route form (COP_CFG_LPM_BKT) on the step path too: its
// index and pair rounds pipelined across steps like DIR-24-8's tbl24 and
// tbl8 probes (1), or the whole-tile body (0)
#ifndef COPK_BKT_STEPS
#define COPK_BKT_STEPS 1
#endif

// Whether a tile can run step by step (tile_steps): segmented lists, no
// optional feature, the firewall in LDS, and coalesced 64-byte slots with
// the route in LDS or DIR-24-8 (whose two dependent probes tile_steps_v
// pipelines across steps; the trie's and the bucketed form's chains are
// not; the bucketed form's two rounds are, COPK_BKT_STEPS), or IMIX with a
// DIR-24-8 or bucketed route.
template <int FW, int LPM, int LAY, bool EXT>
constexpr bool steps_ok()
{
    return !EXT && FW != COPK_TBL_DIR && FW != COPK_TBL_BKT &&
           ((LAY == COPK_LAY_COALESCED && LPM != COPK_TBL_TRIE && (LPM != COPK_TBL_BKT || COPK_BKT_STEPS)) ||
            (LAY == COPK_LAY_IMIX && COPK_IMIX_STEPS &&
             (LPM == COPK_TBL_DIR || (LPM == COPK_TBL_BKT && COPK_BKT_STEPS))));
}

// One tile of the poll-mode kernel, step by step (tile_body does the same
// work pass by pass). The header loads of all PPT steps go out first; then
// each step, as its loads land, is classified and finished: its records
// (16-byte write-through stores from lane pairs), its list segment (one
// barrier for the four waves' counts, then each forwarded lane writes its
// index) and its segment length. The counters are folded into the last
// step's barrier. So when a worker's last loads land (the CU serves its
// workers' loads about in order: the last worker's after everything else),
// one step is left to finish, not the whole tile. Same outputs as tile_body.
// experiment builds only (timing ablations, wrong results): COPK_XP bit 1 =
// no classification, 2 = no records, 4 = no list stores and no barrier
#ifndef COPK_XP
#define COPK_XP 0
#endif
// Steps of a tile whose header loads are in flight at once per wave: one.
// A CU serves its five workers' requests about in issue order, so the more
// steps each wave issues up front, the later the CU's last worker gets its
// data. With one step in flight a wave issues its next
// step's loads as it gathers the current one, and the workers' requests
// interleave. The driver's 20-batch post: four steps 44.4-45.4, two
// 45.8-47.2 (profiles/r05/check5/, check6/), one 51.5-52.2 against two's
// 46.9-47.3 in three alternating pairs on one box (check8/); the poll-mode
// steady state is the same. It also leaves room for the next tile's first
// step (dynamic tiles).
#ifndef COPK_PMD_WIN
#define COPK_PMD_WIN 1
#endif
// experiment builds: the window of the route's DIR-24-8 step pipeline
#ifndef COPK_PMD_WIN_DIR
#define COPK_PMD_WIN_DIR COPK_PMD_WIN
#endif
template <int PPT, int WIN>
constexpr int win_of()
{
    return WIN < PPT ? WIN : PPT;
}
// Wave priority by progress: s_setprio 3 for a tile's first step down to 0
// for its last step and while the worker waits. A SIMD issues from the
// highest-priority ready wave, then the oldest, so without it the CU's
// oldest workers issue (and get their data) first and its youngest worker
// finishes last. With it a wave that is a step behind issues first. The
// driver's 20-batch post: 53.8 / 53.7 / 52.8 against 50.7 / 51.5 / 51.1
// Gpkt/s, poll-mode steady state 0.59-0.61 against 0.56-0.57, the spread
// between a CU's first and fifth worker 2.0 against 3.3 us
// (profiles/r05/check10/, three alternating pairs on one box)
#ifndef COPK_PMD_PRIO
#define COPK_PMD_PRIO 1
#endif
template <int K>
__device__ __forceinline__ void step_prio()
{
    if constexpr (COPK_PMD_PRIO) __builtin_amdgcn_s_setprio(K >= 3 ? 0 : 3 - K);
}
// experiment builds: the same for the poll-mode tile body (global-probe
// lookups), by phase: headers, lookups, outputs
#ifndef COPK_PMD_PRIO_BODY
#define COPK_PMD_PRIO_BODY 0
#endif
template <bool WT, int K>
__device__ __forceinline__ void body_prio()
{
    if constexpr (WT && COPK_PMD_PRIO_BODY) step_prio<K>();
}
// the step's forward-list segment through LDS and out as 16-byte stores
#ifndef COPK_PMD_STAGE_LIST
#define COPK_PMD_STAGE_LIST 1
#endif
// Segments per wave (1024-packet tiles): wave w of a tile owns the tile's
// segment w (packets w*256 .. w*256+255) and walks it in four steps of 64
// packets, so a segment's list is one wave's own forwarded packets in order
// and no step waits at a barrier for the other waves' counts (one barrier
// per tile, for the counters). Against step k = segment k with a barrier per
// step (COPK_SEG_WAVE=0): the driver's command 55,253 / 54,380 / 53,711
// against 52,950 / 51,901 / 53,188 Mpkt/s, a one-batch post 13.0 against
// 14.6 us, a lone tile's body 7.4 against 8.7 us (profiles/r05/check23/).
#ifndef COPK_SEG_WAVE
#define COPK_SEG_WAVE 1
#endif
// With segments per wave, each wave also adds its own counters (nine lanes,
// a shard of its own) and the tile has no barrier left: the driver's command
// 55,417 / 56,131 / 55,461 against 52,822 / 52,673 / 53,930 Mpkt/s, three
// alternating pairs (profiles/r05/check25/; COPK_WAVE_COUNTERS=0 reduces
// the four waves' counters through LDS behind a barrier)
#ifndef COPK_WAVE_COUNTERS
#define COPK_WAVE_COUNTERS 1
#endif
// the first packet of wave `wave`'s 64 packets in step k, from the tile's base
template <int PPT>
__device__ __forceinline__ uint32_t step_off(int k, int wave)
{
    if constexpr (COPK_SEG_WAVE && PPT == WAVES) return (uint32_t)(wave * PPT * 64 + k * 64);
    else return (uint32_t)(k * BLOCK + wave * 64);
}

// The header loads of steps K0 .. K1 - 1 of a tile (of tile_steps_v's
// window: K1 <= W, all PPT steps when W == PPT): issued, not waited for.
// SYS: plain loads (0), system-coherent loads (1), or the run-time choice
// sys_rt (2). A run-time choice between two load forms writing the same
// registers makes the compiler's wait insertion put vmcnt waits before the
// coherent form (for the other form's loads, on a path that never runs),
// which wait for every store and probe still in flight; so the static order
// picks 0 or 1 per tile (cop_pmd.hip). The dynamic order keeps 2: two
// instantiations there hold more load registers than fit.
template <int PPT, int K0, int K1, int SYS = 2, int WIN = COPK_PMD_WIN>
__device__ __forceinline__ void steps_load(const CopKBatch &B, uint32_t j, int lane, int wave,
                                           u32x4 (&v)[win_of<PPT, WIN>()][3], bool sys_rt = false)
{
    const bool sys = SYS == 2 ? sys_rt : SYS == 1;
    static_assert(K1 <= win_of<PPT, WIN>(), "steps beyond the window");
    const StepGeom sg = step_geom(lane);
    const uint32_t base = j * (BLOCK * PPT);
    const uint32_t last = B.n ? B.n - 1 : 0u;
#pragma unroll
    for (int k = K0; k < K1; k++)
        load_step(sg, B.pkts + B.data_off, B.stride, base + step_off<PPT>(k, wave), last, v[k], sys);
}

// v: the tile's first W steps as steps_load issued them. SYS: the later
// steps' loads are system-coherent too (as steps_load's were: a reused or
// host-memory slot, cop_pmd.hip)
template <int FW, int LPM, int PPT, bool WT, int SYS = 2, int WIN = COPK_PMD_WIN,
          bool STAGE_LIST = COPK_PMD_STAGE_LIST, int LAY = COPK_LAY_COALESCED>
__device__ __forceinline__ void tile_steps_v(const CopKParams &p, const LdsCarve &lc, const CopKBatch &B, uint32_t j,
                                             int tid, int lane, int wave, u32x4 (&v)[win_of<PPT, WIN>()][3],
                                             bool sys_rt = false)
{
    const bool sys = SYS == 2 ? sys_rt : SYS == 1;
    static_assert(COPK_SEG == BLOCK, "one segment per tile step");
    const Tables &tb = lc.tb;
    constexpr int TILE = BLOCK * PPT;
    const uint32_t base = j * TILE;
    const uint32_t last = B.n ? B.n - 1 : 0u;
    const StepGeom sg = step_geom(lane);
    // a window of W steps in flight: step k + W is loaded once step k is
    // gathered, so the CU's queue holds every worker's early steps before
    // any worker's late ones and the workers' last steps land together
    constexpr int W = win_of<PPT, WIN>();
    Counts tot;
    uint32_t *r = (uint32_t *)B.results;
    const int i2 = lane & 31;
    // Staged lists: each step's forward-list segment is written into LDS and
    // leaves as 16-byte stores (whole chunks, the last clamped to n) once a
    // later barrier has ordered it. Write-through stores of single words,
    // one per forwarded lane, cost the poll-mode kernel's steady state 9 %.
    const bool staged = STAGE_LIST && B.fwd_idx && lc.cl.stage && !(COPK_XP & 4);
    uint32_t all_prev = 0;
    auto flush = [&](int k, uint32_t len) {
        const uint32_t cc = (uint32_t)wave * 16u + (uint32_t)(lane & 15);
        const uint32_t pk = base + (uint32_t)k * BLOCK;
        if (lane < 16 && cc * 4u < len)
            st_list_chunk<WT>(&lc.cl.stage[k * BLOCK + cc * 4u], B.fwd_idx, pk + cc * 4u, B.n);
    };
    // step k's outputs once its verdicts are known: counts, records (lane
    // i < 32 stores records 2i, 2i+1 of the wave's 64 packets as one 16-byte
    // write-through store), the list segment and, after the last step, the
    // counters
    uint32_t run = 0;   // COPK_SEG_WAVE: the wave's segment list so far
    auto emit = [&](int k, bool valid0, uint32_t verdict0, uint32_t flags0, uint32_t port0, uint32_t rnh0) {
        const uint32_t pk0 = base + k * BLOCK;
        const uint32_t wb = base + step_off<PPT>(k, wave);   // this wave's 64 packets
        const bool valid[1] = {valid0};
        const uint32_t verdict[1] = {verdict0}, flags[1] = {flags0};
        const Counts c = wave_counts<FW, 1>(valid, verdict, flags);
        tot.total += c.total;
        tot.notv4 += c.notv4;
        tot.fwd += c.fwd;
        tot.dropfw += c.dropfw;
        tot.parse += c.parse;
        tot.noport += c.noport;
        tot.rhit += c.rhit;
        tot.rx += c.rx;
        const unsigned long long bal = __ballot(valid0 && verdict0 == COPK_FORWARD);
        if (lane == 0) {
            lc.cl.cnt[k * WAVES + wave] = (uint32_t)__popcll(bal);
            if (k == PPT - 1) {
                const uint32_t c8[8] = {tot.total, tot.notv4, tot.fwd, tot.dropfw, tot.parse, tot.noport, tot.rhit,
                                        tot.rx};
#pragma unroll
                for (int q = 0; q < 8; q++) lc.s_red[wave * 8 + q] = c8[q];
            }
        }
        const uint32_t rx = verdict0 | (flags0 << 8) | (port0 << 16);
        const uint32_t a0 = (uint32_t)__shfl((int)rx, 2 * i2), a1 = (uint32_t)__shfl((int)rnh0, 2 * i2);
        const uint32_t a2 = (uint32_t)__shfl((int)rx, 2 * i2 + 1), a3 = (uint32_t)__shfl((int)rnh0, 2 * i2 + 1);
        const uint32_t idx = wb + 2u * (uint32_t)i2;
        if (lane < 32 && !(COPK_XP & 2)) {
            if (idx + 1 < B.n) st_u32x4<WT>(u32x4{a0, a1, a2, a3}, r, 2 * (long)idx);
            else if (idx < B.n) st_u32x2<WT>(u32x2{a0, a1}, (u32x2 *)&r[2 * (size_t)idx]);
        }
        if (COPK_XP & 4) {
            if (k == PPT - 1) {
                lds_barrier();
                counters_add(p, lc.s_red, tid);
            }
            return;
        }
        if constexpr (COPK_SEG_WAVE && PPT == WAVES) {
            // segment w = this wave's: its list is the wave's own forwarded
            // packets in order (no other wave's counts needed)
            const uint32_t sb = base + (uint32_t)wave * COPK_SEG;
            const uint32_t rank = run + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
            if (staged) {
                if ((bal >> lane) & 1ull) lc.cl.stage[wave * COPK_SEG + rank] = wb + (uint32_t)lane;
            } else if (B.fwd_idx && ((bal >> lane) & 1ull)) {
                st_u32<WT>(wb + (uint32_t)lane, &B.fwd_idx[sb + rank]);
            }
            run += (uint32_t)__popcll(bal);
            if (k == PPT - 1) {
                if (staged) {
                    // read back by the wave's other lanes: LDS operations of one
                    // wave complete in order; keep the compiler from moving them
                    asm volatile("" ::: "memory");
                    if ((uint32_t)lane * 4u < run)
                        st_list_chunk<WT>(&lc.cl.stage[wave * COPK_SEG + lane * 4], B.fwd_idx, sb + (uint32_t)lane * 4u,
                                          B.n);
                }
                if (B.fwd_count && lane == 0 && sb < B.n) st_u32<WT>(run, B.fwd_count + sb / COPK_SEG);
                if (COPK_WAVE_COUNTERS) {
                    counters_add_wave(p, tot, lane, blockIdx.x * WAVES + (uint32_t)wave);
                } else {
                    lds_barrier();   // every wave's counters in s_red
                    counters_add(p, lc.s_red, tid);
                }
            }
            return;
        }
        lds_barrier();
        // the step's segment: this wave's forwarded packets after the lower
        // waves' ones, in lane order
        uint32_t off = 0, all = 0;
#pragma unroll
        for (int w = 0; w < WAVES; w++) {
            const uint32_t cw = lc.cl.cnt[k * WAVES + w];
            off += w < wave ? cw : 0u;
            all += cw;
        }
        const uint32_t rank = off + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
        if (staged) {
            // the segment's list through LDS; it goes out after the next
            // step's barrier (the last one's after the loop)
            if (k > 0) flush(k - 1, all_prev);
            if ((bal >> lane) & 1ull) lc.cl.stage[k * BLOCK + rank] = pk0 + tid;
            all_prev = all;
        } else if (B.fwd_idx && ((bal >> lane) & 1ull)) {
            st_u32<WT>(pk0 + tid, &B.fwd_idx[pk0 + rank]);
        }
        if (B.fwd_count && tid == 0 && pk0 < B.n) st_u32<WT>(all, B.fwd_count + pk0 / COPK_SEG);
        if (k == PPT - 1) counters_add(p, lc.s_red, tid);
    };
    auto prio = [&](int k) {
        if (COPK_PMD_PRIO) {
            if (k == 0) step_prio<0>();   // (a prefetched tile starts at the waiting priority)
            else if (k == 1) step_prio<1>();
            else if (k == 2) step_prio<2>();
            else if (k == 3) step_prio<3>();
        }
    };
    if constexpr (LAY == COPK_LAY_IMIX) {
        // IMIX (a slab with u32 offsets): five stages across steps, each
        // round waiting only for loads the previous round issued. Round k:
        // step k's headers (landed) are gathered and classified and its
        // tbl24 probe issued; step k + 1's header loads go out at its
        // offsets (landed); step k + 2's offsets are loaded; step k - 1's
        // tbl8 load is issued; step k - 2 is finished and written out. The
        // prologue loads step 0's offsets, then its headers and step 1's
        // offsets. (The whole-tile body instead waits for every step's
        // offsets, then every step's headers, then the probes: four
        // dependent round trips with nothing else in flight.)
        static_assert((LPM == COPK_TBL_DIR || LPM == COPK_TBL_BKT) && FW != COPK_TBL_DIR && FW != COPK_TBL_BKT,
                      "IMIX steps: DIR-24-8 or bucketed route");
        struct St {
            uint32_t w3, src, dst, verdict, port, fwe, lpe, lpe2;
            bool valid;
            T8 t8;
            BkQ bq;
        };
        St a{}, b{}, c{};
        u32x4 h[3];
        uint32_t off = load_off_imix(B.offsets, base + step_off<PPT>(0, wave), lane, last, sys);
        load_step_imix(sg, B.pkts, off, B.data_off, h, sys);
        if (PPT > 1) off = load_off_imix(B.offsets, base + step_off<PPT>(1, wave), lane, last, sys);
#pragma unroll
        for (int k = 0; k < PPT + 2; k++) {
            if (k < PPT) {
                uint32_t w3[1], w6[1], w7[1], w8[1];
                prio(k);
                gather_step(sg, h, w3[0], w6[0], w7[0], w8[0]);
                uint32_t verdict[1], port[1], fwe[1], lpe[1], lpe2[1], fwe2[1], src[1], dst[1];
                pass1<FW, LPM, 1>(p, tb, w3, w6, w7, w8, verdict, port, src, dst, fwe, lpe, lpe2, fwe2);
                a = St{w3[0], src[0], dst[0], verdict[0], port[0], fwe[0], lpe[0], lpe2[0],
                       base + step_off<PPT>(k, wave) + (uint32_t)lane < B.n && B.n != 0, T8{false, 0ull}, BkQ{}};
                if (k + 1 < PPT) {
                    load_step_imix(sg, B.pkts, off, B.data_off, h, sys);
                    if (k + 2 < PPT) off = load_off_imix(B.offsets, base + step_off<PPT>(k + 2, wave), lane, last, sys);
                }
            }
            if (k >= 1 && k <= PPT) {
                if constexpr (LPM == COPK_TBL_BKT) b.bq = bkt_pairs_issue(p.lpm_bpairs, b.lpe, b.verdict == COPK_FORWARD);
                else b.t8 = tbl8_issue(p.lpm_tbl8, p.lpm_tbl8_packed, b.dst, b.lpe);
            }
            if (k >= 2) {
                const uint32_t w3[1] = {c.w3}, src[1] = {c.src}, dst[1] = {c.dst}, lpe2[1] = {0}, fwe2[1] = {0};
                const bool valid[1] = {c.valid};
                uint32_t verdict[1] = {c.verdict}, fwe[1] = {c.fwe}, flags[1], rnh[1], ct = 0, cn = 0;
                uint32_t lpe[1];
                if constexpr (LPM == COPK_TBL_BKT)
                    lpe[0] = bkt_pairs_finish(p.lpm_bpairs, c.dst, c.lpe, c.lpe2, c.verdict == COPK_FORWARD, c.bq);
                else lpe[0] = tbl8_finish(p.lpm_tbl8, p.lpm_tbl8_packed, c.dst, c.lpe, c.t8);
                pass2<FW, LPM, 1, false>(p, w3, src, dst, valid, fwe, lpe, lpe2, fwe2, verdict, flags, rnh, ct, cn);
                emit(k - 2, valid[0], verdict[0], flags[0], c.port, rnh[0]);
            }
            c = b;
            b = a;
        }
    } else if constexpr (LPM != COPK_TBL_DIR && LPM != COPK_TBL_BKT) {
        // LDS-only lookups: each step classified as its headers land
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            uint32_t w3[1], w6[1], w7[1], w8[1];
            prio(k);
            gather_step(sg, v[k % W], w3[0], w6[0], w7[0], w8[0]);
            if (k + W < PPT)
                load_step(sg, B.pkts + B.data_off, B.stride, base + step_off<PPT>(k + W, wave), last, v[k % W], sys);
            const bool valid[1] = {base + step_off<PPT>(k, wave) + (uint32_t)lane < B.n && B.n != 0};
            uint32_t verdict[1], port[1], flags[1], rnh[1], fwe[1], lpe[1], lpe2[1], fwe2[1], src[1], dst[1], ct = 0,
                cn = 0;
            if (COPK_XP & 1) {
                verdict[0] = (w3[0] ^ w6[0] ^ w7[0] ^ w8[0]) & 1u;
                port[0] = w7[0] & 3u;
                flags[0] = 0;
                rnh[0] = w8[0];
            } else {
                pass1<FW, LPM, 1>(p, tb, w3, w6, w7, w8, verdict, port, src, dst, fwe, lpe, lpe2, fwe2);
                pass2<FW, LPM, 1>(p, w3, src, dst, valid, fwe, lpe, lpe2, fwe2, verdict, flags, rnh, ct, cn);
            }
            emit(k, valid[0], verdict[0], flags[0], port[0], rnh[0]);
        }
    } else {
        // The route's DIR-24-8 probes: two dependent global loads per packet
        // (tbl24, then tbl8 for an extended entry: most wave-steps have one);
        // or the bucketed form's two L2 rounds (the bucket index, then eight
        // pairs), the same pipeline.
        // A three-step pipeline keeps them off the step's critical path: in
        // round k, step k's headers are gathered and classified and its tbl24
        // probe issued, step k - 1's tbl8 load is issued (its tbl24 entry has
        // landed), and step k - 2 is finished and written out.
        static_assert(FW != COPK_TBL_DIR && FW != COPK_TBL_BKT, "firewall lookups in LDS only");
        struct St {
            uint32_t w3, src, dst, verdict, port, fwe, lpe, lpe2;
            bool valid;
            T8 t8;
            BkQ bq;
        };
        St a{}, b{}, c{};
#pragma unroll
        for (int k = 0; k < PPT + 2; k++) {
            if (k < PPT) {
                uint32_t w3[1], w6[1], w7[1], w8[1];
                prio(k);
                gather_step(sg, v[k % W], w3[0], w6[0], w7[0], w8[0]);
                if (k + W < PPT)
                    load_step(sg, B.pkts + B.data_off, B.stride, base + step_off<PPT>(k + W, wave), last, v[k % W],
                              sys);
                uint32_t verdict[1], port[1], fwe[1], lpe[1], lpe2[1], fwe2[1], src[1], dst[1];
                pass1<FW, LPM, 1>(p, tb, w3, w6, w7, w8, verdict, port, src, dst, fwe, lpe, lpe2, fwe2);
                a = St{w3[0], src[0], dst[0], verdict[0], port[0], fwe[0], lpe[0], lpe2[0],
                       base + step_off<PPT>(k, wave) + (uint32_t)lane < B.n && B.n != 0, T8{false, 0ull}, BkQ{}};
            }
            if (k >= 1 && k <= PPT) {
                if constexpr (LPM == COPK_TBL_BKT) b.bq = bkt_pairs_issue(p.lpm_bpairs, b.lpe, b.verdict == COPK_FORWARD);
                else b.t8 = tbl8_issue(p.lpm_tbl8, p.lpm_tbl8_packed, b.dst, b.lpe);
            }
            if (k >= 2) {
                const uint32_t w3[1] = {c.w3}, src[1] = {c.src}, dst[1] = {c.dst}, lpe2[1] = {0}, fwe2[1] = {0};
                const bool valid[1] = {c.valid};
                uint32_t verdict[1] = {c.verdict}, fwe[1] = {c.fwe}, flags[1], rnh[1], ct = 0, cn = 0;
                uint32_t lpe[1];
                if constexpr (LPM == COPK_TBL_BKT)
                    lpe[0] = bkt_pairs_finish(p.lpm_bpairs, c.dst, c.lpe, c.lpe2, c.verdict == COPK_FORWARD, c.bq);
                else lpe[0] = tbl8_finish(p.lpm_tbl8, p.lpm_tbl8_packed, c.dst, c.lpe, c.t8);
                pass2<FW, LPM, 1, false>(p, w3, src, dst, valid, fwe, lpe, lpe2, fwe2, verdict, flags, rnh, ct, cn);
                emit(k - 2, valid[0], verdict[0], flags[0], c.port, rnh[0]);
            }
            c = b;
            b = a;
        }
    }
    if (staged && !(COPK_SEG_WAVE && PPT == WAVES)) {
        lds_barrier();
        flush(PPT - 1, all_prev);
    }
    step_prio<3>();
}

// One tile of the poll-mode kernel, step by step: loads, then tile_steps_v
// (IMIX: tile_steps_v issues every load itself)
template <int FW, int LPM, int PPT, bool WT, int SYS, int WIN = COPK_PMD_WIN, int LAY = COPK_LAY_COALESCED>
__device__ __forceinline__ void tile_steps(const CopKParams &p, const LdsCarve &lc, const CopKBatch &B, uint32_t j,
                                           int tid, int lane, int wave)
{
    u32x4 v[win_of<PPT, WIN>()][3];
    step_prio<0>();
    if constexpr (LAY != COPK_LAY_IMIX) steps_load<PPT, 0, win_of<PPT, WIN>(), SYS, WIN>(B, j, lane, wave, v);
    tile_steps_v<FW, LPM, PPT, WT, SYS, WIN, COPK_PMD_STAGE_LIST, LAY>(p, lc, B, j, tid, lane, wave, v);
}

// One tile of 256 * PPT packets (base = j * TILE) of batch B: header loads,
// parse/route, lookups, verdicts, records, ordered compaction and the
// counter flush. Shared by the one-shot kernel (one tile per workgroup)
// and the poll-mode kernel (cop_pmd.hip: a persistent loop over tiles).
// WT: write-through output stores (poll-mode). sync_tables: wait for the
// LDS-DMA table staging after the header loads are issued. hit_tile: the
// tile's binned-hit region index (one-shot: blockIdx; poll mode: its slot's
// tile). Returns false when the tile's look-back gave up (poll-mode abort):
// the tile must not be counted as done (workgroup-uniform).
template <int FW, int LPM, int LAY, int PPT, bool EXT, bool WT>
__device__ __forceinline__ bool tile_body(const CopKParams &p, const Opt &o, const LdsCarve &lc, const CopKBatch &B,
                                          uint32_t look_off, uint32_t j, const LookCtx &lk, int tid, int lane, int wave,
                                          bool sync_tables, size_t hit_tile, bool sys = false)
{
    constexpr bool IMIX = LAY == COPK_LAY_IMIX;
    const Tables &tb = lc.tb;
    constexpr int TILE = BLOCK * PPT;
    const uint32_t base = j * TILE;
    // ---- packet header loads (all PPT packets, no branches). Lanes past
    // the end of the batch re-read the last packet and are masked out of
    // every store and count. ----
    uint32_t w3[PPT], w6[PPT], w7[PPT], w8[PPT];
    bool valid[PPT];
    const uint32_t last = B.n ? B.n - 1 : 0u;
    if (LAY == COPK_LAY_COALESCED && B.n) {
        const StepGeom sg = step_geom(lane);
#if defined(COPK_STREAM_W) && COPK_STREAM_W > 0
        // experiment builds: a window of W steps in flight; step k + W is
        // loaded into step k's registers once step k is gathered
        constexpr int W = COPK_STREAM_W < PPT ? COPK_STREAM_W : PPT;
        u32x4 v[W][3];
#pragma unroll
        for (int k = 0; k < W; k++) load_step(sg, B.pkts + B.data_off, B.stride, base + k * BLOCK + wave * 64, last, v[k], sys);
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            gather_step(sg, v[k % W], w3[k], w6[k], w7[k], w8[k]);
            if (k + W < PPT) {
                __builtin_amdgcn_sched_barrier(0);
                load_step(sg, B.pkts + B.data_off, B.stride, base + (k + W) * BLOCK + wave * 64, last, v[k % W], sys);
            }
        }
#else
        u32x4 v[PPT][3];
#pragma unroll
        for (int k = 0; k < PPT; k++)
            load_step(sg, B.pkts + B.data_off, B.stride, base + k * BLOCK + wave * 64, last, v[k], sys);
#pragma unroll
        for (int k = 0; k < PPT; k++) gather_step(sg, v[k], w3[k], w6[k], w7[k], w8[k]);
#endif
    } else if (IMIX && COPK_IMIX_COOP && B.n) {
        // IMIX: the offsets (coalesced), then three cooperative 16-byte loads
        // per lane and step at the packets' offsets (load_step_imix)
        const StepGeom sg = step_geom(lane);
        uint32_t off[PPT];
#pragma unroll
        for (int k = 0; k < PPT; k++) off[k] = load_off_imix(B.offsets, base + k * BLOCK + wave * 64, lane, last, sys);
        u32x4 v[PPT][3];
#pragma unroll
        for (int k = 0; k < PPT; k++) load_step_imix(sg, B.pkts, off[k], B.data_off, v[k], sys);
#pragma unroll
        for (int k = 0; k < PPT; k++) gather_step(sg, v[k], w3[k], w6[k], w7[k], w8[k]);
    } else if (LAY == COPK_LAY_HDR16 && B.n && B.stride == 12u) {
        // one 12-byte record per packet (COP_HDR12_STRIDE, one-shot batches):
        // frame bytes 12..15, then 26..29 (src) and 30..33 (dst); bytes
        // 24..35 rebuilt around them as pass1 reads them (the rest unread)
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            const uint32_t ic = min(base + k * BLOCK + tid, last);
            const uint32_t *r = (const uint32_t *)(B.pkts + B.data_off + (size_t)ic * 12u);
            const uint32_t a = __builtin_nontemporal_load(r), s_ = __builtin_nontemporal_load(r + 1),
                           d_ = __builtin_nontemporal_load(r + 2);
            w3[k] = a;
            w6[k] = s_ << 16;
            w7[k] = (s_ >> 16) | (d_ << 16);
            w8[k] = d_ >> 16;
        }
    } else if (LAY == COPK_LAY_HDR16 && B.n) {
        // one 16-byte record per packet: frame bytes 12..15 then 24..35
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            const uint32_t ic = min(base + k * BLOCK + tid, last);
            const u32x4 v = sys ? ld_sys16(sys_rsrc(B.pkts + B.data_off), ic * 16u)
                                : __builtin_nontemporal_load((const u32x4 *)(B.pkts + B.data_off + (size_t)ic * 16u));
            w3[k] = v.x;
            w6[k] = v.y;
            w7[k] = v.z;
            w8[k] = v.w;
        }
    } else if (B.n) {
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            const uint32_t ic = min(base + k * BLOCK + tid, last);
            if (sys) {
                // the offset array and the packet, system-coherent
                const uint32_t po = (IMIX ? ld_sys4(sys_rsrc(B.offsets), ic * 4u) : ic * B.stride) + B.data_off;
                const __amdgpu_buffer_rsrc_t rs = sys_rsrc(B.pkts);
                const u32x4 a = ld_sys16(rs, po + 12u);
                const u32x2 b = ld_sys8(rs, po + 28u);
                w3[k] = a.x;
                w6[k] = a.w;
                w7[k] = b.x;
                w8[k] = b.y;
                continue;
            }
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
    if (sync_tables) __syncthreads();   // LDS-DMA table staging has landed
    body_prio<WT, 1>();

    // ---- pass 1 (parse, route, LDS searches, tbl24 loads issued) ----
    uint32_t verdict[PPT], port[PPT], flags[PPT], rnh[PPT], fwe[PPT], lpe[PPT], lpe2[PPT], fwe2[PPT], src[PPT], dst[PPT];
    pass1<FW, LPM, PPT>(p, tb, w3, w6, w7, w8, verdict, port, src, dst, fwe, lpe, lpe2, fwe2);
    if (o.dbg & 8u) {
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < PPT; k++) x ^= verdict[k] ^ src[k];
        asm volatile("" ::"v"(x));
    }
    STAMP(2);

    // ---- pass 2 (tbl8 step) and the verdicts ----
    Counts cn;
    pass2<FW, LPM, PPT>(p, w3, src, dst, valid, fwe, lpe, lpe2, fwe2, verdict, flags, rnh, cn.total, cn.notv4);
    body_prio<WT, 2>();
    const bool bins = EXT && FW != COPK_TBL_OFF && p.hit_region != nullptr;
    // segmented lists with no optional feature: the lean epilogue (counters
    // from ballots, folded into the list's barriers)
    if (!EXT && p.seg && p.compact && !(o.dbg & 64u)) {
        STAMP(3);
        const bool paired = p.rec_paired != 0;
        bool fwd[PPT];
        Counts dummy;
        auto records = [&] {
            if (paired) store_records_paired<PPT, WT>(B, base, tid, lane, wave, valid, verdict, flags, port, rnh, fwd, dummy);
            else store_records<PPT, WT>(B, base, tid, valid, verdict, flags, port, rnh, fwd, dummy, nullptr);
        };
        seg_epilogue<FW, PPT, WT>(p, B, base, valid, verdict, flags, lc.cl, lc.s_red, tid, lane, wave, records);
        STAMP(5);
        STAMP(6);
        return true;
    }
    if (bins) hit_hist<PPT>(hit_lds<PPT>(p, lc.s_misc - p.lds_misc_off), valid, flags, fwe, tid, p.hit_nb == 1);
    else rule_hit_atomics<FW, PPT>(o, valid, flags, fwe);
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
    uint32_t *rec_stage = (WT && p.lds_rec_off) ? lc.s_misc - p.lds_misc_off + p.lds_rec_off : nullptr;
    const bool paired = p.rec_paired != 0;
    auto records = [&] {
        if (paired) store_records_paired<PPT, WT>(B, base, tid, lane, wave, valid, verdict, flags, port, rnh, fwd, cn);
        else store_records<PPT, WT>(B, base, tid, valid, verdict, flags, port, rnh, fwd, cn, rec_stage);
    };
    bool ok = true;
    if (p.compact)
        ok = compact_tile<PPT, WT>(lk, o, B, look_off, j, base, fwd, port, p.seg != 0, lc.cl, tid, lane, wave, records);
    else records();
    if (rec_stage) {
        // compact_tile's second barrier (or this one) orders the staged records
        if (!p.compact) lds_barrier();
        copy_out_records<WT>(B.results, base, B.n > base ? min(B.n - base, (uint32_t)TILE) : 0u, rec_stage, tid);
    }
    STAMP(5);
    if (!ok) return false;   // gave up (abort): no counters, no hit region

    // ---- counters (one flush per workgroup) ----
    uint32_t prx[COPK_MAX_DEMUX_PORTS] = {}, ptx[COPK_MAX_DEMUX_PORTS] = {};
    if (o.port_stats) port_counts<PPT>(o.port_stats, valid, fwd, port, prx, ptx);
    flush_counters(p, o, cn, prx, ptx, lc.s_red, lc.s_ps, tid, lane, wave);
    // (flush_counters' barrier has landed every hit_hist add)
    if (bins) hit_sort_out<PPT, WT>(p, hit_lds<PPT>(p, lc.s_misc - p.lds_misc_off), tid, lane, wave, hit_tile);
    STAMP(6);
    return true;
}

}  // namespace copd

#endif
