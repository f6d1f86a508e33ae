// cop_kernels.hip — the coprocessor NF pipeline as one gfx950 kernel.
//
// One lane handles PPT packets, one workgroup one tile of 256*PPT packets.
// Per packet the kernel restates, in this order (SURVEY.md §8a contract):
//   stage P   get_next_hop            switch.c:93-136  (+ fast-path drop
//             switch.c:406-410, enqueue_nf_rx port bound switch.c:316-319)
//   stage FW  fw_packet_handler       firewall.c:170-213, lookup =
//             rte_lpm_lookup(lpm_tbl, ntohl(src))     firewall.c:194
//   stage LPM route rte_lpm semantics on ntohl(dst)   (north-star extension)
//   compaction: indices of FORWARD packets in arrival order, the order
//             coprocessor() hands them to enqueue_nf_tx (switch.c:464-470).
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

#include "cop_kernels.h"

namespace {

constexpr int BLOCK = COPK_BLOCK;
constexpr int WAVES = BLOCK / 64;

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ void lb_store(unsigned long long *p, unsigned long long v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ unsigned long long lb_load(unsigned long long *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void lds_stage(uint32_t *lds_dst, const void *gsrc, uint32_t n16, int lane,
                                          int wave)
{
    // one 1 KiB piece per wave-instruction: LDS destination = base + lane*16
    const uint4 *g = (const uint4 *)gsrc;
    for (uint32_t c = (uint32_t)wave; c * 64u < n16; c += WAVES) {
        const uint32_t i = c * 64u + (uint32_t)lane;
        if (i < n16)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(g + i),
                                             (__attribute__((address_space(3))) void *)(lds_dst + c * 256u),
                                             16, 0, 0);
    }
}

// Interval search in LDS over an Eytzinger (BFS-order) tree: tree[1..m-1]
// holds the sorted interval starts s[1..m-1] (s[0] == 0 is implicit), m a
// power of two, padding starts 0xFFFFFFFF. Returns k = #{j >= 1 : s[j] <= ip},
// the index of the interval holding ip. The top levels of the tree sit in
// consecutive LDS words, so the first steps of 64 searches are broadcasts or
// conflict-free, unlike a sorted-array search whose step-s probes all share
// one bank.
__device__ __forceinline__ uint32_t eyt_search(const uint32_t *tree, uint32_t levels, uint32_t ip)
{
    uint32_t i = 1;
    for (uint32_t l = 0; l < levels; l++) i = 2u * i + (tree[i] <= ip ? 1u : 0u);
    return i - (1u << levels);
}

// Decoupled look-back over one chain of tile granules (tile t at
// chain[t * stride]): publish this tile's aggregate, read up to 64
// predecessors per round (lane l reads tile qhi-l), consume the ready prefix
// up to and including the nearest inclusive prefix, then publish the
// inclusive value. Granules are {epoch:32, flag:2 (1 aggregate, 2 inclusive),
// value:30}; a stale epoch counts as not ready. Spins are bounded and report
// through the host-mapped error word. Whole wave; returns the exclusive prefix.
__device__ __forceinline__ uint32_t look_back(unsigned long long *chain, uint32_t stride, uint32_t j, uint32_t agg,
                                              uint32_t epoch, uint32_t *err, int lane)
{
    const unsigned long long ep = (unsigned long long)epoch << 32;
    if (j == 0) {
        if (lane == 0) lb_store(&chain[0], ep | (2ull << 30) | agg);
        return 0;
    }
    if (lane == 0) lb_store(&chain[(size_t)j * stride], ep | (1ull << 30) | agg);
    uint32_t excl = 0;
    int qhi = (int)j - 1;
    uint32_t spins = 0;
    for (;;) {
        const int idx = qhi - lane;
        const bool inb = idx >= 0;
        const unsigned long long v = inb ? lb_load(&chain[(size_t)idx * stride]) : 0ull;
        const uint32_t flag = (uint32_t)(v >> 30) & 3u;
        const bool ok = inb && (uint32_t)(v >> 32) == epoch && flag != 0u;
        const unsigned long long m_incl = __ballot(ok && flag == 2u);
        const unsigned long long m_bad = __ballot(inb && !ok);
        const int first_incl = m_incl ? __ffsll((long long)m_incl) - 1 : 64;
        const int first_bad = m_bad ? __ffsll((long long)m_bad) - 1 : 64;
        const int upto = min(first_incl + 1, first_bad);
        uint32_t val = lane < upto ? ((uint32_t)v & 0x3FFFFFFFu) : 0u;
#pragma unroll
        for (int off = 32; off; off >>= 1) val += __shfl_xor(val, off);
        excl += val;
        if (first_incl < first_bad) break;
        qhi -= upto;
        if (upto == 0) {
            if (++spins > (1u << 22)) {       // bounded: never hang the GPU
                if (lane == 0) *err = 1u;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    if (lane == 0) lb_store(&chain[(size_t)j * stride], ep | (2ull << 30) | (excl + agg));
    return excl;
}

// Inclusive scan of n <= 64 per-lane counts (lanes >= n hold 0); returns the
// exclusive value for this lane, *agg = the total.
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t c, int n, int lane, uint32_t *agg)
{
    uint32_t inc = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t u = __shfl_up(inc, off);
        if (lane >= off) inc += u;
    }
    *agg = __shfl(inc, n - 1);
    return inc - c;
}

// diagnostic-only phase stamps (p.dbg bit 8): wave 0 lane 0 writes
// s_memrealtime (100 MHz) per phase into a buffer nothing else reads
#define STAMP(ph)                                                                          \
    do {                                                                                   \
        if ((p.dbg & 8u) && tid == 0) {                                                    \
            __builtin_amdgcn_sched_barrier(0);                                             \
            p.stamps[blockIdx.x * 8 + (ph)] = __builtin_amdgcn_s_memrealtime();            \
            __builtin_amdgcn_sched_barrier(0);                                             \
        }                                                                                  \
    } while (0)

// experiment builds may raise the occupancy target (KDEFS=-DCOPK_WAVES_PER_EU=8)
#ifndef COPK_WAVES_PER_EU
#define COPK_WAVES_PER_EU 1
#endif
template <int FW, int LPM, bool IMIX, int PPT>
__global__ __launch_bounds__(BLOCK, COPK_WAVES_PER_EU) void cop_pipeline(const CopKParams p)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    constexpr int TILE = BLOCK * PPT;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;

    // ---- LDS carve (offsets in u32 words, all multiples of 4) ----
    uint32_t *rt_top = lds;                                  // 256
    uint16_t *rt_leaf = (uint16_t *)(lds + 256);             // nleaf*256 u16
    uint32_t *fw_s = lds + p.lds_fw_off;
    uint32_t *fw_v = fw_s + p.fw_m;
    uint32_t *lp_s = lds + p.lds_lpm_off;
    uint32_t *lp_v = lp_s + p.lpm_m;
    uint32_t *misc = lds + p.lds_misc_off;
    volatile uint32_t *s_cnt = misc;                          // [PPT*WAVES]
    volatile uint32_t *s_tile = misc + 32;
    volatile uint32_t *s_pref = misc + 33;
    uint32_t *s_red = misc + 40;                              // [WAVES][8]

    STAMP(0);
    // ---- batch of this workgroup: static blockIdx ranges ----
    const uint32_t g = blockIdx.x;
    uint32_t b = 0;
    if (p.uniform_ntiles) {
        b = g / p.uniform_ntiles;      // equal-size batches: no dependent load
    } else {
#pragma unroll
        for (int q = 1; q < COPK_MAXB; q++) b += (q < (int)p.nb && p.tile_begin[q] <= g) ? 1u : 0u;
    }
    b = __builtin_amdgcn_readfirstlane(b);
    CopKBatch B;
    uint32_t look_off;
    if (p.ring) {
        const uint32_t slot = (p.rg.first + b) % p.rg.n_slots;   // count may exceed n_slots
        B.pkts = p.rg.pkts + (size_t)slot * p.rg.pkts_slot_bytes;
        B.offsets = p.rg.offsets ? p.rg.offsets + (size_t)slot * p.rg.offsets_slot_words : nullptr;
        B.results = (uint2 *)p.rg.results + (size_t)slot * p.rg.results_slot;
        B.fwd_idx = p.rg.fwd_idx ? p.rg.fwd_idx + (size_t)slot * p.rg.fwd_slot : nullptr;
        B.fwd_count = p.rg.fwd_count ? p.rg.fwd_count + (size_t)slot * (p.demux ? p.demux : 1u) : nullptr;
        B.n = p.rg.n;
        B.stride = p.rg.stride;
        B.data_off = p.rg.data_off;
        B.ntiles = p.uniform_ntiles;
        look_off = b * p.uniform_ntiles;
    } else {
        B = p.b[b];
        look_off = p.look_begin[b];
    }

    // ---- zero the lane's other ticket buffer for the next launch on this
    // lane (stream order puts that launch after this one completes) ----
    for (uint32_t line = g; line < p.zero_lines; line += gridDim.x)
        if (tid < 16) p.zero_tickets[line * 16 + tid] = 0ull;

    // ---- tile index inside the batch: this batch's ticket counter (or the
    // static order when no look-back runs: p.compact == 0) ----
    const bool dyn = p.compact != 0 && !(p.dbg & 2u);
    unsigned long long tk = 0;
    if (dyn && tid == 0) tk = atomicAdd(&p.tickets[b * 16], 1ull);

    // ---- stage tables into LDS by LDS-DMA while the ticket is in flight ----
    if (!(p.dbg & 4u)) {
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
        j = p.ring ? g - b * p.uniform_ntiles : g - p.tile_begin[b];
    }
    const uint32_t base = j * TILE;
    STAMP(1);

    // ---- packet header loads (all PPT packets, no branches). Lanes past
    // the end of the batch re-read the last packet and are masked out of
    // every store and count. ----
    uint32_t w3[PPT], w6[PPT], w7[PPT], w8[PPT];
    bool valid[PPT];
    const uint32_t last = B.n ? B.n - 1 : 0u;
    if (B.n) {
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            const uint32_t ic = min(base + k * BLOCK + tid, last);
            const uint8_t *pk;
            if (IMIX) pk = B.pkts + B.offsets[ic] + B.data_off;
            else pk = B.pkts + (size_t)ic * B.stride + B.data_off;
            w3[k] = *(const uint32_t *)(pk + 12);
            const uint2 v67 = *(const uint2 *)(pk + 24);
            w6[k] = v67.x;
            w7[k] = v67.y;
            w8[k] = *(const uint32_t *)(pk + 32);
        }
    } else {
#pragma unroll
        for (int k = 0; k < PPT; k++) w3[k] = w6[k] = w7[k] = w8[k] = 0;
    }
#pragma unroll
    for (int k = 0; k < PPT; k++) valid[k] = base + k * BLOCK + tid < B.n;
    if (!dyn) __syncthreads();   // LDS tables (the dynamic path synced above)

    // ---- pass 1, one step at a time as its packet data arrives: parse,
    // vport route (stage P), interval searches in LDS, and the tbl24 loads of
    // DIR-24-8 stages (issued, not waited for) ----
    uint32_t verdict[PPT], port[PPT], flags[PPT], rnh[PPT], fwe[PPT], lpe[PPT], src[PPT], dst[PPT];
    const bool stageP = (p.stages & COPK_STAGE_PARSE) != 0;
    const uint32_t fw_lv = p.fw_m ? (uint32_t)__builtin_ctz(p.fw_m) : 0u;
    const uint32_t lp_lv = p.lpm_m ? (uint32_t)__builtin_ctz(p.lpm_m) : 0u;
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        verdict[k] = COPK_FORWARD;
        port[k] = 0;
        flags[k] = 0;
        rnh[k] = 0;
        const uint32_t et = ((w3[k] & 0xFFu) << 8) | ((w3[k] >> 8) & 0xFFu);
        dst[k] = bswap32(__builtin_amdgcn_alignbit(w8[k], w7[k], 16));
        src[k] = bswap32(__builtin_amdgcn_alignbit(w7[k], w6[k], 16));
        if (stageP) {
            if (et != 0x0800u) {
                verdict[k] = COPK_DROP_PARSE;
                port[k] = 0xFFFFu;
            } else {
                const uint32_t idx = dst[k] & 0xFFFFu;
                const uint32_t top = rt_top[idx >> 8];
                port[k] = (top & 0x80000000u) ? (uint32_t)rt_leaf[((top & 0xFFFFu) << 8) | (idx & 0xFFu)]
                                              : (top & 0xFFFFu);
                if (port[k] == 0xFFFFu) verdict[k] = COPK_DROP_PARSE;
                else if (port[k] >= p.n_ports) verdict[k] = COPK_DROP_NO_PORT;
            }
        }
        if (FW == COPK_TBL_IVT) fwe[k] = fw_v[eyt_search(fw_s, fw_lv, src[k])];
        if (FW == COPK_TBL_DIR) fwe[k] = p.fw_tbl24[src[k] >> 8];
        if (LPM == COPK_TBL_IVT) lpe[k] = lp_v[eyt_search(lp_s, lp_lv, dst[k])];
        if (LPM == COPK_TBL_DIR) lpe[k] = p.lpm_tbl24[dst[k] >> 8];
    }
    bool reached[PPT];
#pragma unroll
    for (int k = 0; k < PPT; k++) reached[k] = verdict[k] == COPK_FORWARD;   // entered the coprocessor
    if (p.dbg & 8u) {
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < PPT; k++) x ^= verdict[k] ^ src[k];
        asm volatile("" ::"v"(x));
    }
    STAMP(2);

    // ---- pass 2: rte_lpm_lookup's tbl8 step for valid+extended entries ----
    if (FW == COPK_TBL_DIR) {
#pragma unroll
        for (int k = 0; k < PPT; k++)
            if ((fwe[k] & 0x03000000u) == 0x03000000u)
                fwe[k] = p.fw_tbl8[((size_t)(fwe[k] & 0x00FFFFFFu) << 8) | (src[k] & 0xFFu)];
    }
    if (LPM == COPK_TBL_DIR) {
#pragma unroll
        for (int k = 0; k < PPT; k++)
            if ((lpe[k] & 0x03000000u) == 0x03000000u)
                lpe[k] = p.lpm_tbl8[((size_t)(lpe[k] & 0x00FFFFFFu) << 8) | (dst[k] & 0xFFu)];
    }

    // ---- verdicts: stage FW (firewall.c:183-210), stage LPM ----
    uint32_t c_total = 0, c_notv4 = 0;
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        if (!reached[k]) continue;
        if (FW != COPK_TBL_OFF) {
            c_total += valid[k];
            if (((w3[k] >> 20) & 0xFu) != 4u) {
                verdict[k] = COPK_DROP_NOT_IPV4;
                c_notv4 += valid[k];
            } else {
                // rule-id image: bit 24 hit, bit 26 = the matching rule's
                // action is non-zero (switch(rule) at firewall.c:201-210)
                flags[k] |= (fwe[k] >> 24) & 1u ? COPK_FLAG_FW_HIT : 0u;
                verdict[k] = (fwe[k] >> 26) & 1u ? COPK_DROP_FW : COPK_FORWARD;
            }
        }
        if (LPM != COPK_TBL_OFF) {
            flags[k] |= (lpe[k] >> 24) & 1u ? COPK_FLAG_ROUTE_HIT : 0u;
            rnh[k] = lpe[k] & 0x00FFFFFFu;
        }
    }
    if (FW != COPK_TBL_OFF && p.rule_hits) {
        // per-rule hit counters: one relaxed device-scope u64 add per hit
        // (no return value: fire-and-forget atomics at the L2/fabric)
#pragma unroll
        for (int k = 0; k < PPT; k++)
            if (valid[k] && (flags[k] & COPK_FLAG_FW_HIT))
                __hip_atomic_fetch_add(&p.rule_hits[fwe[k] & 0x00FFFFFFu], 1ull, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
    }
    if (p.dbg & 8u) {
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < PPT; k++) x ^= verdict[k] ^ rnh[k];
        asm volatile("" ::"v"(x));
    }
    STAMP(3);
    // ---- result records (8 B per packet, coalesced dwordx2) + counts ----
    uint32_t c_fwd = 0, c_dropfw = 0, c_parse = 0, c_noport = 0, c_rhit = 0, c_rx = 0;
    bool fwd[PPT];
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        fwd[k] = valid[k] && verdict[k] == COPK_FORWARD;
        if (valid[k]) {
            // non-temporal: results are read by the host / next stage, not by
            // this kernel; streaming them out avoids a dirty-L2 write-back
            // at the kernel boundary
            typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
            u32x2 rec;
            rec.x = verdict[k] | (flags[k] << 8) | (port[k] << 16);
            rec.y = rnh[k];
            __builtin_nontemporal_store(rec, &((u32x2 *)B.results)[base + k * BLOCK + tid]);
            c_rx++;
            c_fwd += verdict[k] == COPK_FORWARD;
            c_dropfw += verdict[k] == COPK_DROP_FW;
            c_parse += verdict[k] == COPK_DROP_PARSE;
            c_noport += verdict[k] == COPK_DROP_NO_PORT;
            c_rhit += flags[k] & COPK_FLAG_ROUTE_HIT;
        }
    }

    STAMP(4);
    if (p.compact && !p.demux) {
        // ---- ordered compaction: one forward list per batch ----
        unsigned long long bal[PPT];
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            bal[k] = __ballot(fwd[k]);
            if (lane == 0) s_cnt[k * WAVES + wave] = (uint32_t)__popcll(bal[k]);
        }
        __syncthreads();
        if (wave == 0) {
            // tile-local exclusive scan over the (step, wave) counts
            constexpr int NQ = PPT * WAVES;
            uint32_t agg;
            const uint32_t ex = wave_excl_scan(lane < NQ ? s_cnt[lane] : 0u, NQ, lane, &agg);
            if (lane < NQ) s_cnt[lane] = ex;
            // dbg bit 32 (timing-only ablation): no look-back wait, wrong offsets
            const uint32_t excl =
                (p.dbg & 32u) ? j * 1024u : look_back(p.look + look_off, 1u, j, agg, p.epoch, p.err, lane);
            if (lane == 0) {
                *s_pref = excl;
                if (B.fwd_count && j == B.ntiles - 1) *B.fwd_count = excl + agg;
            }
        }
        __syncthreads();
        STAMP(5);
        if (B.fwd_idx) {
            const uint32_t pref = *s_pref;
#pragma unroll
            for (int k = 0; k < PPT; k++) {
                if (fwd[k]) {
                    const uint32_t r = __builtin_amdgcn_mbcnt_hi(
                        (uint32_t)(bal[k] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal[k], 0u));
                    __builtin_nontemporal_store(base + k * BLOCK + tid,
                                                &B.fwd_idx[pref + s_cnt[k * WAVES + wave] + r]);
                }
            }
        }
    } else if (p.compact) {
        // ---- demux: one ordered forward list per vport (the tx_q order of
        // each port's coprocessor, switch.c:306-327 + 464-470). Port q's
        // list is at fwd_idx + q*n, its length at fwd_count[q]. One
        // look-back chain per port, the chains spread over the waves. ----
        constexpr int NQ = PPT * WAVES;
        const uint32_t K = p.demux;
        volatile uint32_t *s_dq = misc + COPK_LDS_MISC_WORDS;        // [K][NQ]
        volatile uint32_t *s_dpref = s_dq + COPK_MAX_DEMUX_PORTS * NQ; // [K]
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            for (uint32_t q = 0; q < K; q++) {
                const unsigned long long b = __ballot(fwd[k] && port[k] == q);
                if (lane == 0) s_dq[q * NQ + k * WAVES + wave] = (uint32_t)__popcll(b);
            }
        }
        __syncthreads();
        for (uint32_t q = (uint32_t)wave; q < K; q += WAVES) {
            uint32_t agg;
            const uint32_t ex = wave_excl_scan(lane < NQ ? s_dq[q * NQ + lane] : 0u, NQ, lane, &agg);
            if (lane < NQ) s_dq[q * NQ + lane] = ex;
            const uint32_t excl = look_back(p.look + (size_t)look_off * K + q, K, j, agg, p.epoch, p.err, lane);
            if (lane == 0) {
                s_dpref[q] = excl;
                if (B.fwd_count && j == B.ntiles - 1) B.fwd_count[q] = excl + agg;
            }
        }
        __syncthreads();
        STAMP(5);
        if (B.fwd_idx) {
#pragma unroll
            for (int k = 0; k < PPT; k++) {
                uint32_t r = 0;
                for (uint32_t q = 0; q < K; q++) {
                    const bool mine = fwd[k] && port[k] == q;
                    const unsigned long long b = __ballot(mine);
                    if (mine)
                        r = __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
                }
                if (fwd[k]) {
                    const uint32_t q = port[k];
                    __builtin_nontemporal_store(
                        base + k * BLOCK + tid,
                        &B.fwd_idx[(size_t)q * B.n + s_dpref[q] + s_dq[q * NQ + k * WAVES + wave] + r]);
                }
            }
        }
    }

    // ---- counters: wave reduce -> LDS -> one atomic per counter per
    // workgroup, into one of COPK_COUNTER_SHARDS shards (a 128-byte line
    // each) so no single word serialises thousands of atomics ----
    uint32_t c[8] = {c_total, c_notv4, c_fwd, c_dropfw, c_parse, c_noport, c_rhit, c_rx};
#pragma unroll
    for (int q = 0; q < 8; q++) {
        uint32_t v = c[q];
#pragma unroll
        for (int off = 32; off; off >>= 1) v += __shfl_xor(v, off);
        c[q] = v;
    }
    if (lane == 0) {
#pragma unroll
        for (int q = 0; q < 8; q++) s_red[wave * 8 + q] = c[q];
    }
    __syncthreads();
    if (tid < 9) {
        uint32_t r[8];
#pragma unroll
        for (int q = 0; q < 8; q++) {
            uint32_t v = 0;
#pragma unroll
            for (int w = 0; w < WAVES; w++) v += s_red[w * 8 + q];
            r[q] = v;
        }
        // cop_counters order: drop, accept, not_ipv4, total, parse_err, no_port, forward, route_hit, rx
        uint32_t v;
        switch (tid) {
        case 0: v = r[3] + r[1]; break;
        case 1: v = r[0] - r[1] - r[3]; break;
        case 2: v = r[1]; break;
        case 3: v = r[0]; break;
        case 4: v = r[4]; break;
        case 5: v = r[5]; break;
        case 6: v = r[2]; break;
        case 7: v = r[6]; break;
        default: v = r[7]; break;
        }
        if (v && !(p.dbg & 1u))
            atomicAdd(&p.counters[(blockIdx.x % COPK_COUNTER_SHARDS) * 16 + tid], (unsigned long long)v);
    }
    if (p.port_stats) {
        // per-port coprocessor_stats (switch.h:33-38): rx = packets routed to
        // the port's NF (enqueue_nf_rx), tx = packets it forwarded
        volatile uint32_t *s_ps = misc + COPK_LDS_MISC_WORDS + COPK_MAX_DEMUX_PORTS * PPT * WAVES + 8;
        const uint32_t K = p.port_stats;
        for (uint32_t q = 0; q < K; q++) {
            uint32_t rx = 0, tx = 0;
#pragma unroll
            for (int k = 0; k < PPT; k++) {
                rx += (uint32_t)__popcll(__ballot(valid[k] && port[k] == q));
                tx += (uint32_t)__popcll(__ballot(fwd[k] && port[k] == q));
            }
            if (lane == 0) {
                s_ps[wave * 16 + 2 * q] = rx;
                s_ps[wave * 16 + 2 * q + 1] = tx;
            }
        }
        __syncthreads();
        if (tid < 2 * K) {
            uint32_t v = 0;
#pragma unroll
            for (int w = 0; w < WAVES; w++) v += s_ps[w * 16 + tid];
            if (v) atomicAdd(&p.port_ctr[(blockIdx.x % COPK_COUNTER_SHARDS) * COPK_PORT_WORDS + tid],
                             (unsigned long long)v);
        }
    }
    STAMP(6);
}

template <int FW, int LPM, bool IMIX, int PPT>
hipError_t launch_one(const CopKParams &p, uint32_t grid, uint32_t lds_bytes, hipStream_t s)
{
    hipLaunchKernelGGL((cop_pipeline<FW, LPM, IMIX, PPT>), dim3(grid), dim3(BLOCK), lds_bytes, s, p);
    return hipGetLastError();
}

template <int FW, int LPM, bool IMIX>
hipError_t launch_ppt(const CopKParams &p, int ppt, uint32_t grid, uint32_t lds, hipStream_t s)
{
    if (ppt == 8) return launch_one<FW, LPM, IMIX, 8>(p, grid, lds, s);
    if (ppt == 4) return launch_one<FW, LPM, IMIX, 4>(p, grid, lds, s);
    return launch_one<FW, LPM, IMIX, 1>(p, grid, lds, s);
}

template <int FW, int LPM>
hipError_t launch_imix(const CopKParams &p, bool imix, int ppt, uint32_t grid, uint32_t lds, hipStream_t s)
{
    if (imix) return launch_ppt<FW, LPM, true>(p, ppt, grid, lds, s);
    return launch_ppt<FW, LPM, false>(p, ppt, grid, lds, s);
}

template <int FW>
hipError_t launch_lpm(const CopKParams &p, int lpm, bool imix, int ppt, uint32_t grid, uint32_t lds,
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
