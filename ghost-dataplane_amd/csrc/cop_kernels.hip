// cop_kernels.hip — the coprocessor NF pipeline as one gfx950 kernel.
//
// One lane handles one packet per step. Per packet the kernel restates, in
// this order (SURVEY.md §8a "bit-exact per-packet contract"):
//   stage P   get_next_hop            switch.c:93-136  (+ fast-path drop
//             switch.c:406-410, enqueue_nf_rx port bound switch.c:316-319)
//   stage FW  fw_packet_handler       firewall.c:170-213, lookup =
//             rte_lpm_lookup(lpm_tbl, ntohl(src))     firewall.c:194
//   stage LPM route rte_lpm semantics on ntohl(dst)   (north-star extension)
//   compaction: indices of FORWARD packets in arrival order, the order
//             coprocessor() hands them to enqueue_nf_tx (switch.c:464-470).
//
// Data layout (HBM): packets at 16-byte aligned starts (64-byte slots or
// an IMIX slab + u32 offsets); tables: vport routing table as a two-level
// image (256-entry top + 256-entry u16 leaves), LPM tables either as a
// flattened interval array (LDS, binary search) or as a DPDK-layout
// DIR-24-8 image (tbl24 64 MiB + tbl8 groups, HBM/Infinity-Cache). Small
// tables are copied into LDS once per workgroup; the workgroup then loops
// over 256*PPT-packet tiles handed out by a device ticket counter.
//
// Ordered compaction across workgroups: wave64 ballot + mbcnt inside a
// tile, an LDS scan across (step, wave), then decoupled look-back over the
// tiles of the batch. Tiles are numbered by an atomic ticket, so every
// predecessor of a tile is already running when the tile waits on it.
// Look-back words are 8-byte {epoch, flag, value} granules written and
// polled with agent-scope relaxed atomics (sc1): the data is the flag.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cop_kernels.h"

namespace {

constexpr int BLOCK = COPK_BLOCK;
constexpr int WAVES = BLOCK / 64;

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ uint32_t ivt_lookup(const uint32_t *starts, const uint32_t *vals,
                                               uint32_t m, uint32_t ip)
{
    // largest k with starts[k] <= ip; starts[0] == 0, m a power of two,
    // padding entries repeat the last value.
    uint32_t k = 0;
    for (uint32_t step = m >> 1; step; step >>= 1) {
        uint32_t c = starts[k + step];
        k = (c <= ip) ? k + step : k;
    }
    return vals[k];
}

__device__ __forceinline__ uint32_t dir_lookup(const uint32_t *__restrict__ tbl24,
                                               const uint32_t *__restrict__ tbl8, uint32_t ip)
{
    // rte_lpm_lookup (DPDK 17.11 v1604): one tbl24 load, a tbl8 load when
    // the entry is valid and extended.
    uint32_t e = tbl24[ip >> 8];
    if ((e & 0x03000000u) == 0x03000000u)
        e = tbl8[((size_t)(e & 0x00FFFFFFu) << 8) | (ip & 0xFFu)];
    return e;
}

__device__ __forceinline__ void lb_store(unsigned long long *p, unsigned long long v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ unsigned long long lb_load(unsigned long long *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int FW, int LPM, bool IMIX, int PPT>
__global__ __launch_bounds__(BLOCK) void cop_pipeline(const CopKParams p)
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
    uint32_t *misc = lds + p.lds_misc_off;                    // cnt[PPT*WAVES], next, prefix
    volatile uint32_t *s_cnt = misc;
    volatile uint32_t *s_next = misc + PPT * WAVES;
    volatile uint32_t *s_pref = misc + PPT * WAVES + 1;

    // ---- first ticket early: its latency hides under the table copy ----
    unsigned long long my_next = 0;
    if (tid == 0) my_next = atomicAdd(p.ticket, 1ull);

    // ---- stage tables into LDS ----
    {
        const uint4 *src = (const uint4 *)p.rt_top;
        uint4 *dst = (uint4 *)rt_top;
        for (int i = tid; i < 64; i += BLOCK) dst[i] = src[i];
        const uint4 *ls = (const uint4 *)p.rt_leaf;
        uint4 *ld = (uint4 *)rt_leaf;
        const int nq = (int)(p.rt_nleaf * 32u);
        for (int i = tid; i < nq; i += BLOCK) ld[i] = ls[i];
        if (FW == COPK_TBL_IVT) {
            const uint4 *a = (const uint4 *)p.fw_starts, *b = (const uint4 *)p.fw_vals;
            uint4 *da = (uint4 *)fw_s, *db = (uint4 *)fw_v;
            const int n4 = (int)(p.fw_m >> 2);
            for (int i = tid; i < n4; i += BLOCK) {
                da[i] = a[i];
                db[i] = b[i];
            }
            if (p.fw_m < 4 && tid < (int)p.fw_m) {
                fw_s[tid] = p.fw_starts[tid];
                fw_v[tid] = p.fw_vals[tid];
            }
        }
        if (LPM == COPK_TBL_IVT) {
            const uint4 *a = (const uint4 *)p.lpm_starts, *b = (const uint4 *)p.lpm_vals;
            uint4 *da = (uint4 *)lp_s, *db = (uint4 *)lp_v;
            const int n4 = (int)(p.lpm_m >> 2);
            for (int i = tid; i < n4; i += BLOCK) {
                da[i] = a[i];
                db[i] = b[i];
            }
            if (p.lpm_m < 4 && tid < (int)p.lpm_m) {
                lp_s[tid] = p.lpm_starts[tid];
                lp_v[tid] = p.lpm_vals[tid];
            }
        }
    }
    if (tid == 0) *s_next = (uint32_t)min(my_next - p.ticket_base, (unsigned long long)0xFFFFFFFFu);

    // per-thread counters, reduced once per workgroup at exit
    uint32_t c_total = 0, c_notv4 = 0, c_fwd = 0, c_dropfw = 0, c_parse = 0, c_noport = 0,
             c_rhit = 0, c_rx = 0;

    const bool stageP = (p.stages & COPK_STAGE_PARSE) != 0;

    for (;;) {
        __syncthreads();                       // tables + s_next visible
        const uint32_t t = *s_next;
        if (t >= p.ntiles) break;
        if (tid == 0) my_next = atomicAdd(p.ticket, 1ull);   // prefetch next tile

        // locate batch (wave-uniform scan over <= COPK_MAXB descriptors)
        uint32_t b = 0;
        while (b + 1 < p.nb && p.b[b + 1].tile_begin <= t) b++;
        const CopKBatch &B = p.b[b];
        const uint32_t j = t - B.tile_begin;   // tile index inside the batch
        const uint32_t base = j * TILE;

        uint32_t res0[PPT], res1[PPT];
        bool fwd[PPT];

        // ---- loads first (all PPT packets), then compute ----
        uint32_t w3[PPT], w6[PPT], w7[PPT], w8[PPT];
        bool valid[PPT];
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            const uint32_t i = base + k * BLOCK + tid;
            valid[k] = i < B.n;
            w3[k] = w6[k] = w7[k] = w8[k] = 0;
            if (valid[k]) {
                const uint8_t *pk;
                if (IMIX) pk = B.pkts + B.offsets[i] + B.data_off;
                else pk = B.pkts + (size_t)i * B.stride + B.data_off;
                w3[k] = *(const uint32_t *)(pk + 12);
                const uint2 v67 = *(const uint2 *)(pk + 24);
                w6[k] = v67.x;
                w7[k] = v67.y;
                w8[k] = *(const uint32_t *)(pk + 32);
            }
        }
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            uint32_t verdict = COPK_FORWARD, port = 0, flags = 0, rnh = 0;
            const uint32_t et = ((w3[k] & 0xFFu) << 8) | ((w3[k] >> 8) & 0xFFu);
            const uint32_t dst = bswap32(__builtin_amdgcn_alignbit(w8[k], w7[k], 16));
            const uint32_t src = bswap32(__builtin_amdgcn_alignbit(w7[k], w6[k], 16));
            if (stageP) {
                if (et != 0x0800u) {
                    verdict = COPK_DROP_PARSE;
                    port = 0xFFFFu;
                } else {
                    const uint32_t idx = dst & 0xFFFFu;
                    const uint32_t top = rt_top[idx >> 8];
                    port = (top & 0x80000000u) ? (uint32_t)rt_leaf[((top & 0xFFFFu) << 8) | (idx & 0xFFu)]
                                               : (top & 0xFFFFu);
                    if (port == 0xFFFFu) verdict = COPK_DROP_PARSE;
                    else if (port >= p.n_ports) verdict = COPK_DROP_NO_PORT;
                }
            }
            const bool reached = verdict == COPK_FORWARD;   // entered the coprocessor
            if (FW != COPK_TBL_OFF && reached) {
                c_total += valid[k];
                const uint32_t ver = (w3[k] >> 20) & 0xFu;
                if (ver != 4u) {
                    verdict = COPK_DROP_NOT_IPV4;
                    c_notv4 += valid[k];
                } else {
                    const uint32_t e = (FW == COPK_TBL_IVT) ? ivt_lookup(fw_s, fw_v, p.fw_m, src)
                                                            : dir_lookup(p.fw_tbl24, p.fw_tbl8, src);
                    flags |= (e >> 24) & 1u ? COPK_FLAG_FW_HIT : 0u;
                    verdict = (e & 0x00FFFFFFu) ? COPK_DROP_FW : COPK_FORWARD;
                }
            }
            if (LPM != COPK_TBL_OFF && reached) {
                const uint32_t e = (LPM == COPK_TBL_IVT) ? ivt_lookup(lp_s, lp_v, p.lpm_m, dst)
                                                         : dir_lookup(p.lpm_tbl24, p.lpm_tbl8, dst);
                flags |= (e >> 24) & 1u ? COPK_FLAG_ROUTE_HIT : 0u;
                rnh = e & 0x00FFFFFFu;
            }
            res0[k] = verdict | (flags << 8) | (port << 16);
            res1[k] = rnh;
            fwd[k] = valid[k] && verdict == COPK_FORWARD;
            if (valid[k]) {
                c_rx++;
                c_fwd += verdict == COPK_FORWARD;
                c_dropfw += verdict == COPK_DROP_FW;
                c_parse += verdict == COPK_DROP_PARSE;
                c_noport += verdict == COPK_DROP_NO_PORT;
                c_rhit += flags & COPK_FLAG_ROUTE_HIT;
            }
        }
        // ---- result records (8 B per packet, coalesced dwordx2) ----
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            const uint32_t i = base + k * BLOCK + tid;
            if (valid[k]) ((uint2 *)B.results)[i] = make_uint2(res0[k], res1[k]);
        }

        if (p.compact) {
            // ---- ordered compaction ----
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
                uint32_t c = lane < NQ ? s_cnt[lane] : 0u;
                uint32_t inc = c;
#pragma unroll
                for (int off = 1; off < NQ; off <<= 1) {
                    const uint32_t u = __shfl_up(inc, off);
                    if (lane >= off) inc += u;
                }
                const uint32_t agg = __shfl(inc, NQ - 1);
                if (lane < NQ) s_cnt[lane] = inc - c;
                const unsigned long long ep = (unsigned long long)p.epoch << 32;
                uint32_t excl = 0;
                if (j == 0) {
                    if (lane == 0) lb_store(&p.look[t], ep | (2ull << 30) | agg);
                } else {
                    if (lane == 0) lb_store(&p.look[t], ep | (1ull << 30) | agg);
                    // decoupled look-back, 64 predecessors per round: lane l
                    // reads tile qhi-l; consume the ready prefix up to and
                    // including the nearest inclusive prefix.
                    int qhi = (int)t - 1;
                    const int qlo = (int)B.tile_begin;
                    uint32_t spins = 0;
                    for (;;) {
                        const int idx = qhi - lane;
                        const bool inb = idx >= qlo;
                        const unsigned long long v = inb ? lb_load(&p.look[idx]) : 0ull;
                        const uint32_t flag = (uint32_t)(v >> 30) & 3u;
                        const bool ok = inb && (uint32_t)(v >> 32) == p.epoch && flag != 0u;
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
                                if (lane == 0) *p.err = 1u;   // host-mapped error word
                                break;
                            }
                            __builtin_amdgcn_s_sleep(1);
                        }
                    }
                    if (lane == 0) lb_store(&p.look[t], ep | (2ull << 30) | (excl + agg));
                }
                if (lane == 0) {
                    *s_pref = excl;
                    if (B.fwd_count && j == B.ntiles - 1) *B.fwd_count = excl + agg;
                }
            }
            __syncthreads();
            if (B.fwd_idx) {
                const uint32_t pref = *s_pref;
#pragma unroll
                for (int k = 0; k < PPT; k++) {
                    if (fwd[k]) {
                        const uint32_t r = __builtin_amdgcn_mbcnt_hi(
                            (uint32_t)(bal[k] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal[k], 0u));
                        B.fwd_idx[pref + s_cnt[k * WAVES + wave] + r] = base + k * BLOCK + tid;
                    }
                }
            }
        }
        // every wave has read t (compaction has barriers; else take one) before
        // thread 0 publishes the prefetched ticket; the loop-head barrier orders it
        if (!p.compact) __syncthreads();
        if (tid == 0)
            *s_next = (uint32_t)min(my_next - p.ticket_base, (unsigned long long)0xFFFFFFFFu);
    }

    // ---- counters: wave reduce, then one atomic per counter per wave ----
    uint32_t c[8] = {c_total, c_notv4, c_fwd, c_dropfw, c_parse, c_noport, c_rhit, c_rx};
#pragma unroll
    for (int q = 0; q < 8; q++) {
        uint32_t v = c[q];
        for (int off = 32; off; off >>= 1) v += __shfl_xor(v, off);
        c[q] = v;
    }
    if (lane == 0) {
        // cop_counters order: drop, accept, not_ipv4, total, parse_err, no_port, forward, route_hit, rx
        const uint32_t accept = c[0] - c[1] - c[3];
        if (c[3] + c[1]) atomicAdd(&p.counters[0], (unsigned long long)(c[3] + c[1]));
        if (accept) atomicAdd(&p.counters[1], (unsigned long long)accept);
        if (c[1]) atomicAdd(&p.counters[2], (unsigned long long)c[1]);
        if (c[0]) atomicAdd(&p.counters[3], (unsigned long long)c[0]);
        if (c[4]) atomicAdd(&p.counters[4], (unsigned long long)c[4]);
        if (c[5]) atomicAdd(&p.counters[5], (unsigned long long)c[5]);
        if (c[2]) atomicAdd(&p.counters[6], (unsigned long long)c[2]);
        if (c[6]) atomicAdd(&p.counters[7], (unsigned long long)c[6]);
        if (c[7]) atomicAdd(&p.counters[8], (unsigned long long)c[7]);
    }
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
