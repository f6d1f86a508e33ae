// cop_device.h — device-side pieces of the pipeline kernels
// (cop_kernels.hip). Internal.
//
// Per packet, the classification restates (SURVEY.md §8a contract):
//   stage P   get_next_hop            switch.c:93-136  (+ fast-path drop
//             switch.c:406-410, enqueue_nf_rx port bound switch.c:316-319)
//   stage FW  fw_packet_handler       firewall.c:170-213, lookup =
//             rte_lpm_lookup(lpm_tbl, ntohl(src))     firewall.c:194
//   stage LPM route rte_lpm semantics on ntohl(dst)   (north-star extension)
// and the ordered compaction keeps FORWARD packets in arrival order, the
// order coprocessor() hands them to enqueue_nf_tx (switch.c:464-470).
#ifndef COP_DEVICE_H
#define COP_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cop_kernels.h"

namespace copd {

constexpr int BLOCK = COPK_BLOCK;
constexpr int WAVES = BLOCK / 64;

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// the same vectors at 4-byte alignment (packet fields at offsets 12 and 28)
typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x2a __attribute__((ext_vector_type(2), aligned(4)));

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ void lb_store(unsigned long long *p, unsigned long long v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ unsigned long long lb_load(unsigned long long *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Output stores. The one-shot kernel stores non-temporally (the lines sit
// in the XCD's L2 until the kernel-end write-back); the poll-mode kernel
// has no kernel end per batch, so WT (write-through, sc1) stores make a
// batch's records and forward list visible to the host and to every XCD
// once the storing waves have drained (vmcnt(0)) and the batch is
// signalled (MI355X_MICROARCH.md, Valid forms: sc1 stores + drain + flag).
template <bool WT>
__device__ __forceinline__ void st_u32x2(u32x2 v, u32x2 *p)
{
    if (WT)
        __hip_atomic_store((unsigned long long *)p, ((unsigned long long)v.y << 32) | v.x, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    else
        __builtin_nontemporal_store(v, p);
}

template <bool WT>
__device__ __forceinline__ void st_u32(uint32_t v, uint32_t *p)
{
    if (WT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else __builtin_nontemporal_store(v, p);
}

// 16 bytes at list word w of `base`: a buffer store with sc1 (aux 16) when WT
template <bool WT>
__device__ __forceinline__ void st_u32x4(u32x4 v, uint32_t *base, long w)
{
    if (WT) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7FFFFFFF, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)(w * 4), 0, 16);
    } else {
        __builtin_nontemporal_store(v, (u32x4 *)(base + w));
    }
}

// Workgroup barrier that orders LDS only. __syncthreads() is a workgroup
// fence plus s_barrier, and the fence waits for every outstanding global load
// and store of the wave (vmcnt(0)): prefetched tiles and in-flight record
// stores would drain at every barrier. Cross-workgroup data (look-back
// granules, counters) is ordered by agent-scope atomics, not by barriers.
// LDS-DMA (global_load_lds) completion is counted by vmcnt: wait for staged
// tables with __syncthreads().
// (A fence restricted to LDS, __builtin_amdgcn_fence(..., "workgroup",
// "local"), does this in small kernels but loses its address-space tag in
// the pipeline kernels and falls back to vmcnt(0).) The memory clobber
// keeps the compiler from moving memory accesses across the barrier;
// lgkmcnt(0) completes this wave's LDS writes before it arrives.
__device__ __forceinline__ void lds_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Several LDS-DMA copies in ONE loop over their 1 KiB pieces (piece q of
// the concatenation: its segment picked by scalar compares). The compiler
// puts an s_waitcnt vmcnt(0) in front of every separate LDS-DMA loop (the
// DMA writes LDS that an earlier one may have written), which serialised
// the table staging into one memory round trip per table: 2-3 us at the
// start of every workgroup. One loop has one wait, before any load.
struct StageSeg {
    const void *g;      // global source (16-byte aligned)
    uint32_t *dst;      // LDS destination
    uint32_t n16;       // 16-byte chunks (0: unused)
};

// up to six segments, passed by value and selected by compares (an indexed
// array of them would live in scratch memory, whose loads also wait on vmcnt)
__device__ __forceinline__ void lds_stage_all(StageSeg s0, StageSeg s1, StageSeg s2, StageSeg s3, StageSeg s4,
                                              StageSeg s5, int lane, int wave)
{
    const uint32_t f1 = (s0.n16 + 63u) >> 6;
    const uint32_t f2 = f1 + ((s1.n16 + 63u) >> 6);
    const uint32_t f3 = f2 + ((s2.n16 + 63u) >> 6);
    const uint32_t f4 = f3 + ((s3.n16 + 63u) >> 6);
    const uint32_t f5 = f4 + ((s4.n16 + 63u) >> 6);
    const uint32_t total = f5 + ((s5.n16 + 63u) >> 6);
    for (uint32_t q = (uint32_t)wave; q < total; q += WAVES) {
        // field by field (selecting whole structs by reference puts them in scratch)
        const bool b1 = q >= f1, b2 = q >= f2, b3 = q >= f3, b4 = q >= f4, b5 = q >= f5;
        const void *g = b5 ? s5.g : b4 ? s4.g : b3 ? s3.g : b2 ? s2.g : b1 ? s1.g : s0.g;
        uint32_t *dst = b5 ? s5.dst : b4 ? s4.dst : b3 ? s3.dst : b2 ? s2.dst : b1 ? s1.dst : s0.dst;
        const uint32_t n16 = b5 ? s5.n16 : b4 ? s4.n16 : b3 ? s3.n16 : b2 ? s2.n16 : b1 ? s1.n16 : s0.n16;
        const uint32_t c = q - (b5 ? f5 : b4 ? f4 : b3 ? f3 : b2 ? f2 : b1 ? f1 : 0u);
        const uint32_t i = c * 64u + (uint32_t)lane;
        if (i < n16)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)((const uint4 *)g + i),
                                             (__attribute__((address_space(3))) void *)(dst + c * 256u), 16, 0, 0);
    }
}

__device__ __forceinline__ void lds_stage(uint32_t *lds_dst, const void *gsrc, uint32_t n16, int lane, int wave)
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

// Interval search in LDS over the bucketed form (cop_runtime.cpp
// upload_lpm): sorted starts S[0..M), then idx[0..2^ib] (u16), idx[b] = the
// last k with S[k] <= b << (32 - ib). The answer for ip in bucket b lies in
// [idx[b], idx[b+1]]; binary lifting over lv levels (2^lv > the widest
// bucket) finds the last k in it with S[k] <= ip, clamped to the bucket's
// end (correct since S is sorted). 2 + lv dependent LDS reads.
__device__ __forceinline__ uint32_t ivt_search(const uint32_t *S, uint32_t m, uint32_t ib, uint32_t lv, uint32_t ip)
{
    const uint16_t *idx = (const uint16_t *)(S + m);
    const uint32_t b = ip >> (32u - ib);
    uint32_t k = idx[b];
    const uint32_t hi = idx[b + 1];
    for (uint32_t step = (1u << lv) >> 1; step; step >>= 1) {
        const uint32_t c = min(k + step, hi);
        if (S[c] <= ip) k = c;
    }
    return k;
}

// ivt_search's interval value V[k] directly: the last lift level reads the
// candidate's start and both candidates' values together, so the value
// costs no dependent LDS read of its own (1 + lv reads in the chain, not
// 2 + lv). The driver's command 53,975 / 53,512 / 53,514 against 53,359 /
// 51,514 / 52,191 Mpkt/s, three alternating pairs on one box
// (profiles/r05/check21/); COPK_IVT_VALUE=0 reads the value after the
// search.
#ifndef COPK_IVT_VALUE
#define COPK_IVT_VALUE 1
#endif
__device__ __forceinline__ uint32_t ivt_value(const uint32_t *S, const uint32_t *V, uint32_t m, uint32_t ib, uint32_t lv,
                                              uint32_t ip)
{
    if (!COPK_IVT_VALUE || lv == 0) return V[ivt_search(S, m, ib, lv, ip)];
    const uint16_t *idx = (const uint16_t *)(S + m);
    const uint32_t b = ip >> (32u - ib);
    uint32_t k = idx[b];
    const uint32_t hi = idx[b + 1];
    for (uint32_t step = (1u << lv) >> 1; step > 1; step >>= 1) {
        const uint32_t c = min(k + step, hi);
        if (S[c] <= ip) k = c;
    }
    const uint32_t c = min(k + 1, hi);
    const uint32_t sc = S[c], vk = V[k], vc = V[c];
    return sc <= ip ? vc : vk;
}

// Decoupled look-back over one chain of tile granules (tile t at
// chain[t * stride]): publish this tile's aggregate, read up to 256
// predecessors per round (four loads per lane: lane l reads tiles qhi-l,
// qhi-64-l, ...; one round trip resolves a long chain whose tiles have all
// published), consume the ready prefix up to and including the nearest
// inclusive prefix, then publish the inclusive value. Granules are
// {epoch:32, flag:2 (1 aggregate, 2 inclusive), value:30}; a stale epoch
// counts as not ready. Spins are bounded and report through the host-mapped
// error word. Whole wave; returns the exclusive prefix.
// exitw (poll-mode kernel: its exit word, else null): a wait that sees the
// kernel abort (COPK_PMD_ABORT) gives up without publishing, since the
// predecessor it waits on may belong to a worker that has left, and returns
// LB_GAVE_UP; so does a poll-mode wait that times out. A tile that gave up
// writes no list and is not counted for its slot: the batch never completes
// (the host sees the abort). An idle or stop exit serves every batch it has
// let any worker start (cop_pmd.hip, the gate), so a wait there always ends.
constexpr int LB_GROUPS = 4;
constexpr uint32_t LB_GAVE_UP = 0xFFFFFFFFu;
__device__ __forceinline__ uint32_t look_back(unsigned long long *chain, uint32_t stride, uint32_t j, uint32_t agg,
                                              uint32_t epoch, uint32_t *err, int lane, const uint32_t *exitw = nullptr,
                                              uint32_t spin_log2 = 22)
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
        unsigned long long v[LB_GROUPS];
#pragma unroll
        for (int r = 0; r < LB_GROUPS; r++) {
            const int idx = qhi - r * 64 - lane;
            v[r] = idx >= 0 ? lb_load(&chain[(size_t)idx * stride]) : 0ull;
        }
        int consumed = 0;
        bool done = false;
#pragma unroll
        for (int r = 0; r < LB_GROUPS; r++) {
            const bool inb = qhi - r * 64 - lane >= 0;
            const uint32_t flag = (uint32_t)(v[r] >> 30) & 3u;
            const bool ok = inb && (uint32_t)(v[r] >> 32) == epoch && flag != 0u;
            const unsigned long long m_incl = __ballot(ok && flag == 2u);
            const unsigned long long m_bad = __ballot(inb && !ok);
            const int first_incl = m_incl ? __ffsll((long long)m_incl) - 1 : 64;
            const int first_bad = m_bad ? __ffsll((long long)m_bad) - 1 : 64;
            const int upto = min(first_incl + 1, first_bad);
            uint32_t val = lane < upto ? ((uint32_t)v[r] & 0x3FFFFFFFu) : 0u;
#pragma unroll
            for (int off = 32; off; off >>= 1) val += __shfl_xor(val, off);
            excl += val;
            consumed += upto;
            if (first_incl < first_bad) {
                done = true;
                break;
            }
            if (upto < 64) break;   // a predecessor not ready yet: re-read from it
        }
        if (done) break;
        qhi -= consumed;
        if (consumed == 0) {
            if (++spins > (1u << spin_log2)) {   // bounded: never hang the GPU
                if (lane == 0) *err = 1u;
                if (exitw) return LB_GAVE_UP; // poll mode: publish nothing, count nothing
                break;
            }
            if (exitw && (spins & 63u) == 0 &&
                __hip_atomic_load(exitw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == COPK_PMD_ABORT)
                return LB_GAVE_UP;            // the kernel aborts: publish nothing
            __builtin_amdgcn_s_sleep(1);
        }
    }
    if (lane == 0) lb_store(&chain[(size_t)j * stride], ep | (2ull << 30) | (excl + agg));
    return excl;
}

// Segmented decoupled look-back over K <= 8 chains at once (one per vport
// with demux, else one): lanes [q*seg, (q+1)*seg) resolve chain q, seg =
// 64 / next_pow2(K) predecessors per round. Granule g of chain q sits at
// chain[g*K + q], format as look_back(). The caller has already published
// granule gi's aggregates (lb_publish); this resolves them: returns, in
// every lane of group q, the exclusive prefix of chain q, and publishes the
// inclusive value agg + prefix. agg: chain q's aggregate in group q's lanes.
__device__ __forceinline__ uint32_t look_back_seg(unsigned long long *chain, uint32_t K, uint32_t gi, uint32_t agg,
                                                  uint32_t epoch, uint32_t *err, int lane)
{
    const uint32_t seg = K == 1 ? 64u : K == 2 ? 32u : K <= 4 ? 16u : 8u;
    const uint32_t q = (uint32_t)lane / seg, r = (uint32_t)lane % seg;
    const bool active = q < K;
    const unsigned long long segm = seg == 64 ? ~0ull : ((1ull << seg) - 1ull) << (q * seg);
    const uint32_t sh = seg == 64 ? 0u : q * seg;
    const unsigned long long ep = (unsigned long long)epoch << 32;
    uint32_t excl = 0;
    int qhi = (int)gi - 1;
    bool done = !active || gi == 0;
    uint32_t spins = 0;
    while (__ballot(!done)) {
        const int idx = qhi - (int)r;
        const bool inb = !done && idx >= 0;
        const unsigned long long v = inb ? lb_load(&chain[(size_t)idx * K + q]) : 0ull;
        const uint32_t flag = (uint32_t)(v >> 30) & 3u;
        const bool ok = inb && (uint32_t)(v >> 32) == epoch && flag != 0u;
        const unsigned long long mi = (__ballot(ok && flag == 2u) & segm) >> sh;
        const unsigned long long mb = (__ballot(inb && !ok) & segm) >> sh;
        const uint32_t first_incl = mi ? (uint32_t)__ffsll((long long)mi) - 1u : seg;
        const uint32_t first_bad = mb ? (uint32_t)__ffsll((long long)mb) - 1u : seg;
        const uint32_t upto = min(first_incl + 1u, first_bad);
        uint32_t val = (inb && r < upto) ? ((uint32_t)v & 0x3FFFFFFFu) : 0u;
        for (uint32_t off = seg >> 1; off; off >>= 1) val += __shfl_xor(val, (int)off);
        bool stalled = false;
        if (!done) {
            excl += val;
            if (first_incl < first_bad) {
                done = true;
            } else {
                qhi -= (int)upto;
                stalled = upto == 0;
            }
        }
        if (__ballot(stalled)) {
            if (++spins > (1u << 22)) {       // bounded: never hang the GPU
                if (lane == 0) *err = 1u;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    if (active && r == 0 && gi != 0) lb_store(&chain[(size_t)gi * K + q], ep | (2ull << 30) | (excl + agg));
    return excl;
}

// Publish granule gi's aggregates (lane q < K: chain q's agg_q): inclusive
// at once for the batch's first granule, else an aggregate.
__device__ __forceinline__ void lb_publish(unsigned long long *chain, uint32_t K, uint32_t gi, uint32_t agg_q,
                                           uint32_t epoch, int lane)
{
    if ((uint32_t)lane < K)
        lb_store(&chain[(size_t)gi * K + (uint32_t)lane],
                 ((unsigned long long)epoch << 32) | ((gi == 0 ? 2ull : 1ull) << 30) | agg_q);
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

// The batch a workgroup works on: a ring slot (ring launches) or a
// descriptor (kernarg). *look_off = the batch's first look-back granule.
__device__ __forceinline__ CopKBatch batch_desc(const CopKParams &p, uint32_t b, uint32_t *look_off)
{
    CopKBatch B;
    if (p.ring) {
        const uint32_t slot = (p.rg.first + b) % p.rg.n_slots;   // count may exceed n_slots
        B.pkts = p.rg.pkts + (size_t)slot * p.rg.pkts_slot_bytes;
        B.offsets = p.rg.offsets ? p.rg.offsets + (size_t)slot * p.rg.offsets_slot_words : nullptr;
        B.results = (uint2 *)p.rg.results + (size_t)slot * p.rg.results_slot;
        B.fwd_idx = p.rg.fwd_idx ? p.rg.fwd_idx + (size_t)slot * p.rg.fwd_slot : nullptr;
        // counts per slot: one, one per port (demux), or one per segment
        const uint32_t per = p.seg ? (p.rg.n + COPK_SEG - 1u) / COPK_SEG : p.demux ? p.demux : 1u;
        B.fwd_count = p.rg.fwd_count ? p.rg.fwd_count + (size_t)slot * per : nullptr;
        B.n = p.rg.n;
        B.stride = p.rg.stride;
        B.data_off = p.rg.data_off;
        B.ntiles = p.uniform_ntiles;
        *look_off = b * p.uniform_ntiles;
    } else {
        B = p.b[b];
        *look_off = p.look_begin[b];
    }
    return B;
}

// Batch of global tile g: by division when every batch has the same tile
// count, else a scalar scan of tile_begin[].
__device__ __forceinline__ uint32_t batch_of_tile(const CopKParams &p, uint32_t g)
{
    uint32_t b = 0;
    if (p.uniform_ntiles) {
        b = g / p.uniform_ntiles;
    } else {
#pragma unroll
        for (int q = 1; q < COPK_MAXB; q++) b += (q < (int)p.nb && p.tile_begin[q] <= g) ? 1u : 0u;
    }
    return __builtin_amdgcn_readfirstlane(b);
}

// Coalesced header loads of 64 consecutive packets (one "step" of a wave):
// three 16-byte non-temporal loads per lane move the first 48 bytes of the
// 64 packets; load c of lane l holds chunk (64c+l) mod 3 of packet
// (64c+l)/3, so each load instruction covers about 1 KiB of contiguous slot
// bytes (64-byte slots). StepGeom holds the per-lane constants.
struct StepGeom {
    uint32_t lpk[3], lch[3];   // packet (0..63) and chunk byte offset of load c
    uint32_t r3;               // lane % 3
    int a3, a67, a8;           // ds_bpermute byte addresses of this lane's sources
};

__device__ __forceinline__ StepGeom step_geom(int lane)
{
    StepGeom g;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const uint32_t q = (uint32_t)(c * 64 + lane);
        g.lpk[c] = q / 3u;
        g.lch[c] = (q % 3u) * 16u;
    }
    g.r3 = (uint32_t)lane % 3u;
    g.a3 = ((3 * lane) & 63) << 2;
    g.a67 = ((3 * lane + 1) & 63) << 2;
    g.a8 = ((3 * lane + 2) & 63) << 2;
    return g;
}

// System-coherent loads (sc0 sc1) at byte offset off of base: no L1 or L2
// copy is used, so a ring slot another agent rewrote since this launch last
// read it is read afresh (offsets below 2^31: one batch of a ring slot)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sys_rsrc(const void *base)
{
    return __builtin_amdgcn_make_buffer_rsrc((void *)base, 0, 0x7FFFFFFF, 0x00020000);
}
__device__ __forceinline__ u32x4 ld_sys16(__amdgpu_buffer_rsrc_t rs, uint32_t off)
{
    return __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 1 | 16);
}
__device__ __forceinline__ u32x2 ld_sys8(__amdgpu_buffer_rsrc_t rs, uint32_t off)
{
    return __builtin_amdgcn_raw_buffer_load_b64(rs, (int)off, 0, 1 | 16);
}
__device__ __forceinline__ uint32_t ld_sys4(__amdgpu_buffer_rsrc_t rs, uint32_t off)
{
    return __builtin_amdgcn_raw_buffer_load_b32(rs, (int)off, 0, 1 | 16);
}

// the three loads of the step starting at packet pb (clamped to `last`).
// sys: system-coherent loads (sc0 sc1: no L1 or L2 copy of the slot is
// used), for ring slots another agent may have rewritten since this launch
// last read them, instead of an acquire that invalidates the caches
__device__ __forceinline__ void load_step(const StepGeom &g, const uint8_t *pk0, uint32_t stride, uint32_t pb,
                                          uint32_t last, u32x4 (&v)[3], bool sys = false)
{
    if (sys) {
        const __amdgpu_buffer_rsrc_t rs = sys_rsrc(pk0);
#pragma unroll
        for (int c = 0; c < 3; c++) v[c] = ld_sys16(rs, min(pb + g.lpk[c], last) * stride + g.lch[c]);
        return;
    }
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const uint32_t ic = min(pb + g.lpk[c], last);
        v[c] = __builtin_nontemporal_load((const u32x4 *)(pk0 + (size_t)ic * stride + g.lch[c]));
    }
}

// IMIX (a slab with u32 offsets): the same three cooperative 16-byte loads
// per lane, at the step's packets' own offsets. Lane l holds the offset of
// the step's packet l (one coalesced dword load per lane, `off`); load c of
// lane s reads chunk (64c+s) mod 3 of packet (64c+s)/3, whose offset comes
// over by ds_bpermute, so gather_step applies unchanged. A wave's load
// instruction then touches about 22 packets' first lines, three lanes per
// line, where per-lane loads (a dwordx4 at byte 12 across a 16-byte
// boundary and a dwordx2 at 28) touch 64 lines per instruction, twice.
// Packet starts are 16-byte aligned and hold 48 readable bytes
// (include/cop_gpu.h, cop_batch).
__device__ __forceinline__ void load_step_imix(const StepGeom &g, const uint8_t *pkts, uint32_t off,
                                               uint32_t data_off, u32x4 (&v)[3], bool sys = false)
{
    uint32_t o[3];
#pragma unroll
    for (int c = 0; c < 3; c++)
        o[c] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(g.lpk[c] << 2), (int)off) + data_off + g.lch[c];
    if (sys) {
        const __amdgpu_buffer_rsrc_t rs = sys_rsrc(pkts);
#pragma unroll
        for (int c = 0; c < 3; c++) v[c] = ld_sys16(rs, o[c]);
        return;
    }
#pragma unroll
    for (int c = 0; c < 3; c++) v[c] = __builtin_nontemporal_load((const u32x4 *)(pkts + o[c]));
}

// the offset of the step's packet pb + lane (clamped to `last`)
__device__ __forceinline__ uint32_t load_off_imix(const uint32_t *offsets, uint32_t pb, int lane, uint32_t last,
                                                  bool sys = false)
{
    const uint32_t ic = min(pb + (uint32_t)lane, last);
    return sys ? ld_sys4(sys_rsrc(offsets), ic * 4u) : offsets[ic];
}

// The fields of this lane's packet (bytes 12..15 and 24..35) from the step's
// loads: source lane s holds chunk k of its packet in load (k - s) mod 3, so
// each field is one select at the source plus one ds_bpermute.
__device__ __forceinline__ void gather_step(const StepGeom &g, const u32x4 (&v)[3], uint32_t &w3, uint32_t &w6,
                                            uint32_t &w7, uint32_t &w8)
{
    const uint32_t c0w = g.r3 == 0 ? v[0].w : g.r3 == 1 ? v[2].w : v[1].w;
    const uint32_t c1z = g.r3 == 0 ? v[1].z : g.r3 == 1 ? v[0].z : v[2].z;
    const uint32_t c1w = g.r3 == 0 ? v[1].w : g.r3 == 1 ? v[0].w : v[2].w;
    const uint32_t c2x = g.r3 == 0 ? v[2].x : g.r3 == 1 ? v[1].x : v[0].x;
    w3 = (uint32_t)__builtin_amdgcn_ds_bpermute(g.a3, (int)c0w);
    w6 = (uint32_t)__builtin_amdgcn_ds_bpermute(g.a67, (int)c1z);
    w7 = (uint32_t)__builtin_amdgcn_ds_bpermute(g.a67, (int)c1w);
    w8 = (uint32_t)__builtin_amdgcn_ds_bpermute(g.a8, (int)c2x);
}

// The launch's optional features. A kernel instantiated without them
// (cop_kernels.hip EXT == false) passes all-zero options, so the compiler
// drops their code: the hot configuration's kernel is about half the size,
// and every launch starts with cold instruction caches.
struct Opt {
    uint32_t demux;                  // one ordered forward list per port
    uint32_t port_stats;             // per-port counters for ports < port_stats
    uint32_t dbg;                    // timing-only ablations ($COP_DBG)
    unsigned long long *rule_hits;   // per-rule FW hit counters or nullptr
};

__device__ __forceinline__ Opt opt_all(const CopKParams &p)
{
    return Opt{p.demux, p.port_stats, p.dbg, p.rule_hits};
}

// LDS views of the tables (staged at workgroup start)
struct Tables {
    uint32_t *rt_top;
    uint16_t *rt_leaf;
    uint32_t *fw_s, *fw_v, *lp_s, *lp_v;
};

// A random tbl24 probe: plain (cached) load, or non-temporal ($COP_PROBE_NT,
// experiment: whether the streaming hint changes what a miss fetches)
__device__ __forceinline__ uint32_t probe_ld(const uint32_t *a, uint32_t nt)
{
    return nt ? __builtin_nontemporal_load(a) : *a;
}

// The bucketed route form's first round (COPK_TBL_BKT): the bucket's first
// candidate and the next bucket's (both issued, not waited for)
__device__ __forceinline__ void bkt_issue(const uint32_t *bidx, uint32_t ib, uint32_t ip, bool reach, uint32_t &k0,
                                          uint32_t &k1)
{
    if (reach) {
        const u32x2a x = *(const u32x2a *)(bidx + (ip >> (32u - ib)));
        k0 = x.x;
        k1 = x.y;
    } else {
        k0 = k1 = 0;
    }
}

// Pass 1, per step: parse, vport route (stage P), interval searches in LDS,
// and the tbl24 loads of DIR-24-8 stages (issued, not waited for).
// w3 = bytes 12..15, w6/w7/w8 = bytes 24..35 of the packet as loaded (LE).
template <int FW, int LPM, int PPT>
__device__ __forceinline__ void pass1(const CopKParams &p, const Tables &t, const uint32_t (&w3)[PPT],
                                      const uint32_t (&w6)[PPT], const uint32_t (&w7)[PPT],
                                      const uint32_t (&w8)[PPT], uint32_t (&verdict)[PPT], uint32_t (&port)[PPT],
                                      uint32_t (&src)[PPT], uint32_t (&dst)[PPT], uint32_t (&fwe)[PPT],
                                      uint32_t (&lpe)[PPT], uint32_t (&lpe2)[PPT], uint32_t (&fwe2)[PPT])
{
    const bool stageP = (p.stages & COPK_STAGE_PARSE) != 0;
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        verdict[k] = COPK_FORWARD;
        port[k] = 0;
        const uint32_t et = ((w3[k] & 0xFFu) << 8) | ((w3[k] >> 8) & 0xFFu);
        dst[k] = bswap32(__builtin_amdgcn_alignbit(w8[k], w7[k], 16));
        src[k] = bswap32(__builtin_amdgcn_alignbit(w7[k], w6[k], 16));
        if (stageP) {
            if (et != 0x0800u) {
                verdict[k] = COPK_DROP_PARSE;
                port[k] = 0xFFFFu;
            } else {
                const uint32_t idx = dst[k] & 0xFFFFu;
                const uint32_t top = t.rt_top[idx >> 8];
                port[k] = (top & 0x80000000u) ? (uint32_t)t.rt_leaf[((top & 0xFFFFu) << 8) | (idx & 0xFFu)]
                                              : (top & 0xFFFFu);
                if (port[k] == 0xFFFFu) verdict[k] = COPK_DROP_PARSE;
                else if (port[k] >= p.n_ports) verdict[k] = COPK_DROP_NO_PORT;
            }
        }
        // HBM probes only for packets that reach the coprocessor (masked-off
        // lanes send no request); the others keep their stage-P verdict
        const bool reach = verdict[k] == COPK_FORWARD;
        if (FW == COPK_TBL_IVT) fwe[k] = ivt_value(t.fw_s, t.fw_v, p.fw_m, p.fw_ib, p.fw_lv, src[k]);
        if (FW == COPK_TBL_DIR) fwe[k] = reach ? probe_ld(&p.fw_tbl24[src[k] >> 8], p.probe_nt) : 0u;
        if (FW == COPK_TBL_BKT) bkt_issue(p.fw_bidx, p.fw_ib, src[k], reach, fwe[k], fwe2[k]);
        if (LPM == COPK_TBL_IVT) lpe[k] = ivt_value(t.lp_s, t.lp_v, p.lpm_m, p.lpm_ib, p.lpm_lv, dst[k]);
        if (LPM == COPK_TBL_DIR) lpe[k] = reach ? probe_ld(&p.lpm_tbl24[dst[k] >> 8], p.probe_nt) : 0u;
        if (LPM == COPK_TBL_TRIE) lpe[k] = t.lp_s[dst[k] >> 20];
        if (LPM == COPK_TBL_BKT) bkt_issue(p.lpm_bidx, p.lpm_ib, dst[k], reach, lpe[k], lpe2[k]);
    }
}

// The trie form's walk below its LDS top level (lpm_trie.c): e = the level-0
// entry, a node (bit 31) or already the value. Per level every live lane's
// PPT node loads (24 bytes: a dwordx4 and a dwordx2) are issued before any
// is used; a lane leaves at its first leaf child, whose value is loaded in
// one last round. Nodes and leaves are small enough to stay in the XCD's L2.
template <int PPT>
__device__ __forceinline__ void trie_walk(const uint32_t *nodes, const uint32_t *leaves, const uint32_t (&ip)[PPT],
                                          uint32_t (&e)[PPT], const bool (&live)[PPT])
{
    bool in[PPT], lf[PPT];
    bool any = false;
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        in[k] = live[k] && (e[k] & 0x80000000u);
        lf[k] = false;
        any |= in[k];
    }
#pragma unroll
    for (int l = 0; l < 4; l++) {
        if (!__ballot(any)) break;
        const uint32_t sh = l == 0 ? 14u : l == 1 ? 8u : l == 2 ? 2u : 0u;
        const uint32_t msk = l == 3 ? 3u : 63u;
        u32x4a a[PPT];
        u32x2a b[PPT];
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            if (in[k]) {
                const uint32_t *nd = nodes + (size_t)(e[k] & 0x7FFFFFFFu) * 6u;
                a[k] = *(const u32x4a *)nd;
                b[k] = *(const u32x2a *)(nd + 4);
            }
        }
        any = false;
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            if (in[k]) {
                const uint32_t c = (ip[k] >> sh) & msk;
                const unsigned long long vec = a[k].x | ((unsigned long long)a[k].y << 32);
                const unsigned long long lv = a[k].z | ((unsigned long long)a[k].w << 32);
                const unsigned long long upto = (2ull << c) - 1ull;   // c == 63: all ones
                if ((vec >> c) & 1ull) {
                    e[k] = 0x80000000u | (b[k].x + (uint32_t)__popcll(vec & upto) - 1u);
                    any = true;
                } else {
                    e[k] = b[k].y + (uint32_t)__popcll(lv & upto) - 1u;
                    in[k] = false;
                    lf[k] = true;
                }
            }
        }
    }
#pragma unroll
    for (int k = 0; k < PPT; k++)
        if (lf[k]) e[k] = leaves[e[k]];
}

// rte_lpm_lookup's tbl8 step for valid+extended tbl24 entries e[k]: a
// direct group load, or (packed) the run block's header word, then the run's
// entry (cop_kernels.h COPK_TBL_DIR). All PPT loads of a level are issued
// before any is used.
template <int PPT>
__device__ __forceinline__ void tbl8_step(const uint32_t *tbl8, uint32_t packed, const uint32_t (&ip)[PPT],
                                          uint32_t (&e)[PPT])
{
    bool ext[PPT];
#pragma unroll
    for (int k = 0; k < PPT; k++) ext[k] = (e[k] & 0x03000000u) == 0x03000000u;
    if (!packed) {
#pragma unroll
        for (int k = 0; k < PPT; k++)
            if (ext[k]) e[k] = tbl8[((size_t)(e[k] & 0x00FFFFFFu) << 8) | (ip[k] & 0xFFu)];
        return;
    }
    unsigned long long h[PPT];
#pragma unroll
    for (int k = 0; k < PPT; k++)
        h[k] = ext[k] ? ((const unsigned long long *)(tbl8 + ((size_t)(e[k] & 0x00FFFFFFu) << 4)))[(ip[k] & 0xFFu) >> 5]
                      : 0ull;
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        if (ext[k]) {
            const uint32_t bit = ip[k] & 31u;
            const uint32_t rank = (uint32_t)(h[k] >> 32) + (uint32_t)__popc((uint32_t)h[k] & (0xFFFFFFFFu >> (31u - bit)));
            e[k] = tbl8[((size_t)(e[k] & 0x00FFFFFFu) << 4) + 16u + rank - 1u];
        }
    }
}

// tbl8_step in two halves for one packet per lane, so a step pipeline can
// issue a step's tbl8 load and use it one step later (tile_steps_v):
// tbl8_issue loads the group entry (plain) or the run block's header word
// (packed); tbl8_finish returns the entry (packed: the run's entry, one more
// dependent load).
struct T8 {
    bool ext;
    unsigned long long h;
};
__device__ __forceinline__ T8 tbl8_issue(const uint32_t *tbl8, uint32_t packed, uint32_t ip, uint32_t e)
{
    T8 t;
    t.ext = (e & 0x03000000u) == 0x03000000u;
    t.h = 0;
    if (t.ext) {
        if (!packed) t.h = tbl8[((size_t)(e & 0x00FFFFFFu) << 8) | (ip & 0xFFu)];
        else t.h = ((const unsigned long long *)(tbl8 + ((size_t)(e & 0x00FFFFFFu) << 4)))[(ip & 0xFFu) >> 5];
    }
    return t;
}
__device__ __forceinline__ uint32_t tbl8_finish(const uint32_t *tbl8, uint32_t packed, uint32_t ip, uint32_t e,
                                                const T8 &t)
{
    if (!t.ext) return e;
    if (!packed) return (uint32_t)t.h;
    const uint32_t bit = ip & 31u;
    const uint32_t rank = (uint32_t)(t.h >> 32) + (uint32_t)__popc((uint32_t)t.h & (0xFFFFFFFFu >> (31u - bit)));
    return tbl8[((size_t)(e & 0x00FFFFFFu) << 4) + 16u + rank - 1u];
}

// The bucketed route form's second round (COPK_TBL_BKT, lpm_bkt.c): for
// each reached packet with candidates k0..k1 (start k0 <= ip, R(ip) <= k1),
// one 64-byte read of pairs k0 .. k0 + 7 (four 16-byte loads, all PPT
// packets' issued before any is used) decides every lookup whose bucket
// holds at most 7 boundaries; lanes in a wider bucket (rare) scan on, two
// pairs (one 16-byte load) a round, until a start above ip or k1. So a
// wave's lookups take two dependent L2 rounds, the index and the pairs,
// where a search that read one pair per round paid a third and fourth
// round for the wave's densest bucket.
// e[k] <- the interval's value (the rte_lpm entry form: bit 24 hit, nh).
template <int PPT>
__device__ __forceinline__ void bkt_step(const uint32_t *pairs, const uint32_t (&ip)[PPT], uint32_t (&e)[PPT],
                                         const uint32_t (&k1)[PPT], const bool (&live)[PPT])
{
    u32x4a q[PPT][4];
#pragma unroll
    for (int k = 0; k < PPT; k++)
        if (live[k]) {
            const uint32_t *b = pairs + 2 * (size_t)e[k];
#pragma unroll
            for (int h = 0; h < 4; h++) q[k][h] = *(const u32x4a *)(b + 4 * h);
        }
    bool more[PPT];
    uint32_t nxt[PPT];
    bool any = false;
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        more[k] = false;
        nxt[k] = 0;
        if (!live[k]) continue;
        const uint32_t k0 = e[k], w = k1[k] - k0;   // candidates k0 .. k0 + w
        uint32_t v = q[k][0].y;                      // start k0 <= ip always
#pragma unroll
        for (int t = 1; t < 8; t++) {
            const u32x4a &c = q[k][t >> 1];
            const uint32_t st = (t & 1) ? c.z : c.x, va = (t & 1) ? c.w : c.y;
            if (w >= (uint32_t)t && ip[k] >= st) v = va;
        }
        e[k] = v;
        more[k] = w > 7u && ip[k] >= q[k][3].z;      // start k0 + 7 <= ip: the answer lies further on
        nxt[k] = k0 + 8u;
        any |= more[k];
    }
    // the wide bucket: pairs j, j + 1 per round (pads past the end hold
    // start 0xFFFFFFFF; j <= k1 <= m - 1, so j + 1 < m + 8)
    while (__ballot(any)) {
        u32x4a c[PPT];
#pragma unroll
        for (int k = 0; k < PPT; k++)
            if (more[k]) c[k] = *(const u32x4a *)(pairs + 2 * (size_t)nxt[k]);
        any = false;
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            if (!more[k]) continue;
            const uint32_t j = nxt[k], hi = k1[k];
            if (ip[k] >= c[k].x) e[k] = c[k].y;        // j <= k1 always
            if (j + 1u <= hi && ip[k] >= c[k].z) e[k] = c[k].w;
            more[k] = j + 1u < hi && ip[k] >= c[k].z;
            any |= more[k];
            nxt[k] = j + 2u;
        }
    }
}

// The bucketed form's second round split for the poll-mode step pipeline
// (cop_tile.h tile_steps_v): one packet per lane, its eight pairs' loads
// issued in one round (bkt_pairs_issue) and used in the next
// (bkt_pairs_finish: the selection of bkt_step, then its wide-bucket rounds,
// a wave-uniform loop).
struct BkQ {
    u32x4a q[4];
};
__device__ __forceinline__ BkQ bkt_pairs_issue(const uint32_t *pairs, uint32_t k0, bool live)
{
    BkQ b;
    if (live) {
        const uint32_t *a = pairs + 2 * (size_t)k0;
#pragma unroll
        for (int h = 0; h < 4; h++) b.q[h] = *(const u32x4a *)(a + 4 * h);
    } else {
#pragma unroll
        for (int h = 0; h < 4; h++) b.q[h] = u32x4a{0u, 0u, 0u, 0u};
    }
    return b;
}
__device__ __forceinline__ uint32_t bkt_pairs_finish(const uint32_t *pairs, uint32_t ip, uint32_t k0, uint32_t k1,
                                                     bool live, const BkQ &b)
{
    uint32_t e = k0;
    bool more = false;
    uint32_t nxt = 0;
    if (live) {
        const uint32_t w = k1 - k0;   // candidates k0 .. k0 + w
        uint32_t v = b.q[0].y;        // start k0 <= ip always
#pragma unroll
        for (int t = 1; t < 8; t++) {
            const u32x4a &c = b.q[t >> 1];
            const uint32_t st = (t & 1) ? c.z : c.x, va = (t & 1) ? c.w : c.y;
            if (w >= (uint32_t)t && ip >= st) v = va;
        }
        e = v;
        more = w > 7u && ip >= b.q[3].z;
        nxt = k0 + 8u;
    }
    while (__ballot(more)) {
        u32x4a c{0u, 0u, 0u, 0u};
        if (more) c = *(const u32x4a *)(pairs + 2 * (size_t)nxt);
        if (more) {
            if (ip >= c.x) e = c.y;
            if (nxt + 1u <= k1 && ip >= c.z) e = c.w;
            more = nxt + 1u < k1 && ip >= c.z;
            nxt += 2u;
        }
    }
    return e;
}

// Pass 2: rte_lpm_lookup's tbl8 step for valid+extended entries, then the
// verdicts of stage FW (firewall.c:183-210) and stage LPM. Packets that did
// not reach the coprocessor (stage P drop) keep their verdict. Counts the
// FW stage's pkt_total / pkt_not_ipv4 (firewall.h:56-61) over valid packets.
// LPM_T8 false: the route's second round was done by the caller (tbl8_issue /
// tbl8_finish, or bkt_pairs_issue / bkt_pairs_finish).
template <int FW, int LPM, int PPT, bool LPM_T8 = true>
__device__ __forceinline__ void pass2(const CopKParams &p, const uint32_t (&w3)[PPT], const uint32_t (&src)[PPT],
                                      const uint32_t (&dst)[PPT], const bool (&valid)[PPT], uint32_t (&fwe)[PPT],
                                      uint32_t (&lpe)[PPT], const uint32_t (&lpe2)[PPT], const uint32_t (&fwe2)[PPT],
                                      uint32_t (&verdict)[PPT], uint32_t (&flags)[PPT], uint32_t (&rnh)[PPT],
                                      uint32_t &c_total, uint32_t &c_notv4)
{
    bool reached[PPT];
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        reached[k] = verdict[k] == COPK_FORWARD;   // entered the coprocessor
        flags[k] = 0;
        rnh[k] = 0;
    }
    if (FW == COPK_TBL_DIR) tbl8_step<PPT>(p.fw_tbl8, p.fw_tbl8_packed, src, fwe);
    if (FW == COPK_TBL_BKT) bkt_step<PPT>(p.fw_bpairs, src, fwe, fwe2, reached);
    if (LPM == COPK_TBL_DIR && LPM_T8) tbl8_step<PPT>(p.lpm_tbl8, p.lpm_tbl8_packed, dst, lpe);
    if (LPM == COPK_TBL_TRIE) trie_walk<PPT>(p.lpm_tnodes, p.lpm_tleaves, dst, lpe, reached);
    if (LPM == COPK_TBL_BKT && LPM_T8) bkt_step<PPT>(p.lpm_bpairs, dst, lpe, lpe2, reached);
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
}

// Per-rule hit counters: one relaxed device-scope u64 add per FW-stage hit
// (no return value: fire-and-forget atomics at the L2/fabric).
template <int FW, int PPT>
__device__ __forceinline__ void rule_hit_atomics(const Opt &o, const bool (&valid)[PPT],
                                                 const uint32_t (&flags)[PPT], const uint32_t (&fwe)[PPT])
{
    if (FW != COPK_TBL_OFF && o.rule_hits) {
#pragma unroll
        for (int k = 0; k < PPT; k++)
            if (valid[k] && (flags[k] & COPK_FLAG_FW_HIT))
                __hip_atomic_fetch_add(&o.rule_hits[fwe[k] & 0x00FFFFFFu], 1ull, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Result records (8 B per packet, coalesced, non-temporal: read by the host
// or the next stage, never by this kernel) and the per-lane verdict counts.
struct Counts {
    uint32_t total = 0, notv4 = 0, fwd = 0, dropfw = 0, parse = 0, noport = 0, rhit = 0, rx = 0;
};

// rec_stage != nullptr: the records go to LDS (tile order) instead, and
// copy_out_records writes them as 16-byte stores once the tile's barrier
// has passed (the poll-mode kernel's write-through stores: wide stores)
template <int PPT, bool WT>
__device__ __forceinline__ void store_records(const CopKBatch &B, uint32_t base, int tid, const bool (&valid)[PPT],
                                              const uint32_t (&verdict)[PPT], const uint32_t (&flags)[PPT],
                                              const uint32_t (&port)[PPT], const uint32_t (&rnh)[PPT],
                                              bool (&fwd)[PPT], Counts &c, uint32_t *rec_stage)
{
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        fwd[k] = valid[k] && verdict[k] == COPK_FORWARD;
        if (valid[k]) {
            u32x2 rec;
            rec.x = verdict[k] | (flags[k] << 8) | (port[k] << 16);
            rec.y = rnh[k];
            if (rec_stage) *(u32x2 *)&rec_stage[2 * (k * BLOCK + tid)] = rec;
            else st_u32x2<WT>(rec, &((u32x2 *)B.results)[base + k * BLOCK + tid]);
            c.rx++;
            c.fwd += verdict[k] == COPK_FORWARD;
            c.dropfw += verdict[k] == COPK_DROP_FW;
            c.parse += verdict[k] == COPK_DROP_PARSE;
            c.noport += verdict[k] == COPK_DROP_NO_PORT;
            c.rhit += flags[k] & COPK_FLAG_ROUTE_HIT;
        }
    }
}

// The poll-mode kernel's records without an LDS stage: each wave writes its
// own packets' records as 16-byte write-through stores straight from
// registers. The records of (step k, wave) are 64 consecutive 8-byte slots;
// for two steps at a time, lane i < 32 gathers records 2i and 2i+1 of step k
// and lane 32 + i those of step k+1 (four ds_bpermute per step), so one
// store instruction writes 1 KiB contiguous per step pair. No barrier: waves
// 1..3 store while wave 0 looks back. An odd last record takes an 8-byte
// store. Counts as store_records.
template <int PPT, bool WT>
__device__ __forceinline__ void store_records_paired(const CopKBatch &B, uint32_t base, int tid, int lane, int wave,
                                                     const bool (&valid)[PPT], const uint32_t (&verdict)[PPT],
                                                     const uint32_t (&flags)[PPT], const uint32_t (&port)[PPT],
                                                     const uint32_t (&rnh)[PPT], bool (&fwd)[PPT], Counts &c)
{
    uint32_t rx[PPT];
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        fwd[k] = valid[k] && verdict[k] == COPK_FORWARD;
        rx[k] = verdict[k] | (flags[k] << 8) | (port[k] << 16);
        if (valid[k]) {
            c.rx++;
            c.fwd += verdict[k] == COPK_FORWARD;
            c.dropfw += verdict[k] == COPK_DROP_FW;
            c.parse += verdict[k] == COPK_DROP_PARSE;
            c.noport += verdict[k] == COPK_DROP_NO_PORT;
            c.rhit += flags[k] & COPK_FLAG_ROUTE_HIT;
        }
    }
    (void)tid;
    uint32_t *r = (uint32_t *)B.results;
    const int i = lane & 31;
    const bool hi = lane >= 32;
#pragma unroll
    for (int k = 0; k < PPT; k += 2) {
        const int k1 = k + 1 < PPT ? k + 1 : k;
        const uint32_t a0 = (uint32_t)__shfl((int)rx[k], 2 * i), a1 = (uint32_t)__shfl((int)rnh[k], 2 * i);
        const uint32_t a2 = (uint32_t)__shfl((int)rx[k], 2 * i + 1), a3 = (uint32_t)__shfl((int)rnh[k], 2 * i + 1);
        const uint32_t b0 = (uint32_t)__shfl((int)rx[k1], 2 * i), b1 = (uint32_t)__shfl((int)rnh[k1], 2 * i);
        const uint32_t b2 = (uint32_t)__shfl((int)rx[k1], 2 * i + 1), b3 = (uint32_t)__shfl((int)rnh[k1], 2 * i + 1);
        if (hi && k1 == k) continue;   // PPT 1: one step, lanes 0..31 store it
        const uint32_t idx = base + (uint32_t)(hi ? k1 : k) * BLOCK + (uint32_t)wave * 64u + 2u * (uint32_t)i;
        const u32x4 v = hi ? u32x4{b0, b1, b2, b3} : u32x4{a0, a1, a2, a3};
        if (idx + 1 < B.n) st_u32x4<WT>(v, r, 2 * (long)idx);
        else if (idx < B.n) st_u32x2<WT>(u32x2{v.x, v.y}, (u32x2 *)&r[2 * (size_t)idx]);
    }
}

// Copy a tile's staged records (m = valid packets of the tile, 8 B each,
// LDS in tile order) to results[base ..]: 16-byte stores (two records), an
// 8-byte store for an odd last one. All BLOCK threads; results 16-byte
// aligned at even packet indices (base is a multiple of 256).
template <bool WT>
__device__ __forceinline__ void copy_out_records(void *results, uint32_t base, uint32_t m, const uint32_t *stage,
                                                 int tid)
{
    uint32_t *r = (uint32_t *)results + 2 * (size_t)base;
    for (uint32_t c = (uint32_t)tid; c < m / 2; c += BLOCK) {
        const u32x4 v = *(const u32x4 *)&stage[4 * c];
        st_u32x4<WT>(v, r, 4 * (long)c);
    }
    if ((m & 1u) && tid == 0) st_u32x2<WT>(*(const u32x2 *)&stage[2 * (m - 1)], (u32x2 *)&r[2 * (m - 1)]);
}

// One 16-byte chunk of a segment's list (words w0..w0+3 of fwd_idx, from
// LDS). The chunk that would reach past the batch's n entries (the last
// segment's, when its list length is not a multiple of 4) is stored word by
// word, only its words below n: fwd_idx holds n entries, no more.
template <bool WT>
__device__ __forceinline__ void st_list_chunk(const uint32_t *src, uint32_t *fwd_idx, uint32_t w0, uint32_t n)
{
    if (w0 + 4u <= n) {
        st_u32x4<WT>(*(const u32x4 *)src, fwd_idx, (long)w0);
    } else {
#pragma unroll
        for (uint32_t i = 0; i < 4u; i++)
            if (w0 + i < n) st_u32<WT>(src[i], &fwd_idx[w0 + i]);
    }
}

// Copy a tile's forward list (agg indices staged in LDS, in order) to
// fwd_idx[pref ..]: 16-byte non-temporal stores on 16-byte boundaries of
// the list, partial words only at the two ends. All BLOCK data threads.
template <bool WT>
__device__ __forceinline__ void copy_out_list(uint32_t *fwd_idx, uint32_t pref, uint32_t agg, const uint32_t *stage,
                                              int tid)
{
    const int mis = (int)(((uintptr_t)fwd_idx >> 2) & 3u);
    const long a0 = (long)(((pref + (uint32_t)mis) & ~3u)) - mis;
    const long end = (long)pref + agg;
    const uint32_t nch = (uint32_t)((end - a0 + 3) / 4);
    for (uint32_t c = (uint32_t)tid; c < nch; c += BLOCK) {
        const long w0 = a0 + 4 * (long)c;
        if (w0 >= (long)pref && w0 + 4 <= end) {
            const uint32_t i = (uint32_t)(w0 - (long)pref);
            u32x4 v;
            v.x = stage[i];
            v.y = stage[i + 1];
            v.z = stage[i + 2];
            v.w = stage[i + 3];
            st_u32x4<WT>(v, fwd_idx, w0);
        } else {
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const long w = w0 + i;
                if (w >= (long)pref && w < end) st_u32<WT>(stage[w - (long)pref], &fwd_idx[w]);
            }
        }
    }
}

// The look-back chain state of a launch (one-shot kernel) or of one batch
// (poll-mode kernel: epoch = the batch's sequence tag).
struct LookCtx {
    unsigned long long *look;
    uint32_t epoch;
    uint32_t *err;
    const uint32_t *exitw = nullptr;   // poll-mode kernel: its exit word (look_back)
    uint32_t spin_log2 = 22;           // look_back's spin bound (tests shorten it)
};

// LDS scratch of one compaction: per-(step, wave) counts and the prefix of
// the single-list form, or per-port counts and prefixes with demux.
struct CompactLds {
    uint32_t *cnt;    // [PPT*WAVES]
    uint32_t *pref;   // [1]
    uint32_t *dq;     // [COPK_MAX_DEMUX_PORTS][PPT*WAVES]
    uint32_t *dpref;  // [COPK_MAX_DEMUX_PORTS]
    uint32_t *stage;           // [BLOCK*PPT] the tile's forward list (single-list form) or nullptr
};

// Ordered compaction of one tile (packets base + k*BLOCK + tid): the
// forward list of the batch, or one list per vport with demux (the tx_q
// order of each port's coprocessor, switch.c:306-327 + 464-470; port q's
// list at fwd_idx + q*n, its length at fwd_count[q]). Tile-local ballots and
// an LDS scan over (step, wave), then decoupled look-back over the tiles of
// the batch (one chain per port with demux, spread over the waves).
// Contains two workgroup barriers; lb_off = the batch's first granule.
// mid() runs between the look-back and the second barrier: the caller's
// record stores go there, so the look-back's loads (vmcnt retires in order)
// do not wait for them and the other waves store while wave 0 looks back.
// Returns false when a look-back gave up (poll-mode abort, LB_GAVE_UP): the
// tile then wrote no list and no count (workgroup-uniform).
template <int PPT, bool WT, typename Mid>
__device__ __forceinline__ bool compact_tile(const LookCtx &lk, const Opt &o, const CopKBatch &B, uint32_t lb_off,
                                             uint32_t j,
                                             uint32_t base, const bool (&fwd)[PPT], const uint32_t (&port)[PPT],
                                             bool seg, const CompactLds &s, int tid, int lane, int wave, Mid mid)
{
    constexpr int NQ = PPT * WAVES;
    if (seg) {
        // Segmented lists (COP_CFG_SEG_LISTS): step k of the tile is segment
        // base/COPK_SEG + k, whose list is written at fwd_idx[(base + k*BLOCK) ..]
        // and its length at fwd_count[segment]. Ballots and an LDS scan over
        // the step's four waves order it; no other tile is involved.
        static_assert(COPK_SEG == BLOCK, "one segment per tile step");
        unsigned long long bal[PPT];
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            bal[k] = __ballot(fwd[k]);
            if (lane == 0) s.cnt[k * WAVES + wave] = (uint32_t)__popcll(bal[k]);
        }
        lds_barrier();
        if (B.fwd_idx && !(o.dbg & 64u)) {
#pragma unroll
            for (int k = 0; k < PPT; k++) {
                uint32_t off = 0;
#pragma unroll
                for (int w = 0; w < WAVES; w++) off += w < wave ? s.cnt[k * WAVES + w] : 0u;
                if (fwd[k])
                    s.stage[k * BLOCK + off +
                            __builtin_amdgcn_mbcnt_hi((uint32_t)(bal[k] >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)bal[k], 0u))] =
                        base + k * BLOCK + tid;
            }
        }
        // the segments' lengths (segments holding packets of the batch only)
        if (B.fwd_count && wave == 0 && lane < PPT && base + (uint32_t)lane * BLOCK < B.n) {
            uint32_t c = 0;
#pragma unroll
            for (int w = 0; w < WAVES; w++) c += s.cnt[lane * WAVES + w];
            st_u32<WT>(c, B.fwd_count + base / COPK_SEG + (uint32_t)lane);
        }
        mid();
        lds_barrier();
        if (B.fwd_idx && !(o.dbg & 64u)) {
            // 16-byte stores of each segment's first ceil(len/4) chunks
            for (uint32_t q = (uint32_t)tid; q < (uint32_t)PPT * (BLOCK / 4); q += BLOCK) {
                const uint32_t k = q / (BLOCK / 4), cc = q % (BLOCK / 4);
                uint32_t c = 0;
#pragma unroll
                for (int w = 0; w < WAVES; w++) c += s.cnt[k * WAVES + w];
                if (cc * 4u < c) st_list_chunk<WT>(&s.stage[k * BLOCK + cc * 4u], B.fwd_idx, base + k * BLOCK + cc * 4u, B.n);
            }
        }
        return true;
    }
    if (!o.demux) {
        unsigned long long bal[PPT];
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            bal[k] = __ballot(fwd[k]);
            if (lane == 0) s.cnt[k * WAVES + wave] = (uint32_t)__popcll(bal[k]);
        }
        lds_barrier();
        // every wave scans the tile's (step, wave) counts for its own offsets
        uint32_t agg;
        const uint32_t ex = wave_excl_scan(lane < NQ ? s.cnt[lane] : 0u, NQ, lane, &agg);
        uint32_t off[PPT];
#pragma unroll
        for (int k = 0; k < PPT; k++) off[k] = (uint32_t)__shfl((int)ex, k * WAVES + wave);
        const bool staged = s.stage != nullptr && B.fwd_idx && !(o.dbg & 64u);
        if (staged) {
            // the tile's list in LDS, in order, while wave 0 looks back
#pragma unroll
            for (int k = 0; k < PPT; k++)
                if (fwd[k])
                    s.stage[off[k] + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal[k] >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)bal[k], 0u))] =
                        base + k * BLOCK + tid;
        }
        if (wave == 0) {
            // dbg bit 32 (timing-only ablation): no look-back wait, wrong offsets
            const uint32_t excl =
                (o.dbg & 32u) ? j * 1024u : look_back(lk.look + lb_off, 1u, j, agg, lk.epoch, lk.err, lane, lk.exitw, lk.spin_log2);
            if (lane == 0) {
                *s.pref = excl;
                if (B.fwd_count && j == B.ntiles - 1 && excl != LB_GAVE_UP) st_u32<WT>(excl + agg, B.fwd_count);
            }
        }
        mid();
        lds_barrier();
        const uint32_t pref = *s.pref;
        if (pref == LB_GAVE_UP) return false;
        if (staged) {
            copy_out_list<WT>(B.fwd_idx, pref, agg, s.stage, tid);
        } else if (B.fwd_idx && !(o.dbg & 64u)) {
#pragma unroll
            for (int k = 0; k < PPT; k++) {
                if (fwd[k]) {
                    const uint32_t r = __builtin_amdgcn_mbcnt_hi(
                        (uint32_t)(bal[k] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal[k], 0u));
                    st_u32<WT>(base + k * BLOCK + tid, &B.fwd_idx[pref + off[k] + r]);
                }
            }
        }
        return true;
    }
    const uint32_t K = o.demux;
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        for (uint32_t q = 0; q < K; q++) {
            const unsigned long long b = __ballot(fwd[k] && port[k] == q);
            if (lane == 0) s.dq[q * NQ + k * WAVES + wave] = (uint32_t)__popcll(b);
        }
    }
    lds_barrier();
    for (uint32_t q = (uint32_t)wave; q < K; q += WAVES) {
        uint32_t agg;
        const uint32_t ex = wave_excl_scan(lane < NQ ? s.dq[q * NQ + lane] : 0u, NQ, lane, &agg);
        if (lane < NQ) s.dq[q * NQ + lane] = ex;
        const uint32_t excl = look_back(lk.look + (size_t)lb_off * K + q, K, j, agg, lk.epoch, lk.err, lane, lk.exitw,
                                         lk.spin_log2);
        if (lane == 0) {
            s.dpref[q] = excl;
            if (B.fwd_count && j == B.ntiles - 1 && excl != LB_GAVE_UP) st_u32<WT>(excl + agg, &B.fwd_count[q]);
        }
    }
    mid();
    lds_barrier();
    for (uint32_t q = 0; q < K; q++)
        if (s.dpref[q] == LB_GAVE_UP) return false;
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
                st_u32<WT>(base + k * BLOCK + tid,
                           &B.fwd_idx[(size_t)q * B.n + s.dpref[q] + s.dq[q * NQ + k * WAVES + wave] + r]);
            }
        }
    }
    return true;
}

// The tile's verdict counters as wave-uniform totals from ballots (scalar
// popcounts: no cross-lane reduction chains). Same values as the per-lane
// Counts of pass2 + store_records summed over the wave.
template <int FW, int PPT>
__device__ __forceinline__ Counts wave_counts(const bool (&valid)[PPT], const uint32_t (&verdict)[PPT],
                                              const uint32_t (&flags)[PPT])
{
    Counts c;
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        const uint32_t v = verdict[k];
        const bool in = valid[k];
        const bool reached = v != COPK_DROP_PARSE && v != COPK_DROP_NO_PORT;
        c.rx += (uint32_t)__popcll(__ballot(in));
        c.fwd += (uint32_t)__popcll(__ballot(in && v == COPK_FORWARD));
        c.dropfw += (uint32_t)__popcll(__ballot(in && v == COPK_DROP_FW));
        c.parse += (uint32_t)__popcll(__ballot(in && v == COPK_DROP_PARSE));
        c.noport += (uint32_t)__popcll(__ballot(in && v == COPK_DROP_NO_PORT));
        c.rhit += (uint32_t)__popcll(__ballot(in && (flags[k] & COPK_FLAG_ROUTE_HIT)));
        if (FW != COPK_TBL_OFF) {
            c.total += (uint32_t)__popcll(__ballot(in && reached));
            c.notv4 += (uint32_t)__popcll(__ballot(in && v == COPK_DROP_NOT_IPV4));
        }
    }
    return c;
}

// The counters' per-workgroup adds (after a barrier that follows every
// wave's s_red writes): cop_counters order, one atomic per counter.
__device__ __forceinline__ void counters_add(const CopKParams &p, const uint32_t *s_red, int tid)
{
    if (tid < 9) {
        uint32_t r[8];
#pragma unroll
        for (int q = 0; q < 8; q++) {
            uint32_t v = 0;
#pragma unroll
            for (int w = 0; w < WAVES; w++) v += s_red[w * 8 + q];
            r[q] = v;
        }
        // s_red order: total, notv4, fwd, dropfw, parse, noport, rhit, rx;
        // cop_counters order: drop, accept, not_ipv4, total, parse_err, no_port, forward, route_hit, rx
        const uint32_t v = tid == 0 ? r[3] + r[1] : tid == 1 ? r[0] - r[1] - r[3] : tid == 2 ? r[1] : tid == 3 ? r[0]
                         : tid == 4 ? r[4] : tid == 5 ? r[5] : tid == 6 ? r[2] : tid == 7 ? r[6] : r[7];
        if (v) atomicAdd(&p.counters[(blockIdx.x % COPK_COUNTER_SHARDS) * 16 + tid], (unsigned long long)v);
    }
}

// One wave's counters (its own Counts, wave-uniform) added by nine of its
// lanes to shard `shard`: no cross-wave reduction, so no barrier.
__device__ __forceinline__ void counters_add_wave(const CopKParams &p, const Counts &t, int lane, uint32_t shard)
{
    if (lane < 9) {
        const uint32_t v = lane == 0 ? t.dropfw + t.notv4 : lane == 1 ? t.total - t.notv4 - t.dropfw
                         : lane == 2 ? t.notv4 : lane == 3 ? t.total : lane == 4 ? t.parse : lane == 5 ? t.noport
                         : lane == 6 ? t.fwd : lane == 7 ? t.rhit : t.rx;
        if (v) atomicAdd(&p.counters[(shard % COPK_COUNTER_SHARDS) * 16 + lane], (unsigned long long)v);
    }
}

// The segmented-list tile epilogue with the counters folded in (no optional
// features: COP_CFG_SEG_LISTS without per-rule bins or port statistics).
// Per (step, wave): ballot of FORWARD; the wave's verdict counters from
// ballots; one barrier; then each wave stages its packets' list entries at
// their segment positions, wave 0 writes the segment lengths, the records go
// out (mid) and nine lanes add the counters; a second barrier; the segments'
// 16-byte list stores. Two barriers per tile against four for the general
// path (compaction, counter reduction), and no shuffle reductions.
template <int FW, int PPT, bool WT, typename Mid>
__device__ __forceinline__ void seg_epilogue(const CopKParams &p, const CopKBatch &B, uint32_t base,
                                             const bool (&valid)[PPT], const uint32_t (&verdict)[PPT],
                                             const uint32_t (&flags)[PPT], const CompactLds &s, uint32_t *s_red,
                                             int tid, int lane, int wave, Mid mid)
{
    static_assert(COPK_SEG == BLOCK, "one segment per tile step");
    const Counts cw = wave_counts<FW, PPT>(valid, verdict, flags);
    unsigned long long bal[PPT];
#pragma unroll
    for (int k = 0; k < PPT; k++) bal[k] = __ballot(valid[k] && verdict[k] == COPK_FORWARD);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < PPT; k++) s.cnt[k * WAVES + wave] = (uint32_t)__popcll(bal[k]);
        const uint32_t c8[8] = {cw.total, cw.notv4, cw.fwd, cw.dropfw, cw.parse, cw.noport, cw.rhit, cw.rx};
#pragma unroll
        for (int q = 0; q < 8; q++) s_red[wave * 8 + q] = c8[q];
    }
    lds_barrier();
    if (B.fwd_idx) {
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            uint32_t off = 0;
#pragma unroll
            for (int w = 0; w < WAVES; w++) off += w < wave ? s.cnt[k * WAVES + w] : 0u;
            if ((bal[k] >> lane) & 1ull)
                s.stage[k * BLOCK + off +
                        __builtin_amdgcn_mbcnt_hi((uint32_t)(bal[k] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal[k], 0u))] =
                    base + k * BLOCK + tid;
        }
    }
    if (B.fwd_count && wave == 0 && lane < PPT && base + (uint32_t)lane * BLOCK < B.n) {
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < WAVES; w++) c += s.cnt[lane * WAVES + w];
        st_u32<WT>(c, B.fwd_count + base / COPK_SEG + (uint32_t)lane);
    }
    mid();
    counters_add(p, s_red, tid);
    lds_barrier();
    if (B.fwd_idx) {
        for (uint32_t q = (uint32_t)tid; q < (uint32_t)PPT * (BLOCK / 4); q += BLOCK) {
            const uint32_t k = q / (BLOCK / 4), cc = q % (BLOCK / 4);
            uint32_t c = 0;
#pragma unroll
            for (int w = 0; w < WAVES; w++) c += s.cnt[k * WAVES + w];
            if (cc * 4u < c) st_list_chunk<WT>(&s.stage[k * BLOCK + cc * 4u], B.fwd_idx, base + k * BLOCK + cc * 4u, B.n);
        }
    }
}

// Per-port coprocessor_stats (switch.h:33-38) of one tile, added to
// wave-uniform accumulators: rx = packets routed to the port's NF
// (enqueue_nf_rx), tx = packets it forwarded.
template <int PPT>
__device__ __forceinline__ void port_counts(uint32_t K, const bool (&valid)[PPT], const bool (&fwd)[PPT],
                                            const uint32_t (&port)[PPT], uint32_t (&prx)[COPK_MAX_DEMUX_PORTS],
                                            uint32_t (&ptx)[COPK_MAX_DEMUX_PORTS])
{
#pragma unroll
    for (int q = 0; q < COPK_MAX_DEMUX_PORTS; q++) {
        if ((uint32_t)q >= K) break;
#pragma unroll
        for (int k = 0; k < PPT; k++) {
            prx[q] += (uint32_t)__popcll(__ballot(valid[k] && port[k] == (uint32_t)q));
            ptx[q] += (uint32_t)__popcll(__ballot(fwd[k] && port[k] == (uint32_t)q));
        }
    }
}

// Workgroup counter flush: wave reduce -> LDS -> one atomic per counter per
// workgroup, into one of COPK_COUNTER_SHARDS shards (a 128-byte line each)
// so no single word serialises thousands of atomics; then the per-port
// counters the same way. s_red: WAVES*8 words, s_ps: WAVES*16 words.
// Split in two: flush_counters_lds (wave reduce into LDS) and, after a
// workgroup barrier, flush_counters_add (the sums and the atomics). The
// poll-mode kernel runs the second half after it has signalled the tile, so
// the tile's store drain never waits behind counter atomics.
__device__ __forceinline__ void flush_counters_lds(const Opt &o, const Counts &cn,
                                                   const uint32_t (&prx)[COPK_MAX_DEMUX_PORTS],
                                                   const uint32_t (&ptx)[COPK_MAX_DEMUX_PORTS], uint32_t *s_red,
                                                   uint32_t *s_ps, int lane, int wave)
{
    uint32_t c[8] = {cn.total, cn.notv4, cn.fwd, cn.dropfw, cn.parse, cn.noport, cn.rhit, cn.rx};
#pragma unroll
    for (int q = 0; q < 8; q++) {
        uint32_t v = c[q];
#pragma unroll
        for (int off = 32; off; off >>= 1) v += __shfl_xor(v, off);
        c[q] = v;
    }
    if (lane == 0 && wave < WAVES) {   // (a coordinator wave beyond the data waves adds nothing)
#pragma unroll
        for (int q = 0; q < 8; q++) s_red[wave * 8 + q] = c[q];
    }
    const uint32_t K = o.port_stats;
    if (K && lane == 0 && wave < WAVES) {
#pragma unroll
        for (int q = 0; q < COPK_MAX_DEMUX_PORTS; q++) {
            if ((uint32_t)q >= K) break;
            s_ps[wave * 16 + 2 * q] = prx[q];
            s_ps[wave * 16 + 2 * q + 1] = ptx[q];
        }
    }
}

__device__ __forceinline__ void flush_counters_add(const CopKParams &p, const Opt &o, const uint32_t *s_red,
                                                   const uint32_t *s_ps, int tid)
{
    const uint32_t K = o.port_stats;
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
        if (v && !(o.dbg & 1u))
            atomicAdd(&p.counters[(blockIdx.x % COPK_COUNTER_SHARDS) * 16 + tid], (unsigned long long)v);
    }
    if (K && tid < 2 * K) {
        uint32_t v = 0;
#pragma unroll
        for (int w = 0; w < WAVES; w++) v += s_ps[w * 16 + tid];
        if (v)
            atomicAdd(&p.port_ctr[(blockIdx.x % COPK_COUNTER_SHARDS) * COPK_PORT_WORDS + tid], (unsigned long long)v);
    }
}

__device__ __forceinline__ void flush_counters(const CopKParams &p, const Opt &o, const Counts &cn,
                                               const uint32_t (&prx)[COPK_MAX_DEMUX_PORTS],
                                               const uint32_t (&ptx)[COPK_MAX_DEMUX_PORTS], uint32_t *s_red,
                                               uint32_t *s_ps, int tid, int lane, int wave)
{
    flush_counters_lds(o, cn, prx, ptx, s_red, s_ps, lane, wave);
    lds_barrier();
    flush_counters_add(p, o, s_red, s_ps, tid);
}

}  // namespace copd

#endif
