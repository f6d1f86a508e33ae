// cop_pmd.hip — the coprocessor NF pipeline as a poll-mode (persistent)
// kernel: the GPU analogue of the reference's coprocessor lcores, which
// spin on their rx rings forever (main_loop -> coprocessor(),
// switch.c:529-535) instead of being started per burst.
//
// One launch serves a batch ring in HBM (cop_batch_ring) for as long as the
// host posts batches to it. The host posts by bumping a counter in mapped
// host memory (the doorbell); batch sequence b lives in ring slot
// b % n_slots. The grid is n_work worker workgroups, all co-resident:
//   - waiting workers poll a device copy of the doorbell; a few leaders
//     also read the host counter over PCIe and raise the copy (wait_posted);
//   - worker w processes the global tile sequence T = seq0*tpb + w, + n_work,
//     ... (tile j = T % tpb of batch b = T / tpb; tpb tiles per batch). The
//     assignment is static, so no ticket atomics: every tile a look-back
//     waits on belongs to a lower T, held by a resident worker that reaches
//     it first (no deadlock while all n_work workers are resident, which a
//     start-up census checks).
// A tile is the one-shot kernel's tile body (cop_tile.h) with write-through
// (sc1) output stores; after it every wave drains its stores, and one lane
// counts the tile for its slot; the slot's last tile writes the batch's
// sequence + 1 into the host-mapped completion word. With dense forward lists the look-back chain of slot s is tagged with
// the batch sequence, so chains of successive batches in one slot never mix;
// segmented lists (COP_CFG_SEG_LISTS) need no chain at all. Tables are
// staged into LDS once per worker.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "cop_device.h"
#include "cop_kernels.h"
#include "cop_tile.h"

namespace {

using namespace copd;

constexpr uint32_t CENSUS_SPINS = 1u << 21;   // ~0.2 s of s_sleep(2) for every worker to become resident

// diagnostic stamps: write-through, so a host copy sees them while the
// kernel still runs (no kernel-end L2 write-back)
__device__ __forceinline__ void st_stamp(unsigned long long *p, unsigned long long v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t ld_agent(uint32_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr unsigned long long GATE_POSTED = (1ull << COPK_PMD_GATE_SHIFT) - 1ull;
// experiment builds only: COPK_PMD_NOGATE=1 relays without publishing
// through the gate (timing of the gate's CAS on the doorbell path; exits may
// then leave batches half done)
#ifndef COPK_PMD_NOGATE
#define COPK_PMD_NOGATE 0
#endif

__device__ __forceinline__ unsigned long long ld_u64(const unsigned long long *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Publish posted count h through a ring's gate (doorbell leaders, before they
// raise the ring's relays): false once an exit has closed it. guess: the
// relay value the leader read in the same poll, usually the gate's value
// (relays copy the gate), so the first compare-exchange goes out without a
// load of the gate before it: one agent-scope round trip less between the
// doorbell and the relays (profiles/r05/check12/tail_*.log: relay -> seen
// 1.79 against 2.01 us, host post -> done 25.6 against 26.5 us). A wrong
// guess costs what the load did: the failed exchange returns the gate.
#ifndef COPK_PMD_GATE_GUESS
#define COPK_PMD_GATE_GUESS 1
#endif
__device__ __forceinline__ bool gate_publish(unsigned long long *gate, unsigned long long h, unsigned long long guess)
{
    unsigned long long g = COPK_PMD_GATE_GUESS ? guess : ld_u64(gate);
    for (;;) {
        if (g >> COPK_PMD_GATE_SHIFT) return false;
        if ((g & GATE_POSTED) >= h) return true;   // another leader published as much
        const unsigned long long seen = atomicCAS(gate, g, h);
        if (seen == g) return true;
        g = seen;
    }
}

// Leave: close every ring's gate (its posted count then bounds the batches
// of that ring served: every batch a worker may have started is finished
// before anyone leaves, so an idle or stop exit never leaves a batch half
// done), then claim the exit word (first reason wins; the gates are closed
// before it is set) and tell the host.
__device__ __forceinline__ void pmd_leave(const CopKPmd &P, uint32_t why)
{
    for (uint32_t r = 0; r < P.n_rings; r++) {
        unsigned long long *gate = P.d_gate + (size_t)r * 16;
        unsigned long long g = ld_u64(gate);
        while (!(g >> COPK_PMD_GATE_SHIFT)) {
            const unsigned long long seen = atomicCAS(gate, g, g | ((unsigned long long)why << COPK_PMD_GATE_SHIFT));
            if (seen == g) break;
            g = seen;
        }
    }
    if (atomicCAS(&P.d_ctl[0], 0u, why) == 0u)
        __hip_atomic_store(&P.h_state[0], why, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One lane of a worker of ring r (its wr-th) waits until the ring's batch b
// is posted (returns the posted count) or the kernel is to leave (returns
// 0). After an idle or stop exit batch b is still served when it lies below
// the closed gate's count (the returned count is then that bound). Doorbell
// leaders (every relay_stride-th worker of the ring) also read the ring's
// host counter over PCIe and raise the device copies every waiting worker
// polls: a handful of PCIe readers, not one per worker, and no workgroup
// slot spent on a doorbell. Leaders also turn the host's stop flag, a
// look-back timeout or an idle spell (no new post on any ring for
// idle_ticks) into the exit word.
__device__ __attribute__((unused)) unsigned long long wait_posted(const CopKPmd &P, uint32_t r, uint32_t wr,
                                                                  unsigned long long b, bool leader)
{
    // this worker's copy of the relay (one 128-byte line per group of the
    // ring's workers): a thousand pollers on one line would hammer one
    // memory channel while other workers stream
    unsigned long long *relay = P.d_posted + ((size_t)r * COPK_PMD_RELAYS + wr % COPK_PMD_RELAYS) * 16;
    unsigned long long *relays = P.d_posted + (size_t)r * COPK_PMD_RELAYS * 16;
    unsigned long long *gate = P.d_gate + (size_t)r * 16;
    const unsigned long long *h_posted = P.h_posted + (size_t)r * 8;
    unsigned long long seen = 0, t_seen = __builtin_amdgcn_s_memrealtime();
    for (uint32_t spins = 0;; spins++) {
        // every load of a poll is issued before any is used: one round trip
        // per poll, not one per load (a leader's PCIe read overlaps the rest)
        const unsigned long long hp = ld_u64(relay);
        const uint32_t ex = ld_agent(&P.d_ctl[0]);
        unsigned long long h = 0;
        uint32_t stop = 0;
        if (leader) {
            // the doorbell and the stop word in one PCIe round trip
            h = __hip_atomic_load(h_posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            stop = __hip_atomic_load(P.h_stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (hp > b) return hp;
        if (ex) {
            if (ex == COPK_PMD_ABORT) return 0;
            // idle or stop: the gate was closed before the exit word was set
            unsigned long long g;
            for (uint32_t k = 0; !((g = ld_u64(gate)) >> COPK_PMD_GATE_SHIFT) && k < (1u << 20); k++)
                __builtin_amdgcn_s_sleep(1);
            const unsigned long long lim = g & GATE_POSTED;
            return (g >> COPK_PMD_GATE_SHIFT) && b < lim ? lim : 0ull;
        }
        if (leader) {
            const unsigned long long now = __builtin_amdgcn_s_memrealtime();
            if (h > hp && (COPK_PMD_NOGATE || gate_publish(gate, h, hp))) {
                for (int x = 0; x < COPK_PMD_RELAYS; x++) atomicMax(relays + x * 16, h);
                if (P.stamps && r == 0) {   // diagnostic: when each doorbell value was relayed
                    st_stamp(&P.stamps[(size_t)P.n_work * 8 + (h % 64) * 2], h);
                    st_stamp(&P.stamps[(size_t)P.n_work * 8 + (h % 64) * 2 + 1], now);
                }
                if (h > b) return h;
            }
            if (h != seen) {
                seen = h;
                t_seen = now;
                if (P.n_rings > 1) atomicMax(P.d_act, now);   // activity on this ring keeps every ring's kernel up
            }
            // stop or pause at once (the host waits for them); a look-back
            // timeout and the idle clock every 16th poll
            if (stop) {
                pmd_leave(P, stop == 2u ? COPK_PMD_PAUSED : COPK_PMD_STOPPED);
            } else if ((spins & 15u) == 15u) {
                if (ld_agent(&P.d_ctl[2])) {
                    pmd_leave(P, COPK_PMD_ABORT);   // a look-back timed out
                } else {
                    unsigned long long last = t_seen;
                    if (P.n_rings > 1) last = max(last, ld_u64(P.d_act));
                    if (now - last > P.idle_ticks) pmd_leave(P, COPK_PMD_IDLE);
                }
            }
        } else {
            // back off to ~0.5 us between polls while nothing comes
            for (uint32_t k = spins < 16 ? 0u : P.poll_backoff; k; k--) __builtin_amdgcn_s_sleep(4);
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// Batch descriptor of ring rg's slot with n packets (pmd rings: ring mode)
__device__ __forceinline__ __attribute__((unused)) CopKBatch pmd_batch(const CopKParams &p, const CopKRing &rg, uint32_t slot, uint32_t n,
                                               uint32_t ntiles)
{
    CopKBatch B;
    B.pkts = rg.pkts + (size_t)slot * rg.pkts_slot_bytes;
    B.offsets = rg.offsets ? rg.offsets + (size_t)slot * rg.offsets_slot_words : nullptr;
    B.results = (uint2 *)rg.results + (size_t)slot * rg.results_slot;
    B.fwd_idx = rg.fwd_idx ? rg.fwd_idx + (size_t)slot * rg.fwd_slot : nullptr;
    // counts per slot: one, one per port (demux), or one per segment
    const uint32_t per = p.seg ? (rg.n + COPK_SEG - 1u) / COPK_SEG : p.demux ? p.demux : 1u;
    B.fwd_count = rg.fwd_count ? rg.fwd_count + (size_t)slot * per : nullptr;
    B.n = n;
    B.stride = rg.stride;
    B.data_off = rg.data_off;
    B.ntiles = ntiles;
    return B;
}

// experiment builds only: COPK_PMD_WT=0 stores non-temporally (timing of the
// write-through cost; results are then not guaranteed visible at completion)
#ifndef COPK_PMD_WT
#define COPK_PMD_WT 1
#endif
#ifndef COPK_PMD_RELEASE
#define COPK_PMD_RELEASE 0
#endif
// Workers per CU (waves per SIMD): 4 for 2048-packet tiles (<= 128 VGPRs),
// 5 for 1024-packet tiles (<= 96), 6 for 256-packet tiles (<= 80; the SGPR
// limit admits no more, MI355X_MICROARCH.md Residency)
#ifndef COPK_PMD_WPE4   // experiment builds: workers per CU of the 1024-packet-tile kernel
#define COPK_PMD_WPE4 5
#endif
#ifndef COPK_PMD_WAVES_PER_EU
#define COPK_PMD_WAVES_PER_EU(ppt) ((ppt) == 8 ? 4 : (ppt) == 4 ? COPK_PMD_WPE4 : 6)
#endif
template <int FW, int LPM, int LAY, int PPT, bool EXT>
__global__ __launch_bounds__(BLOCK, COPK_PMD_WAVES_PER_EU(PPT)) void cop_pmd(const CopKPmd P)
{
    const CopKParams &p = P.k;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const Opt o = EXT ? opt_all(p) : Opt{0u, 0u, 0u, nullptr};
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const LdsCarve lc = lds_carve<PPT>(p, lds);
    uint32_t *s_door = lc.s_misc + 36;   // [0..1] posted, [2] leave, [3] the batch's packets
    stage_tables<FW, LPM>(p, lc.tb, lane, wave);

    // census: every worker and the doorbell resident, or nobody works
    if (tid == 0) {
        atomicAdd(&P.d_ctl[1], 1u);
        uint32_t spins = 0;
        while (ld_agent(&P.d_ctl[1]) < P.n_work && ld_agent(&P.d_ctl[0]) == 0) {
            if (++spins > CENSUS_SPINS) {
                pmd_leave(P, COPK_PMD_ABORT);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        s_door[2] = ld_agent(&P.d_ctl[0]) == COPK_PMD_ABORT ? 1u : 0u;
    }
    __syncthreads();   // also lands the LDS-DMA table staging
    if (s_door[2]) return;
    if (blockIdx.x == 0 && tid == 0)   // tell the host every worker is resident
        __hip_atomic_store(&P.h_state[1], P.n_work, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);

    const uint32_t tpb = p.uniform_ntiles;
    const uint32_t n_slots = p.rg.n_slots;
    constexpr uint32_t TILE = BLOCK * PPT;
    // this worker's ring and its index among the ring's G workers
    const uint32_t R = P.n_rings;
    const uint32_t r = __builtin_amdgcn_readfirstlane(blockIdx.x % R);
    const uint32_t wr = blockIdx.x / R;
    const uint32_t G = (P.n_work - r + R - 1) / R;
    const CopKRing &rg = P.rings[r];
    const uint32_t rs0 = r * n_slots;   // ring r's first (slot-count, completion, n) word
    // The serving loop, in two forms (the choice is loop-invariant): tiles
    // step by step (tile_steps: segmented lists, records from lane pairs, no
    // optional feature), or tile_body. Two loops, so neither form's
    // registers are live through the other.
    auto serve = [&](auto steps_c) {
        constexpr bool STEPS = decltype(steps_c)::value;
        // tile (b, j, slot) of T = seq0r[r]*tpb + wr, advanced by G per step
        unsigned long long b = P.seq0r[r] + wr / tpb;
        uint32_t j = wr % tpb;
        uint32_t slot = (uint32_t)(b % n_slots);
        const uint32_t qb = G / tpb, rb = G % tpb;
        unsigned long long posted = 0;
        const bool leader = wr % P.relay_stride == 0;
        unsigned long long *stamp = P.stamps ? P.stamps + (size_t)blockIdx.x * 8 : nullptr;
        // the tile's completion, by one lane once every wave's stores
        // (write-through) and counter adds have landed: count it for its
        // slot; the slot's last tile writes the batch's sequence + 1 to host
        // memory. (One host-memory word per tile instead was measured: the
        // host saw a 20-batch post complete ~20 us after its last tile, 1280
        // PCIe writes against 20; profiles/r03/first/probe_seg.log.)
        auto count_tile = [&](uint32_t sl, unsigned long long bb) {
            const unsigned long long old = atomicAdd(&P.slot_tiles[(size_t)(rs0 + sl) * P.slot_stride], 1ull);
            const bool last_tile = (old + 1) % tpb == 0;
            if (last_tile) __hip_atomic_store(&P.h_done[rs0 + sl], bb + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (stamp) {
                st_stamp(&stamp[3], __builtin_amdgcn_s_memrealtime());   // stores drained, tile counted
                st_stamp(&stamp[5], last_tile ? 1ull : 0ull);
            }
        };
        // T += G
        auto advance = [&] {
            j += rb;
            uint32_t db = qb;
            if (j >= tpb) {
                j -= tpb;
                db++;
            }
            b += db;
            slot += db % n_slots;
            if (slot >= n_slots) slot -= n_slots;
        };
        for (;;) {
            if (stamp && tid == 0) st_stamp(&stamp[0], __builtin_amdgcn_s_memrealtime());   // diagnostic: tile start
            if (b >= posted) {
                // wait for batch b to be posted (one lane polls the relay)
                if (tid == 0) {
                    const unsigned long long hp = wait_posted(P, r, wr, b, leader);
                    s_door[0] = (uint32_t)hp;
                    s_door[1] = (uint32_t)(hp >> 32);
                    s_door[2] = hp == 0 ? 1u : 0u;
                }
                lds_barrier();
                posted = ((unsigned long long)s_door[1] << 32) | s_door[0];
                const uint32_t leave = s_door[2];
                lds_barrier();   // s_door is rewritten only after every wave has read it
                if (leave) break;
            }
            if (stamp && tid == 0) {
                st_stamp(&stamp[1], __builtin_amdgcn_s_memrealtime());   // batch b posted (as seen here)
                st_stamp(&stamp[4], b);
            }
            // the batch's packets: fixed (the ring's n), or the host's count for
            // the slot (written before the doorbell that posted the batch)
            uint32_t n = rg.n;
            if (P.h_n) {
                if (tid == 0)
                    s_door[3] = __hip_atomic_load(&P.h_n[rs0 + slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                lds_barrier();
                n = min(s_door[3], rg.n);
                lds_barrier();
            }
            const uint32_t ntiles = (n + TILE - 1) / TILE;
            // Slot reuse: another agent (the host, a copy engine, a NIC) may
            // have rewritten the slot since this CU (or its XCD's L2) last
            // read it, and a persistent kernel gets no dispatch-time cache
            // invalidation. So the tile reads the slot with system-coherent
            // loads (sc0 sc1: no cached copy is used; the doorbell read that
            // made the batch visible came first): mode 4, the default, from
            // the ring's second lap in this launch on (a slot's first read in
            // a launch follows the launch's own invalidation); mode 3 on every
            // tile (host-memory rings, COP_PMD_SYS_ACQUIRE); mode 0 never
            // (COP_PMD_STATIC_SLOTS). Modes 1 / 2 (A/B runs, $COP_PMD_ACQUIRE)
            // acquire at system scope instead, every tile / once wrapped: an
            // acquire invalidates the CU's and the XCD's caches for every
            // worker there, which halved the driver's 20-step rate
            // (profiles/r05/check2/acq*.log).
            const bool wrapped = b >= P.seq0r[r] + n_slots;
            const bool sysld = P.sys_acquire == 3u || (P.sys_acquire == 4u && wrapped);
            if (P.sys_acquire == 1u || (P.sys_acquire == 2u && wrapped)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            // The lane's index is made opaque each iteration, so the per-lane
            // values the tile derives from it (load geometry, LDS addresses) are
            // recomputed in the tile rather than hoisted out of the loop and held
            // live across it: loop-invariant code motion cost the persistent
            // kernel ~50 VGPRs over the one-shot kernel's tile.
            int tid_i = tid;
            asm volatile("" : "+v"(tid_i));
            const int lane_i = tid_i & 63;
            const int wave_i = __builtin_amdgcn_readfirstlane(tid_i >> 6);
            bool ok = true;
            if constexpr (STEPS) {
                // (a tile past a short batch's packets has nothing to do;
                // the load form is picked per tile: cop_tile.h steps_load)
                if (j < ntiles) {
                    const CopKBatch bt = pmd_batch(p, rg, slot, n, ntiles);
                    constexpr int WIN = LPM == COPK_TBL_DIR ? COPK_PMD_WIN_DIR : COPK_PMD_WIN;
                    if (sysld) tile_steps<FW, LPM, PPT, COPK_PMD_WT != 0, 1, WIN, LAY>(p, lc, bt, j, tid_i, lane_i, wave_i);
                    else tile_steps<FW, LPM, PPT, COPK_PMD_WT != 0, 0, WIN, LAY>(p, lc, bt, j, tid_i, lane_i, wave_i);
                }
            } else {
                if (P.test_skip && r == 0 && b == 0 && j + 1 == P.test_skip) {
                    ok = false;   // tests: this tile never runs nor publishes (its successors give up)
                } else if (j < ntiles) {
                    if (EXT && p.hit_region) {
                        // binned rule hits: the tile's bucket counts start at zero (the
                        // last tile's sort is done with them: the barrier below ordered it)
                        for (uint32_t i = (uint32_t)tid_i; i < p.hit_nb; i += BLOCK) lds[p.lds_hit_off + i] = 0u;
                        lds_barrier();
                    }
                    // (tests shorten the look-back's spin bound: the skipped
                    // tile's successors give up in well under a second)
                    const LookCtx lk{p.look, (uint32_t)(b + 1), &P.d_ctl[2], &P.d_ctl[0], P.test_skip ? 14u : 22u};
                    body_prio<COPK_PMD_WT != 0, 0>();
                    ok = tile_body<FW, LPM, LAY, PPT, EXT, COPK_PMD_WT != 0>(
                        p, o, lc, pmd_batch(p, rg, slot, n, ntiles), (rs0 + slot) * tpb, j, lk, tid_i, lane_i, wave_i,
                        false, (size_t)(rs0 + slot) * tpb + j, sysld);
                    body_prio<COPK_PMD_WT != 0, 3>();
                }
            }
            if (stamp && tid == 0) st_stamp(&stamp[2], __builtin_amdgcn_s_memrealtime());   // tile body done
            // completion (a tile whose look-back gave up, ok false, is not
            // counted: its batch never completes and the host sees the abort)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            lds_barrier();
            if (tid == 0 && ok) {
                // experiment builds (COPK_PMD_RELEASE with COPK_PMD_WT=0):
                // plain stores, then one agent-scope release per tile
                // (the XCD's L2 written back) before the count
                if (COPK_PMD_RELEASE) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                count_tile(slot, b);
            }
            advance();
        }
    };
    // Dynamic tiles (P.dyn, step-by-step tiles only: segmented lists need no
    // look-back, so any worker may take any tile and none ever waits on
    // another). A worker claims tiles from its ring's ticket counters: once
    // tile T's batch is posted and its loads are issued, it claims its next
    // tile Tn, and when Tn's batch is posted too, Tn's header loads go out
    // before T is classified and stored, so they are in flight during T's
    // work. Once T's stores, counter adds and those loads have drained (one
    // vmcnt(0)), T is counted for its slot;
    // that returning add is read one tile later (or before the worker waits
    // for a post), so no round trip stands between two tiles. Workers the
    // memory system serves first simply take more tiles: no static tail.
    // Exits: a worker leaves only when its claimed tile's batch is at or
    // above the closed gate's count; tickets are claimed in order, so every
    // tile of every batch below the gate was claimed by a worker that serves
    // it. A relaunch zeroes the tickets (ticket 0 = tile 0 of batch seq0r).
    constexpr bool DYN_OK = (PPT <= 2 || (COPK_PMD_WIN < PPT ? COPK_PMD_WIN : PPT) <= 2) && LAY == COPK_LAY_COALESCED;
    auto serve_dyn = [&](auto steps_c) {
        // (two tiles' loads live at once: 256- and 512-packet tiles, or
        // 1024-packet tiles with a window of at most two steps in flight,
        // COPK_PMD_WIN <= 2)
        constexpr bool STEPS = decltype(steps_c)::value && DYN_OK;
        if constexpr (STEPS) {
            constexpr int W = COPK_PMD_WIN < PPT ? COPK_PMD_WIN : PPT;
            // ticket lanes: one per XCD-sized group of the ring's workers
            // (worker wr claims from lane wr % nx; with one ring that is its
            // XCD, workgroups being dealt round-robin over the 8 XCDs), lane
            // x owning tiles j = x, x + nx, ... of every batch, so no one
            // counter takes every claim (one counter for all 1536 workers
            // held a 256-packet-tile kernel at ~80 claims per us)
            // P.dyn 2: the static order (T = wr, wr + G, ...: no tickets)
            // with the same next-tile prefetch
            const bool det = P.dyn == 2u;
            const uint32_t nx = (!det && P.tk_lanes > 1 && tpb % P.tk_lanes == 0) ? P.tk_lanes : 1u;
            const uint32_t xl = wr % nx;
            const uint32_t per = tpb / nx;   // tiles of one batch in one lane
            unsigned long long *ticket = P.d_ticket + ((size_t)r * COPK_PMD_TK_LANES + xl) * 16;
            uint32_t *s_tk = lc.s_misc + 72;   // the next claimed ticket (lo, hi)
            unsigned long long *stamp = P.stamps ? P.stamps + (size_t)blockIdx.x * 8 : nullptr;
            const bool leader = wr % P.relay_stride == 0;
            unsigned long long posted = 0;
            // lane 0 of wave 0: the pending slot count (issued after a tile's
            // stores drained, its return read one tile later)
            unsigned long long pend_old = 0, pend_b = 0;
            uint32_t pend_sl = 0;
            bool pend = false;
            auto pend_flush = [&] {
                if (pend && (pend_old + 1) % tpb == 0)
                    __hip_atomic_store(&P.h_done[rs0 + pend_sl], pend_b + 1, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
                pend = false;
            };
            auto claim = [&](unsigned long long cur) {
                return det ? cur + G : __hip_atomic_fetch_add(ticket, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            };
            auto tk_get = [&] { return ((unsigned long long)s_tk[1] << 32) | s_tk[0]; };
            // the first claim. A worker holds one unserved ticket while it
            // waits for a post and claims its next tile only once the
            // current one's batch is posted: holding two at the post would
            // give some workers two tiles of a 20-batch post and others none
            // (1024-packet tiles: 29 against 46 Gpkt/s at 20 steps,
            // profiles/r05/check5/)
            if (tid == 0) {
                const unsigned long long t0 = det ? (unsigned long long)wr : claim(0);
                s_tk[0] = (uint32_t)t0;
                s_tk[1] = (uint32_t)(t0 >> 32);
            }
            lds_barrier();
            unsigned long long T = tk_get();
            lds_barrier();
            // two load buffers used in turn (the loop body is instantiated
            // once per buffer order): a tile's loads land in the registers
            // its body reads, never in ones that must be copied (a copy of a
            // register with a load in flight waits for the load)
            u32x4 va[W][3], vb[W][3];
            bool loaded = false;   // the current buffer holds tile T's header loads
            uint32_t n = rg.n, ntiles = (rg.n + TILE - 1) / TILE;
            const unsigned long long seq0 = P.seq0r[r];
            // one tile: T's loads in cur (or issued here), Tn's into nxt;
            // returns true when the worker is to leave
            auto one = [&](u32x4 (&cur)[W][3], u32x4 (&nxt)[W][3]) -> bool {
                int tid_i = tid;
                asm volatile("" : "+v"(tid_i));
                const int lane_i = tid_i & 63;
                const int wave_i = __builtin_amdgcn_readfirstlane(tid_i >> 6);
                const unsigned long long b = seq0 + T / per;
                const uint32_t j = (uint32_t)(T % per) * nx + xl;
                const uint32_t slot = (uint32_t)(b % n_slots);
                if (stamp && tid == 0) {
                    st_stamp(&stamp[0], __builtin_amdgcn_s_memrealtime());   // diagnostic: tile start
                    st_stamp(&stamp[4], b);
                }
                if (!loaded) {
                    if (b >= posted) {
                        // nothing posted for this tile yet: report the pending
                        // count first (it may complete a batch), then wait
                        if (tid == 0) {
                            pend_flush();
                            const unsigned long long hp = wait_posted(P, r, wr, b, leader);
                            s_door[0] = (uint32_t)hp;
                            s_door[1] = (uint32_t)(hp >> 32);
                            s_door[2] = hp == 0 ? 1u : 0u;
                        }
                        lds_barrier();
                        posted = ((unsigned long long)s_door[1] << 32) | s_door[0];
                        const uint32_t leave = s_door[2];
                        lds_barrier();
                        if (leave) return true;
                    }
                    n = rg.n;
                    if (P.h_n) {
                        if (tid == 0)
                            s_door[3] = __hip_atomic_load(&P.h_n[rs0 + slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        lds_barrier();
                        n = min(s_door[3], rg.n);
                        lds_barrier();
                    }
                    ntiles = (n + TILE - 1) / TILE;
                    const bool wrapped = b >= seq0 + n_slots;
                    if (P.sys_acquire == 1u || (P.sys_acquire == 2u && wrapped))
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                    const bool sysld = P.sys_acquire == 3u || (P.sys_acquire == 4u && wrapped);
                    step_prio<0>();
                    if (j < ntiles)
                        steps_load<PPT, 0, W>(pmd_batch(p, rg, slot, n, ntiles), j, lane_i, wave_i, cur, sysld);
                }
                if (stamp && tid == 0) st_stamp(&stamp[1], __builtin_amdgcn_s_memrealtime());   // loads issued
                // T is posted: claim the next tile (its return lands after
                // T's loads, which this tile waits for anyway)
                if (tid == 0) {
                    const unsigned long long tn = claim(T);
                    s_tk[0] = (uint32_t)tn;
                    s_tk[1] = (uint32_t)(tn >> 32);
                }
                lds_barrier();
                const unsigned long long Tn = tk_get();
                // the next tile's loads, before this tile's work, when its
                // batch is known posted (fixed-size batches)
                const unsigned long long bn = seq0 + Tn / per;
                const uint32_t jn = (uint32_t)(Tn % per) * nx + xl;
                const uint32_t sn = (uint32_t)(bn % n_slots);
                const bool pf = bn < posted && !P.h_n;
                if (pf) {
                    const bool wrapped = bn >= seq0 + n_slots;
                    if (P.sys_acquire == 1u || (P.sys_acquire == 2u && wrapped))
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                    const bool sysld = P.sys_acquire == 3u || (P.sys_acquire == 4u && wrapped);
                    if (jn < ntiles)
                        steps_load<PPT, 0, W>(pmd_batch(p, rg, sn, rg.n, ntiles), jn, lane_i, wave_i, nxt, sysld);
                }
                if (j < ntiles) {
                    const bool sys_t = P.sys_acquire == 3u || (P.sys_acquire == 4u && b >= seq0 + n_slots);
                    tile_steps_v<FW, LPM, PPT, COPK_PMD_WT != 0>(p, lc, pmd_batch(p, rg, slot, n, ntiles), j, tid_i,
                                                                  lane_i, wave_i, cur, sys_t);
                }
                if (stamp && tid == 0) st_stamp(&stamp[2], __builtin_amdgcn_s_memrealtime());   // tile body done
                // this tile's stores and counter adds landed (and the next
                // tile's loads and the claim), then it is counted. The wait
                // is the builtin, not inline asm: the compiler's wait
                // insertion sees it, so it knows the claim's return (read by
                // one lane below) has landed on every path and puts no
                // vmcnt(0) after the next tile's loads
                asm volatile("" ::: "memory");
                __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0), expcnt/lgkmcnt untouched
                asm volatile("" ::: "memory");
                lds_barrier();
                if (tid == 0) {
                    pend_flush();
                    pend_old = atomicAdd(&P.slot_tiles[(size_t)(rs0 + slot) * P.slot_stride], 1ull);
                    pend_b = b;
                    pend_sl = slot;
                    pend = true;
                    if (stamp) st_stamp(&stamp[3], __builtin_amdgcn_s_memrealtime());   // counted
                }
                T = Tn;
                loaded = pf;
                return false;
            };
            for (;;) {
                if (one(va, vb)) break;
                if (one(vb, va)) break;
            }
            // leaving: the pending count was reported before the last wait
        }
    };
    if (steps_ok<FW, LPM, LAY, EXT>() && p.seg && p.compact && p.rec_paired && P.stepwise) {
        if (DYN_OK && P.dyn) serve_dyn(std::integral_constant<bool, steps_ok<FW, LPM, LAY, EXT>()>{});
        else serve(std::integral_constant<bool, steps_ok<FW, LPM, LAY, EXT>()>{});
    } else {
        serve(std::integral_constant<bool, false>{});
    }
}

template <int FW, int LPM, int LAY, int PPT>
hipError_t pmd_one(const CopKPmd *p, int ext, uint32_t lds, hipStream_t s, int *occ)
{
    if (occ) {
        if (ext) return hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, cop_pmd<FW, LPM, LAY, PPT, true>, BLOCK, lds);
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, cop_pmd<FW, LPM, LAY, PPT, false>, BLOCK, lds);
    }
    const dim3 grid(p->n_work);
    if (ext) hipLaunchKernelGGL((cop_pmd<FW, LPM, LAY, PPT, true>), grid, dim3(BLOCK), lds, s, *p);
    else hipLaunchKernelGGL((cop_pmd<FW, LPM, LAY, PPT, false>), grid, dim3(BLOCK), lds, s, *p);
    return hipGetLastError();
}

template <int FW, int LPM, int LAY>
hipError_t pmd_ppt(const CopKPmd *p, int ppt, int ext, uint32_t lds, hipStream_t s, int *occ)
{
    if (ppt == 8) return pmd_one<FW, LPM, LAY, 8>(p, ext, lds, s, occ);
    if (ppt == 4) return pmd_one<FW, LPM, LAY, 4>(p, ext, lds, s, occ);
    return pmd_one<FW, LPM, LAY, 1>(p, ext, lds, s, occ);
}

template <int FW, int LPM>
hipError_t pmd_lay(const CopKPmd *p, int lay, int ppt, int ext, uint32_t lds, hipStream_t s, int *occ)
{
    if (lay == COPK_LAY_IMIX) return pmd_ppt<FW, LPM, COPK_LAY_IMIX>(p, ppt, ext, lds, s, occ);
    if (lay == COPK_LAY_COALESCED) return pmd_ppt<FW, LPM, COPK_LAY_COALESCED>(p, ppt, ext, lds, s, occ);
    if (lay == COPK_LAY_HDR16) return pmd_ppt<FW, LPM, COPK_LAY_HDR16>(p, ppt, ext, lds, s, occ);
    return pmd_ppt<FW, LPM, COPK_LAY_SLOTS>(p, ppt, ext, lds, s, occ);
}

template <int FW>
hipError_t pmd_lpm(const CopKPmd *p, int lpm, int lay, int ppt, int ext, uint32_t lds, hipStream_t s, int *occ)
{
#ifdef COPK_ISA_PROBE   // ISA inspection builds only: one instantiation (tools/isa.sh)
#ifndef COPK_ISA_LPM
#define COPK_ISA_LPM COPK_TBL_OFF
#endif
    return pmd_one<FW, COPK_ISA_LPM, COPK_LAY_COALESCED, COPK_ISA_PROBE>(p, ext, lds, s, occ);
#else
    if constexpr (FW == COPK_TBL_BKT) {   // as cop_kernels.hip launch_lpm
        if (lpm == COPK_TBL_DIR) return pmd_lay<FW, COPK_TBL_DIR>(p, lay, ppt, ext, lds, s, occ);
        if (lpm == COPK_TBL_BKT) return pmd_lay<FW, COPK_TBL_BKT>(p, lay, ppt, ext, lds, s, occ);
        if (lpm == COPK_TBL_OFF) return pmd_lay<FW, COPK_TBL_OFF>(p, lay, ppt, ext, lds, s, occ);
        return hipErrorInvalidValue;   // fill_launch maps IVT / TRIE routes to DIR-24-8 here
    } else {
        if (lpm == COPK_TBL_IVT) return pmd_lay<FW, COPK_TBL_IVT>(p, lay, ppt, ext, lds, s, occ);
        if (lpm == COPK_TBL_DIR) return pmd_lay<FW, COPK_TBL_DIR>(p, lay, ppt, ext, lds, s, occ);
        if (lpm == COPK_TBL_TRIE) return pmd_lay<FW, COPK_TBL_TRIE>(p, lay, ppt, ext, lds, s, occ);
        if (lpm == COPK_TBL_BKT) return pmd_lay<FW, COPK_TBL_BKT>(p, lay, ppt, ext, lds, s, occ);
        return pmd_lay<FW, COPK_TBL_OFF>(p, lay, ppt, ext, lds, s, occ);
    }
#endif
}

}  // namespace

// compiled in three parts, one per firewall table mode (as cop_kernels.hip)
#define COPK_PMD_ARGS const CopKPmd *p, int lpm, int lay, int ppt, int ext, uint32_t lds, hipStream_t s, int *occ
extern "C" hipError_t copk_pmd_fw0(COPK_PMD_ARGS);
extern "C" hipError_t copk_pmd_fw1(COPK_PMD_ARGS);
extern "C" hipError_t copk_pmd_fw2(COPK_PMD_ARGS);
extern "C" hipError_t copk_pmd_fw4(COPK_PMD_ARGS);
#if defined(COPK_FW_PART)
#define COPK_CAT2(a, b) a##b
#define COPK_CAT(a, b) COPK_CAT2(a, b)
extern "C" hipError_t COPK_CAT(copk_pmd_fw, COPK_FW_PART)(COPK_PMD_ARGS)
{
    return pmd_lpm<COPK_FW_PART>(p, lpm, lay, ppt, ext, lds, s, occ);
}
#else
static hipError_t pmd_dispatch(const CopKPmd *p, int fw, int lpm, int lay, int ppt, int ext, uint32_t lds,
                               hipStream_t s, int *occ)
{
    if (fw == COPK_TBL_IVT) return copk_pmd_fw1(p, lpm, lay, ppt, ext, lds, s, occ);
    if (fw == COPK_TBL_DIR) return copk_pmd_fw2(p, lpm, lay, ppt, ext, lds, s, occ);
    if (fw == COPK_TBL_BKT) return copk_pmd_fw4(p, lpm, lay, ppt, ext, lds, s, occ);
    return copk_pmd_fw0(p, lpm, lay, ppt, ext, lds, s, occ);
}

extern "C" hipError_t copk_pmd_launch(const CopKPmd *p, int fw_mode, int lpm_mode, int layout, int ppt, int ext,
                                      uint32_t lds_bytes, hipStream_t stream)
{
    return pmd_dispatch(p, fw_mode, lpm_mode, layout, ppt, ext, lds_bytes, stream, nullptr);
}

extern "C" hipError_t copk_pmd_occupancy(int fw_mode, int lpm_mode, int layout, int ppt, int ext, uint32_t lds_bytes,
                                         int *per_cu)
{
    *per_cu = 0;
    return pmd_dispatch(nullptr, fw_mode, lpm_mode, layout, ppt, ext, lds_bytes, nullptr, per_cu);
}
#endif  // COPK_FW_PART
