// cop_kernels.h — launch parameters shared by the HIP runtime and the
// pipeline kernel. Internal (not part of the C ABI).
#ifndef COP_KERNELS_H
#define COP_KERNELS_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#define COPK_BLOCK 256
#define COPK_MAXB 32
#define COPK_MAX_LAUNCH_BATCHES 1024   /* ring launches; ticket lines per lane buffer */
#define COPK_COUNTER_SHARDS 256  /* 16 u64 per shard (128 B) */
static_assert(sizeof(void *) == 8, "64-bit only");
#define COPK_LDS_MISC_WORDS 80       /* counts, tile, prefix, counter reduction */
#define COPK_LDS_MISC_EXT_WORDS 408  /* + per-port counts/prefixes (demux, port stats) */
#define COPK_COALESCED_MIN_STRIDE 48 /* coalesced loads move the first 48 bytes of every slot */
#define COPK_MAX_DEMUX_PORTS 8
#define COPK_PORT_WORDS 16           /* per shard: 8 ports x {rx, tx} */
#define COPK_STAMP_WG 65536

#define COPK_TBL_OFF 0
#define COPK_TBL_IVT 1  /* flattened intervals, binary search in LDS */
#define COPK_TBL_DIR 2  /* DIR-24-8 image in HBM */
#define COPK_TBL_TRIE 3 /* multibit trie: 12-bit top level in LDS, 6-bit popcount nodes in L2 (route stage) */
#define COPK_TBL_BKT 4  /* bucketed intervals in global memory (L2): first candidate per top-ib-bit bucket,
                           then (start, value) pairs (route stage; firewall stage with COP_CFG_FW_BKT) */
#define COPK_TRIE_L0 4096u
/* Packed tbl8 form of a DIR-24-8 image: an extended tbl24 entry's payload is
 * the offset (in 64-byte units) of its /24's run block instead of a group
 * index. A block describes the group's 256 entries as runs of equal
 * entries: 8 u64 header words h[w] = (runs starting before entry 32w) << 32
 * | bitmap of the run starts among entries 32w..32w+31, then the runs'
 * entries (u32). Entry i = value[prefix(w) + popcount(bits 0..i%32) - 1],
 * w = i/32. Blocks are 64-byte aligned: 64 + 4*runs bytes, rounded up. */

#define COPK_LAY_SLOTS 0      /* packet layouts of the one-shot kernel */
#define COPK_LAY_IMIX 1
#define COPK_LAY_COALESCED 2
#define COPK_LAY_HDR16 3      /* packed 16-byte header records (COP_HDR16_STRIDE) */

#define COPK_STAGE_PARSE 0x1u

#define COPK_FORWARD 0u
#define COPK_DROP_FW 1u
#define COPK_DROP_PARSE 2u
#define COPK_DROP_NOT_IPV4 3u
#define COPK_DROP_NO_PORT 4u
#define COPK_FLAG_ROUTE_HIT 0x1u
#define COPK_FLAG_FW_HIT 0x2u

struct CopKBatch {
    const uint8_t *pkts;
    const uint32_t *offsets;
    void *results;            // uint2 per packet
    uint32_t *fwd_idx;
    uint32_t *fwd_count;
    uint32_t n;
    uint32_t stride;
    uint32_t data_off;
    uint32_t ntiles;
};

struct CopKRing {
    const uint8_t *pkts;
    const uint32_t *offsets;
    void *results;
    uint32_t *fwd_idx;
    uint32_t *fwd_count;
    unsigned long long pkts_slot_bytes, offsets_slot_words, results_slot, fwd_slot;
    uint32_t n_slots, first, n, stride, data_off;
};

struct CopKParams {
    CopKBatch b[COPK_MAXB];                  // descriptor mode (ring == 0)
    uint32_t tile_begin[COPK_MAXB];          // first blockIdx of each batch
    uint32_t look_begin[COPK_MAXB];          // look-back word offset of each batch
    CopKRing rg;                             // ring mode (ring == 1): batch b = slot first+b
    uint32_t ring;
    uint32_t nb;
    uint32_t ntiles;
    uint32_t uniform_ntiles;  // tiles per batch when all batches are equal, else 0
    uint32_t stages;
    uint32_t n_ports;
    uint32_t compact;
    // forward lists in segments of COPK_SEG packets (COP_CFG_SEG_LISTS):
    // segment k's forward indices at fwd_idx[k*COPK_SEG ..), its length at
    // fwd_count[k]; no cross-tile prefix, so no tickets and no look-back
    uint32_t seg;
    uint32_t static_order;    // tile j of a batch = its blockIdx order (small launches: no ticket atomics)
    uint32_t epoch;
    uint32_t dbg;             // timing-only ablations ($COP_DBG), 0 in production
    // vport routing table (two-level image)
    const uint32_t *rt_top;   // 256 entries: value, or 0x80000000|leaf
    const uint16_t *rt_leaf;  // nleaf * 256
    uint32_t rt_nleaf;
    // firewall LPM. Interval form in LDS: fw_starts = fw_m sorted starts,
    // then fw_iw words of bucket index (2^fw_ib + 1 u16); fw_lv levels of
    // binary lifting inside a bucket (cop_runtime.cpp upload_lpm)
    uint32_t fw_m, fw_ib, fw_lv, fw_iw;
    const uint32_t *fw_starts, *fw_vals;
    const uint32_t *fw_tbl24, *fw_tbl8;
    uint32_t fw_tbl8_packed;  // tbl8 groups as packed run blocks (COPK_TBL8_PACKED form)
    // route LPM (the same forms)
    uint32_t lpm_m, lpm_ib, lpm_lv, lpm_iw;
    const uint32_t *lpm_starts, *lpm_vals;
    const uint32_t *lpm_tbl24, *lpm_tbl8;
    uint32_t lpm_tbl8_packed;
    uint32_t probe_nt;           // tbl24 probes as non-temporal loads (experiment, $COP_PROBE_NT)
    const uint32_t *lpm_tl0;     // trie form (lpm_trie.c): 4096 top entries (staged in LDS)
    const uint32_t *lpm_tnodes;  // 6 u32 per node: vec, leafvec (u64 each), child_base, leaf_base
    const uint32_t *lpm_tleaves;
    // bucketed form (COPK_TBL_BKT): lpm_bidx[b] = the last interval k with
    // start <= b << (32 - lpm_ib), b in [0, 2^lpm_ib] (the last entry: m - 1);
    // lpm_bpairs[2k] = start k, [2k + 1] = its value (padded with COP_BKT_PADS = 8
    // {0xFFFFFFFF, last value} pairs); lpm_lv lifting levels above the
    // widest bucket
    const uint32_t *lpm_bidx, *lpm_bpairs;
    // the firewall table in the same bucketed form (COPK_TBL_BKT firewall,
    // COP_CFG_FW_BKT: 1M-rule tables; fw_ib its index bits)
    const uint32_t *fw_bidx, *fw_bpairs;
    // LDS carve (u32 words)
    uint32_t lds_fw_off, lds_lpm_off, lds_misc_off;
    uint32_t lds_stage_off;   // one-shot kernel: the tile's forward list staged in LDS (0: none)
    uint32_t lds_rec_off;     // poll-mode kernel: the tile's records staged in LDS (0: none)
    uint32_t rec_paired;      // poll-mode kernel: records as 16-byte stores from lane pairs, no LDS stage
    // ordering / accounting state
    unsigned long long *tickets;   // one counter per batch, one 128-byte line each (zero at launch)
    unsigned long long *zero_tickets;  // the lane's other ticket buffer: zeroed by this launch
    uint32_t zero_lines;               // its dirty lines
    unsigned long long *look;
    unsigned long long *counters;
    unsigned long long *rule_hits;     // per-rule FW hit counters or nullptr
    unsigned long long *port_ctr;      // per-port {rx, tx} shards (port_stats)
    uint32_t demux;                    // > 0: one ordered forward list per port (count = ports)
    uint32_t port_stats;               // > 0: per-port counters for ports < port_stats
    uint32_t *err;
    unsigned long long *stamps;   // diagnostic phase stamps (dbg bit 8)
    // per-rule hit counters by binning (one-shot launches): each tile sorts
    // its FW hits' rule ids by bucket (id >> COPK_HIT_SHIFT) in LDS and
    // writes them to its region (runs padded to 4 ids with ~0u) plus the run
    // offsets; cop_hit_count then counts bucket by bucket in LDS and adds
    // the sums to rule_hits. hit_region == nullptr: one atomic per hit.
    uint32_t *hit_region;     // [tile][hit_reg_words]
    uint32_t *hit_off;        // [tile][hit_nb + 1]: run start of each bucket, then the end
    uint32_t hit_nb;          // buckets (<= COPK_HIT_MAX_BUCKETS)
    uint32_t hit_reg_words;   // tile * PPT*BLOCK + 4 * hit_nb
    uint32_t lds_hit_off;     // LDS: cnt[nb] | cur[nb] | wsum[4] | off[nb+1] (padded to 4) | tmp[tile] | ids[hit_reg_words]
};
#define COPK_HIT_SHIFT 14            /* 16384 rules per bucket: the count kernel's LDS counters (64 KiB) */
#define COPK_HIT_MAX_BUCKETS 256     /* 4M rules */
#define COPK_SEG 256                 /* packets per forward-list segment (= COPK_BLOCK: one tile step) */

// Poll-mode (persistent) kernel, cop_pmd.hip: n_work worker workgroups
// serve n_rings batch rings (worker w serves ring w % n_rings); every
// relay_stride-th worker of a ring relays that ring's doorbell.
#define COPK_PMD_MAX_RINGS 8
struct CopKPmd {
    CopKParams k;                        // ring mode (k.rg = ring 0, rg.first = 0), tables, counters,
                                         // options; k.uniform_ntiles = tiles per batch
    // ring r (all rings: k.rg's geometry: n, n_slots, stride, layout); each
    // ring has its own batch sequence, doorbell, gate, relays, slot counts
    // and completion words (per-ring arrays below, ring-major)
    CopKRing rings[COPK_PMD_MAX_RINGS];
    unsigned long long seq0r[COPK_PMD_MAX_RINGS];   // first batch of ring r this launch serves
    uint32_t n_rings;
    // host-mapped [r * n_slots + slot]: the packets of the batch in that
    // slot (variable-size batches, cop_pmd_post_batch), or null (every batch
    // has k.rg.n packets)
    const uint32_t *h_n;
    unsigned long long *d_act;           // device: s_memrealtime of the last doorbell change of any ring
    const unsigned long long *h_posted;  // host-mapped: batches posted (monotonic), ring r's at [8 r]
    const uint32_t *h_stop;              // host-mapped: 1 = stop, 2 = pause (leave, to be relaunched)
    // host-mapped completion: [r * n_slots + slot] = sequence + 1 of its
    // last completed batch, written by the slot's last tile (every output
    // byte of the batch, and its counter adds, landed before)
    unsigned long long *h_done;
    uint32_t *h_state;                   // host-mapped: [0] exit reason (COPK_PMD_*), [1] census
    unsigned long long *d_posted;        // device relays of ring r's posted count: COPK_PMD_RELAYS copies,
                                         // 128 B apart, ring r's at [16 (r * COPK_PMD_RELAYS + x)]
    // device: the gate, {exit reason:8 | posted:56}. Leaders publish a posted
    // count through it (CAS) before raising the relays; an exit closes it. Its
    // count then bounds the batches this launch serves: every worker finishes
    // every batch below it before leaving, none above it is started. Ring
    // r's gate at [16 r]
    unsigned long long *d_gate;
    uint32_t *d_ctl;                     // device: [0] exit (COPK_PMD_*), [1] census, [2] look-back timeout
    unsigned long long *slot_tiles;      // per (ring, slot): tiles completed (multiples of tiles per batch
                                         // between batches; zeroed at every launch), slot_stride u64 apart
    uint32_t slot_stride;                // 520 (4160 B): every counter on its own line, lines spread over
                                         // channels (packed counters cost a 20-batch burst ~3 us: tools/burst)
    unsigned long long *stamps;          // diagnostic: s_memrealtime per worker phase (COP_PMD_STAMPS) or null
    unsigned long long idle_ticks;       // s_memrealtime ticks (100 MHz) without a post before leaving
    uint32_t n_work;                     // worker workgroups
    uint32_t relay_stride;               // every relay_stride-th worker also reads the host doorbell
    uint32_t stepwise;                   // tiles step by step where tile_steps applies ($COP_PMD_STEPWISE=0: off)
    uint32_t sys_acquire;                // slot reuse: 0 plain loads (static slots); system-coherent packet
                                         // loads on every tile (3: host-memory rings) or once the ring wraps in
                                         // this launch (4: the default); A/B only: a system-scope acquire before
                                         // the loads instead, every tile (1) / once wrapped (2)
    uint32_t test_skip;                  // tests: tile test_skip - 1 of ring 0's batch 0 never runs ($COP_PMD_TEST_SKIP_TILE)
    uint32_t poll_backoff;               // waiting workers' s_sleep(4) rounds between relay polls once idle
                                         // (3: ~0.3 us, the default; 0: busy polling, $COP_PMD_BACKOFF)
    // dynamic tiles (segmented lists, step-by-step tiles): the ring's tiles
    // are claimed from a ticket counter, tile T = seq0r[r] * tiles per batch
    // + the T-th claim, instead of the static T = w + k * workers; a worker
    // claims its next tile and issues that tile's header loads before it
    // finishes the current one ($COP_PMD_DYN); 2: the same prefetch in the
    // static order, no tickets ($COP_PMD_PF)
    uint32_t dyn;
    uint32_t tk_lanes;                   // ticket lanes per ring (1, or 8: one per XCD-sized worker group)
    unsigned long long *d_ticket;        // device: ring r's lane x claim counter at [16 (r * COPK_PMD_TK_LANES + x)]
                                         // (zeroed at every launch)
};
#define COPK_PMD_TK_LANES 8
#define COPK_PMD_RELAYS 8
#define COPK_PMD_GATE_SHIFT 56
#define COPK_PMD_RUNNING 0u
#define COPK_PMD_STOPPED 1u   /* the host asked (cop_pmd_stop) */
#define COPK_PMD_IDLE 2u      /* no post for idle_ticks: left; the next post relaunches */
#define COPK_PMD_ABORT 3u     /* not every worker became resident, or a look-back timed out */
#define COPK_PMD_PAUSED 4u    /* the host asked it to make room for other kernels; relaunched after */

#ifdef __cplusplus
extern "C" {
#endif
hipError_t copk_pmd_launch(const CopKPmd *p, int fw_mode, int lpm_mode, int layout, int ppt, int ext,
                           uint32_t lds_bytes, hipStream_t stream);
// resident workgroups per CU of that kernel at lds_bytes (the occupancy API)
hipError_t copk_pmd_occupancy(int fw_mode, int lpm_mode, int layout, int ppt, int ext, uint32_t lds_bytes,
                              int *per_cu);
// layout: COPK_LAY_*
hipError_t copk_launch(const CopKParams *p, int fw_mode, int lpm_mode, int layout, int ppt,
                       uint32_t grid, uint32_t lds_bytes, hipStream_t stream);
// per-rule hit counters from the binned ids of n_tiles tiles (see hit_region)
hipError_t copk_hit_count(const CopKParams *p, uint32_t n_tiles, uint32_t tile_pkts, hipStream_t stream);
// dst[i] = src[i] (atomic load) or atomic exchange with 0 when reset
hipError_t copk_snapshot(unsigned long long *src, uint32_t n_words, unsigned long long *dst, int reset,
                         hipStream_t stream);
#ifdef __cplusplus
}
#endif

#endif
