/*
 * cop_gpu.h — C-ABI boundary of the MI355X coprocessor NF pipeline.
 *
 * This is the drop-in boundary for the per-packet coprocessor path of
 * google/ghost-dataplane (reference, read-only at /root/reference):
 *
 *   engine/switch.c:443-474   coprocessor()        burst loop, forward/free
 *   engine/coprocessor.c:21-65 coprocessor_setup / coprocessor_teardown /
 *                              process_packet       (declared coprocessor.h:23-30)
 *   engine/nfs/firewall/firewall.c:170-213 fw_packet_handler
 *   engine/nfs/firewall/firewall.c:215-255 lpm_setup (rte_lpm_create/add)
 *   engine/nfs/firewall/firewall.c:276-323 setup_rules (rules.json loader)
 *   engine/switch.c:93-136    get_next_hop (parse + vport route)
 *   engine/init.c:40-84       read_config (routing table defaults)
 *
 * Everything here is plain C: pointers, sizes, negative-errno return codes.
 * No torch, no CUDA-compat headers; HIP is called only inside libcopgpu.so.
 */
#ifndef COP_GPU_H
#define COP_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------ */
/* Constants mirrored from the reference                                    */
/* ------------------------------------------------------------------------ */

#define COP_UNKNOWN_PORT      0xFFFFu   /* UNKNOWN_PORT       init.h:28 */
#define COP_ROUTING_TBL_SZ    0x10000u  /* ROUTING_TBL_SZ     init.h:29 */
#define COP_PKT_BURST_SZ      32u       /* PKT_BURST_SZ       init.h:47 */
#define COP_KNI_KTHREAD       5u        /* KNI_KTHREAD        init.h:52 */
#define COP_NF_QUEUE_RINGSIZE 16384u    /* NF_QUEUE_RINGSIZE  init.h:54 */
#define COP_ETHER_TYPE_IPV4   0x0800u   /* ETHER_TYPE_IPv4    switch.c:118 */
#define COP_FW_MAX_RULES      1024u     /* conf.max_rules     firewall.c:234 */
#define COP_FW_NUMBER_TBL8S   24u       /* conf.number_tbl8s  firewall.c:235 */
#define COP_LPM_MAX_DEPTH     32u       /* RTE_LPM_MAX_DEPTH  (DPDK rte_lpm.h) */
#define COP_LPM_NH_MASK       0x00FFFFFFu /* 24-bit next hop  (DPDK v1604 ABI) */

/* Stage flags. The reference selects stages at compile time with
 * ENABLE_FW_NF / DISABLE_NF (coprocessor.h:19-21, switch.c:411,426,524);
 * the same macro names select COP_DEFAULT_STAGES here, and cop_config.stages
 * carries the mask to the device at run time. */
#define COP_STAGE_PARSE 0x1u  /* get_next_hop switch.c:93-136            */
#define COP_STAGE_FW    0x2u  /* fw_packet_handler firewall.c:170-213    */
#define COP_STAGE_LPM   0x4u  /* route LPM on dst (north-star extension) */

#if defined(DISABLE_NF)
#define COP_DEFAULT_STAGES (COP_STAGE_PARSE)
#elif defined(ENABLE_FW_NF)
#define COP_DEFAULT_STAGES (COP_STAGE_PARSE | COP_STAGE_FW)
#else
#define COP_DEFAULT_STAGES (COP_STAGE_PARSE | COP_STAGE_FW)
#endif

/* Stages of the drop-in coprocessor API (process_packet, process_burst,
 * cop_coprocessor_poll*): the coprocessor thread's NF chain only. Parse and
 * vport routing (get_next_hop, the UNKNOWN_PORT drop) are the fast path's
 * job before a packet is enqueued to the coprocessor (switch.c:406-415), so
 * the drop-in never drops on them: an IPv4 packet whose dst&0xFFFF is in
 * 0..4, or an IPv6 EtherType, gets the firewall's verdict. The batch API
 * (cop_submit*, cop_process_host*) runs cop_config.stages.
 *   - process_packet runs fw_packet_handler under ENABLE_FW_NF
 *     (coprocessor.c:59-62), which the reference's coprocessor.h:21 always
 *     defines: COP_STAGE_FW, also when neither macro is defined.
 *   - DISABLE_NF (coprocessor.h:19): switch.c never calls the coprocessor
 *     (switch.c:411,426,524); if it is called anyway, every packet forwards
 *     (no NF stage), as process_packet does without ENABLE_FW_NF
 *     (coprocessor.c:59-64). Define COP_DROPIN_NO_NF for that chain alone.
 * The library is built once, so the caller's macros reach it through
 * coprocessor_setup, which this header makes an alias of
 * cop_coprocessor_setup_fw or cop_coprocessor_setup_no_nf in the caller's
 * build (cop_set_dropin_stages sets the same at run time, e.g. from an FFI). */
#if defined(DISABLE_NF) || defined(COP_DROPIN_NO_NF)
#define COP_DROPIN_STAGES 0u
#else
#define COP_DROPIN_STAGES (COP_STAGE_FW)
#endif

/* Per-packet verdicts (one byte of the result record).
 *   FORWARD/DROP_FW : enum FW_ACTION firewall.h:71-74 (FW_FORWARD=0, FW_DROP=1)
 *   DROP_PARSE      : get_next_hop() == UNKNOWN_PORT, freed by the fast path
 *                     (switch.c:406-410); never reaches the coprocessor
 *   DROP_NOT_IPV4   : version nibble != 4. The reference counts it
 *                     (firewall.c:186-190) and then dereferences NULL at
 *                     firewall.c:193-194 (undefined behaviour); this build
 *                     defines the outcome as a drop.
 *   DROP_NO_PORT    : port >= number of active vports; the reference's
 *                     enqueue_nf_rx silently discards it (switch.c:316-319). */
enum cop_verdict {
    COP_FORWARD       = 0,
    COP_DROP_FW       = 1,
    COP_DROP_PARSE    = 2,
    COP_DROP_NOT_IPV4 = 3,
    COP_DROP_NO_PORT  = 4
};

#define COP_FLAG_ROUTE_HIT 0x1u /* route LPM lookup hit (rte_lpm_lookup ret == 0) */
#define COP_FLAG_FW_HIT    0x2u /* firewall LPM lookup hit                         */

/* 8-byte per-packet result record (SURVEY.md §8a "bit-exact contract"). */
typedef struct cop_result {
    uint8_t  verdict;   /* enum cop_verdict */
    uint8_t  flags;     /* COP_FLAG_* */
    uint16_t port;      /* vport from the routing table, or COP_UNKNOWN_PORT */
    uint32_t route_nh;  /* 24-bit next hop of the route LPM stage (0 on miss) */
} cop_result;

/* One prefix rule: struct fw_rule firewall.h:49-53 ({src_ip, depth, action})
 * generalised to a 24-bit next hop so the same type carries route prefixes. */
typedef struct cop_prefix {
    uint32_t ip;        /* host byte order, unmasked (rte_lpm_add masks it) */
    uint32_t next_hop;  /* FW: action (uint8 in the reference); routes: 24-bit */
    uint8_t  depth;     /* 1..32 accepted; anything else is -EINVAL */
    uint8_t  _pad[3];
} cop_prefix;

/* rte_lpm_config as used by lpm_setup (firewall.c:229-235). */
typedef struct cop_lpm_config {
    uint32_t max_rules;     /* distinct (prefix, depth) rules; default 1024 */
    uint32_t number_tbl8s;  /* tbl8 groups (/24s holding a depth>24 prefix); default 24 */
    uint32_t flags;         /* COP_LPM_* */
} cop_lpm_config;

/* Reproduce lpm_setup's "print, return 1 at the first failed rte_lpm_add"
 * (firewall.c:245-251): every later rule is dropped. Without this flag a
 * failed rule is skipped, counted in the report, and loading continues. */
#define COP_LPM_STOP_AT_FIRST_ERROR 0x1u

typedef struct cop_lpm_report {
    uint32_t n_in;            /* rules presented */
    uint32_t n_added;         /* rte_lpm_add calls that returned 0 */
    uint32_t n_distinct;      /* distinct rules held (rule-table occupancy) */
    uint32_t n_updated;       /* adds that hit an existing rule (last write wins) */
    uint32_t n_failed;        /* adds that returned < 0 */
    uint32_t n_skipped;       /* rules never presented (after a stop-at-first-error) */
    int32_t  first_error;     /* errno of the first failure (negative) or 0 */
    uint32_t first_error_idx; /* index of the first failed rule */
    uint32_t tbl8_used;       /* tbl8 groups in use */
    uint32_t n_intervals;     /* disjoint address intervals of the flattened table */
} cop_lpm_report;

/* ------------------------------------------------------------------------ */
/* Host-side LPM table (build once, upload to every GPU context)            */
/* ------------------------------------------------------------------------ */

typedef struct cop_lpm_table cop_lpm_table;

/* Build a table with DPDK rte_lpm_add semantics:
 * depth 1..32 else -EINVAL; ip masked to depth; a duplicate (prefix, depth)
 * overwrites the next hop; a new rule fails -ENOSPC once max_rules distinct
 * rules are held, or when it needs a tbl8 group and all number_tbl8s are in
 * use; a failed add leaves the table unchanged. Returns 0 or -errno. */
int  cop_lpm_build(const cop_prefix *rules, uint32_t n, const cop_lpm_config *cfg,
                   cop_lpm_table **out, cop_lpm_report *report);
void cop_lpm_free(cop_lpm_table *t);
/* Export the DIR-24-8 image: tbl24 has 1<<24 entries, tbl8 has tbl8_used*256.
 * Entry layout: bits 0-23 next hop (or tbl8 group), bit 24 valid,
 * bit 25 valid_group (extended), bits 26-31 depth — the DPDK v1604 layout. */
int  cop_lpm_export_dir24(const cop_lpm_table *t, uint32_t *tbl24, uint32_t *tbl8,
                          uint32_t tbl8_cap_entries);
/* Export the flattened form: starts[k] ascending, starts[0] == 0; value[k] =
 * (hit << 24) | next_hop for addresses in [starts[k], starts[k+1]). */
int  cop_lpm_export_intervals(const cop_lpm_table *t, uint32_t *starts, uint32_t *values,
                              uint32_t cap);
/* Accepted rule set after all adds: masked prefix, depth, final next hop.
 * The position in this list is the rule id (first-acceptance order of the
 * distinct (prefix, depth) pairs); per-rule hit counters are indexed by it. */
int  cop_lpm_export_rules(const cop_lpm_table *t, cop_prefix *out, uint32_t cap);
/* Host lookup of the matching (longest-prefix) rule id per address, -1 on a
 * miss. Setup/diagnostic use; the data path runs on the GPU. */
int  cop_lpm_lookup_rules(const cop_lpm_table *t, const uint32_t *ips, uint32_t n, int32_t *rule_id);

/* ------------------------------------------------------------------------ */
/* Rule files (rules.json format, firewall.c:57-105,276-323)                */
/* ------------------------------------------------------------------------ */

/* Parse a rules file: a JSON object (or array) whose children are objects
 * with case-insensitive keys "ip" (dotted quad, parsed with the reference's
 * sscanf("%u.%u.%u.%u") and &0xff per byte), "depth" and "action" (cJSON
 * valueint truncated to uint8). *out is malloc'd; free with cop_rules_free.
 * Errors: -ENOENT (open), -EINVAL (syntax, missing key, bad ip). */
int  cop_rules_load_json(const char *path, cop_prefix **out, uint32_t *n);
void cop_rules_free(cop_prefix *rules);
/* Write rules pretty-printed with short lines (<255 chars, firewall.c:72,95). */
int  cop_rules_write_json(const char *path, const cop_prefix *rules, uint32_t n);
/* Binary prefix dump for large sets: 16-byte header ("CPRB", u32 version 1,
 * u64 count) + count 12-byte cop_prefix records, little-endian, file order.
 * load: *out malloc'd (free with cop_rules_free); -ENOENT (open), -EINVAL
 * (magic, version, or size != header + count * 12), -ENOMEM, -EIO. */
int  cop_rules_load_bin(const char *path, cop_prefix **out, uint32_t *n);
int  cop_rules_write_bin(const char *path, const cop_prefix *rules, uint32_t n);

/* Default vport routing table (read_config, init.c:40-84): all 0, entries
 * 0..n_ports-1 = UNKNOWN_PORT, entry (192.167.10.(i+1) & 0xFFFF) = i. */
void cop_route_table_default(uint16_t *rt /* COP_ROUTING_TBL_SZ */, uint32_t n_ports);

/* ------------------------------------------------------------------------ */
/* GPU context: one per coprocessor thread or per GPU                       */
/* ------------------------------------------------------------------------ */

typedef struct cop_ctx cop_ctx;

#define COP_CFG_FW_FORCE_DIR24  0x1u  /* FW lookups from the HBM DIR-24-8 image, not LDS */
#define COP_CFG_LPM_FORCE_DIR24 0x2u  /* route lookups from HBM even if small */
#define COP_CFG_NO_COMPACT      0x4u  /* never build the ordered forward list */
#define COP_CFG_RULE_COUNTERS   0x8u  /* per-rule firewall hit counters (u64 per rule id) */
/* Demux: one ordered forward list per vport instead of one per batch — the
 * tx_q order of each port's coprocessor (enqueue_nf_rx switch.c:306-327,
 * then coprocessor() switch.c:464-470). Port q's list is at fwd_idx + q*n
 * (n = the batch's packet count), its length at fwd_count[q]; so fwd_idx
 * holds n_ports*n entries and fwd_count n_ports (ring: fwd_slot >=
 * n_ports*n, counts at fwd_count + slot*n_ports). Needs n_ports <= 8. */
#define COP_CFG_DEMUX_PORTS     0x10u
/* Per-port coprocessor_stats (switch.h:33-38) kept on the device. */
#define COP_CFG_PORT_STATS      0x20u
/* Route tables too large for LDS: look them up in the multibit-trie form
 * (12-bit top level in LDS, popcount-compressed 6-bit nodes, a few MiB that
 * stay in L2) instead of the 64 MiB DIR-24-8 image. Results are identical. */
#define COP_CFG_LPM_TRIE        0x40u
/* Segmented forward lists: a batch's ordered forward list is kept in
 * segments of COP_SEG_PKTS consecutive packets. Segment k (packets
 * k*COP_SEG_PKTS ..) holds its forwarded packets' indices, in arrival order,
 * at fwd_idx[k*COP_SEG_PKTS ..] and their number at fwd_count[k]; so
 * fwd_count holds ceil(n / COP_SEG_PKTS) words per batch (ring: per slot, at
 * fwd_count + slot*ceil(n/COP_SEG_PKTS)), and fwd_idx must be 16-byte
 * aligned (ring: fwd_slot a multiple of 4). Walking the segments in order
 * yields exactly the dense list — the tx side drains it segment by segment,
 * as coprocessor() hands its forward buffer over per burst of PKT_BURST_SZ
 * (switch.c:464-473). No tile waits for another's count, so the kernels
 * need no cross-workgroup prefix. Not combinable with DEMUX_PORTS. */
#define COP_CFG_SEG_LISTS       0x80u
#define COP_SEG_PKTS            256u
/* Route tables too large for LDS: look them up in the bucketed interval form
 * in global memory (a few MiB that stay in L2 / the Infinity Cache): the
 * bucket of the address's top bits gives the first candidate interval, one
 * 16-byte load of two (start, value) pairs decides almost every lookup.
 * Results are identical; takes precedence over COP_CFG_LPM_TRIE. */
#define COP_CFG_LPM_BKT         0x100u
/* Firewall tables too large for LDS (config 5's 1M rules) in the same
 * bucketed interval form, keyed by rule id, instead of the DIR-24-8 image:
 * about 16 + 12 MiB per 1M rules against 64 MiB, two dependent L2 / Infinity
 * Cache reads per lookup instead of one random 64 MiB probe. Results, rule
 * ids and per-rule counters are identical. */
#define COP_CFG_FW_BKT          0x200u
#define COP_MAX_DEMUX_PORTS     8

typedef struct cop_config {
    int      device;          /* HIP device ordinal */
    uint32_t stages;          /* COP_STAGE_* mask */
    uint32_t n_ports;         /* nb_active_kni (init.c:63), default 5 */
    uint32_t max_batch;       /* packets per batch, default 262144 */
    uint32_t max_batches;     /* batches per cop_submit, default 32 */
    uint32_t flags;           /* COP_CFG_* */
    uint32_t n_streams;       /* launch lanes (HIP streams) used round-robin, 1..4, default 2 */
    const uint16_t *routing_table; /* 65536 entries, or NULL = read_config default */
} cop_config;

void cop_config_default(cop_config *cfg);

/* Returns 0 or -ENODEV (no GPU), -EINVAL, -ENOMEM, -EIO (HIP error). */
int  cop_create(const cop_config *cfg, cop_ctx **out);
void cop_destroy(cop_ctx *ctx);
const char *cop_last_error(cop_ctx *ctx);
int  cop_device_count(void);
/* PCI bus id of a device ("dddd:bb:dd.f"), so a caller can run its
 * coprocessor threads and place their host buffers on the GPU's NUMA node
 * (as DPDK places lcores on the NIC's socket). 0, -EINVAL or -ENODEV. */
int  cop_device_pci_bus_id(int device, char *buf, int len);

/* Upload tables (synchronous). The table may be freed afterwards. */
int  cop_set_fw_table(cop_ctx *ctx, const cop_lpm_table *t);
int  cop_set_route_lpm(cop_ctx *ctx, const cop_lpm_table *t);
int  cop_set_routing_table(cop_ctx *ctx, const uint16_t *rt /* 65536 */);
/* setup_rules + lpm_setup in one call: read a rules.json file and build the
 * firewall table with cfg (NULL = reference 1024/24, stop at first error). */
int  cop_load_fw_rules_file(cop_ctx *ctx, const char *path, const cop_lpm_config *cfg,
                            cop_lpm_report *report);

/* Packed header records: a batch (or ring) with stride == COP_HDR16_STRIDE
 * and no offsets holds, instead of frames, one 16-byte record per packet:
 * frame bytes 12..15 (EtherType, version/IHL, TOS) followed by bytes 24..35
 * (IPv4 checksum, src, dst, UDP ports), the only bytes the pipeline reads.
 * Results are identical to the frames'. cop_pack_headers() builds them on
 * the host; the end-to-end host path moves 16 bytes per packet over PCIe
 * this way instead of a 64-byte header line. */
#define COP_HDR16_STRIDE 16u
void cop_pack_headers(const void *const *pkt_data, uint32_t n, uint8_t *out /* n * 16 bytes */);
/* Compact header records (cop_submit batches only, not rings): stride ==
 * COP_HDR12_STRIDE holds one 12-byte record per packet (pkts 4-byte
 * aligned), frame bytes 12..15 then 26..33 (src, dst): the bytes the
 * verdicts depend on, a quarter fewer
 * than a 16-byte record. Results are identical to the frames'. The
 * end-to-end host path (cop_process_host_stream) sends these. */
#define COP_HDR12_STRIDE 12u
void cop_pack_headers12(const void *const *pkt_data, uint32_t n, uint8_t *out /* n * 12 bytes */);

/* One batch of packets resident in device memory (HBM).
 * Packet i starts at  pkts + (offsets ? offsets[i] : i * stride) + data_off.
 * Every packet start must be 16-byte aligned and hold >= 48 readable bytes
 * (the fields sit at fixed offsets 12..33, as firewall.c:143-145 /
 * switch.c:125-127 read them; the streaming kernel moves whole 16-byte
 * chunks, and any Ethernet frame has >= 60). Outputs: results[i] for every packet;
 * fwd_idx[0..*fwd_count) = indices of FORWARD packets in arrival order (the
 * order coprocessor() enqueues them to tx_q, switch.c:464-470). */
typedef struct cop_batch {
    const void     *pkts;      /* device pointer */
    const uint32_t *offsets;   /* device pointer or NULL (IMIX slab mode) */
    uint32_t        n;         /* packets */
    uint32_t        stride;    /* bytes between packet slots (no offsets) */
    uint32_t        data_off;  /* added to every packet start (mbuf headroom) */
    uint32_t        _pad;
    cop_result     *results;   /* device pointer, n records */
    uint32_t       *fwd_idx;   /* device pointer, n entries, or NULL */
    uint32_t       *fwd_count; /* device pointer, 1 entry, or NULL */
} cop_batch;

/* Enqueue nb batches (nb <= max_batches) as ONE kernel launch on the next
 * launch lane (stream) of the context, round-robin. Launches on different
 * lanes may run concurrently. Asynchronous: returns once queued; outputs are
 * valid after cop_sync. */
int  cop_submit(cop_ctx *ctx, const cop_batch *batches, uint32_t nb);
/* A ring of equally shaped batch slots resident in device memory (a batch
 * ring buffer in HBM). Slot s: packets at pkts + s*pkts_slot_bytes (packet i
 * at + i*stride + data_off, or, when offsets != NULL, at + offsets_s[i] +
 * data_off with offsets_s = offsets + s*offsets_slot_words), records at
 * results + s*results_slot, forward list at fwd_idx + s*fwd_slot (may be
 * NULL), its length at fwd_count[s] (may be NULL). */
typedef struct cop_batch_ring {
    const void     *pkts;
    const uint32_t *offsets;
    cop_result     *results;
    uint32_t       *fwd_idx;
    uint32_t       *fwd_count;
    uint64_t        pkts_slot_bytes;
    uint64_t        offsets_slot_words;
    uint64_t        results_slot;      /* records per slot (>= n) */
    uint64_t        fwd_slot;          /* forward-list entries per slot (>= n) */
    uint32_t        n_slots;
    uint32_t        n;                 /* packets per batch */
    uint32_t        stride;
    uint32_t        data_off;
} cop_batch_ring;

#define COP_MAX_RING_BATCHES 1024u

/* Enqueue `count` (<= COP_MAX_RING_BATCHES) consecutive slots starting at
 * first_slot (wrapping at n_slots) as ONE kernel launch on the next lane.
 * Per-batch semantics are exactly those of cop_submit. */
int  cop_submit_ring(cop_ctx *ctx, const cop_batch_ring *ring, uint32_t first_slot, uint32_t count);

/* Block until everything submitted on every lane has completed. 0 or -EIO. */
int  cop_sync(cop_ctx *ctx);
/* Non-blocking: 0 when idle, -EAGAIN while work is in flight. */
int  cop_poll(cop_ctx *ctx);

/* End-to-end path from host memory (NIC/KNI mbuf data): gather the first 64
 * bytes of each packet into pinned staging, hipMemcpyAsync H2D, run the
 * pipeline, hipMemcpyAsync D2H of results and forward list. Synchronous. */
int  cop_process_host(cop_ctx *ctx, const void *const *pkt_data, uint32_t n,
                      cop_result *results, uint32_t *fwd_idx, uint32_t *fwd_count);
/* Streaming form of the end-to-end path: n packets at host addresses
 * pkt_data[i], in batches of `batch` (<= max_batch): the host gather of one
 * batch overlaps the H2D copy, kernel and D2H copy of earlier batches on the
 * other lanes. results[i] for every packet. Synchronous on return. */
int  cop_process_host_stream(cop_ctx *ctx, const void *const *pkt_data, uint64_t n, uint32_t batch,
                             cop_result *results);
/* Host threads for the header gather of the two calls above: the calling
 * thread plus n-1 persistent workers (default 1 = the caller alone). */
int  cop_set_host_threads(cop_ctx *ctx, uint32_t n);

/* Asynchronous host batches (the building block of
 * cop_coprocessor_poll_async): slot s < COP_HOST_SLOTS gathers the packets'
 * 16-byte header records into its mapped pinned staging on the calling
 * thread, then queues the pipeline on launch lane s % n_streams (the kernel
 * reads the records from, and writes its results to, host memory) and
 * returns.
 * cop_host_batch_wait blocks until slot s's records are in pinned host
 * memory and points *results at them (valid until slot s is submitted
 * again). -EBUSY if the slot is still in flight. */
#define COP_HOST_SLOTS 2u
int  cop_host_batch_submit(cop_ctx *ctx, uint32_t slot, const void *const *pkt_data, uint32_t n);
int  cop_host_batch_wait(cop_ctx *ctx, uint32_t slot, const cop_result **results, uint32_t *n);

/* ------------------------------------------------------------------------ */
/* Poll-mode coprocessor: a persistent kernel serving a batch ring          */
/* ------------------------------------------------------------------------ */

/* The GPU form of the reference's coprocessor lcores, which poll their rx
 * rings forever (main_loop -> coprocessor(), switch.c:529-535) rather than
 * being started per burst. cop_pmd_start launches ONE long-lived kernel on
 * its own stream that serves `ring` (a batch ring in HBM, as for
 * cop_submit_ring) until cop_pmd_stop: the host posts batches by bumping a
 * doorbell counter in mapped host memory, and the kernel writes each batch's
 * completion back there. Batch sequence number b (0, 1, 2, ... in post
 * order) lives in ring slot b % n_slots; per-batch outputs and counters are
 * exactly those of cop_submit_ring. No launch per post: no launch latency,
 * no grid ramp, tables staged into LDS once.
 * While it runs, the context's tables cannot change (-EBUSY) and it holds
 * every worker slot it could get: another kernel is NOT guaranteed to run
 * beside it. Counters stay readable: cop_counters_read /
 * cop_counters_snapshot / cop_rule_counters_read / cop_coll_reduce_counters
 * see every completed batch (a batch's counter adds land before its
 * completion), and their reset is an atomic read-and-zero, so nothing is
 * lost or counted twice while batches run. Those that need a kernel of
 * their own (the rule-hit count, the snapshot, the RCCL all-reduce) PAUSE
 * the poll-mode kernel: it finishes every batch posted so far and leaves,
 * the side work runs, and it is relaunched (microseconds, not a wait for
 * an idle exit). Posts during a pause wait for the relaunch. One per
 * context. The kernel leaves by itself after 1 s without a post
 * ($COP_PMD_IDLE_MS) and is relaunched by the next post.
 * A ring whose pkts / results / lists live in mapped host memory must be
 * allocated coherent (cop_host_alloc_mapped does): a persistent kernel has
 * no kernel-end cache writeback, so its stores to non-coherent host pages
 * can stay in the GPU's L2. */
typedef struct cop_pmd cop_pmd;
int cop_pmd_start(cop_ctx *ctx, const cop_batch_ring *ring, cop_pmd **out);
/* Post the next `count` batches (<= n_slots): sequence numbers posted ..
 * posted+count-1. Blocks while that would reuse a slot whose batch has not
 * completed. 0 or -errno. */
int cop_pmd_post(cop_pmd *pmd, uint32_t count);
/* Spin until every batch with sequence number < seq has completed: records,
 * forward lists and counts are in HBM, visible to the host and to later
 * kernels. 0, -ETIMEDOUT (30 s) or -EIO (the kernel aborted). */
int cop_pmd_wait(cop_pmd *pmd, uint64_t seq);
uint64_t cop_pmd_posted(const cop_pmd *pmd);
/* Post `count` batches (in posts of a quarter ring, so it never drains) and
 * wait for all of them: one synchronous burst. 0 or -errno. */
int cop_pmd_run(cop_pmd *pmd, uint64_t count);
/* cop_pmd_run, stamped: CLOCK_MONOTONIC (ns) just before the first post and
 * just after the last batch is seen complete (benchmarks: the window of the
 * library call itself, no caller overhead in it). 0 or -errno. */
int cop_pmd_run_timed(cop_pmd *pmd, uint64_t count, uint64_t *t_post_ns, uint64_t *t_done_ns);
typedef struct cop_pmd_info_t {
    uint32_t workers;          /* worker workgroups (all co-resident) */
    uint32_t workers_per_cu;
    uint32_t tiles_per_batch;
    uint32_t packets_per_tile;
    uint32_t launches;         /* 1 + relaunches after idle exits */
    uint32_t state;            /* 0 running, 1 stopped, 2 left idle, 3 aborted, 4 paused */
    uint64_t posted, completed; /* summed over the rings */
    uint32_t slot_loads;       /* how tiles read their slots: 0 plain (COP_PMD_STATIC_SLOTS),
                                  3 system-coherent loads every tile (COP_PMD_SYS_ACQUIRE,
                                  host-memory rings, or slots not on 128-byte lines),
                                  4 coherent loads once the ring wraps (default); 1 and 2
                                  (acquires) only through $COP_PMD_ACQUIRE A/B runs */
    uint32_t kernel;           /* the kernel instantiation serving the rings,
                                  cop_pmd<fw, route, layout, ppt, ext>: fw table form | route form << 4
                                  | layout << 8 | ext << 12 (forms: 0 off, 1 LDS intervals, 2 DIR-24-8,
                                  3 trie, 4 bucketed; layouts: 0 slots, 1 IMIX, 2 coalesced 64 B,
                                  3 16-byte records; ppt = packets_per_tile / 256) */
} cop_pmd_info_t;
int cop_pmd_info(const cop_pmd *pmd, cop_pmd_info_t *out);
/* Complete everything posted, stop the kernel, free. */
int cop_pmd_stop(cop_pmd *pmd);

/* Several rx rings served by ONE poll-mode kernel: the GPU form of the
 * reference's five coprocessor lcores, each polling its own rx ring
 * (KNI_KTHREAD, main.c:92-94, switch.c:463). The kernel's workers are split
 * among the rings (worker w serves ring w % n_rings); each ring has its own
 * batch sequence, doorbell and completion words, so its batches complete in
 * its own order and one ring's thread never waits for another's. Every ring
 * must have ring 0's geometry (n, n_slots, stride, data_off, layout, slot
 * sizes); the pointers are each ring's own. Ring r is posted and waited by
 * one thread (different rings from different threads). At most
 * COP_PMD_MAX_RINGS. The single-ring calls above act on ring 0. */
#define COP_PMD_MAX_RINGS 8
#define COP_PMD_VARIABLE_N 1u   /* batches carry their own packet count (cop_pmd_post_batch) */
/* Slot reuse. The reference's fast path refills its rings forever
 * (switch.c:463-470), and a ring slot here may likewise be rewritten by
 * another agent (the host with cop_memcpy_h2d, a NIC, another GPU) between
 * its batches. A persistent kernel gets no dispatch-time cache invalidation,
 * so a CU or L2 could serve a slot's previous contents. By DEFAULT (no flag,
 * and always through cop_pmd_start) every tile reads its packets with
 * system-coherent loads (no cached copy used) once its ring has wrapped in
 * the running launch: a slot's first read in a launch is fresh, every reuse
 * is safe. COP_PMD_SYS_ACQUIRE: coherent loads on every tile (rings in host
 * memory get this without the flag). COP_PMD_STATIC_SLOTS: the caller
 * declares the slots written once before cop_pmd_start_rings and never again
 * while the kernel runs (a benchmark's resident pool): plain loads. The two
 * contradict (-EINVAL). */
#define COP_PMD_SYS_ACQUIRE 2u
#define COP_PMD_STATIC_SLOTS 4u
/* Dynamic tiles (rings with segmented lists, COP_CFG_SEG_LISTS): workers
 * claim tiles from ticket counters instead of a static order, and issue the
 * next tile's header loads before they classify the current one. Same
 * outputs; a higher poll-mode steady state on long streams, about the same
 * rate on short bursts. Ignored without segmented lists. */
#define COP_PMD_DYNAMIC_TILES 8u
int cop_pmd_start_rings(cop_ctx *ctx, const cop_batch_ring *rings, uint32_t n_rings, uint32_t flags,
                        cop_pmd **out);
/* Post the next `count` full batches (n packets each) of one ring. */
int cop_pmd_post_ring(cop_pmd *pmd, uint32_t ring, uint32_t count);
/* Post ONE batch of n (1..ring n) packets to one ring: the packets
 * 0..n-1 of its next slot (COP_PMD_VARIABLE_N). */
int cop_pmd_post_batch(cop_pmd *pmd, uint32_t ring, uint32_t n);
/* As cop_pmd_wait, for one ring's sequence numbers. */
int cop_pmd_wait_ring(cop_pmd *pmd, uint32_t ring, uint64_t seq);
uint64_t cop_pmd_posted_ring(const cop_pmd *pmd, uint32_t ring);
/* Batches of the ring known complete (reads the completion words). */
uint64_t cop_pmd_completed_ring(cop_pmd *pmd, uint32_t ring);

/* Counters (u64, device-resident, summed over every submitted packet).
 * On the device they are kept in COP_COUNTER_SHARDS shards of
 * COP_N_COUNTERS words (one 128-byte line each, to spread the atomics);
 * cop_counters_read folds the shards.
 * pkt_total / pkt_not_ipv4 mirror struct firewall_pkt_stats
 * (firewall.h:56-61, incremented at firewall.c:184,188); pkt_accept /
 * pkt_drop are filled here although the reference never increments them. */
typedef struct cop_counters {
    uint64_t pkt_drop;       /* DROP_FW + DROP_NOT_IPV4 (FW stage) */
    uint64_t pkt_accept;     /* FORWARD after the FW stage */
    uint64_t pkt_not_ipv4;
    uint64_t pkt_total;      /* packets that entered the FW stage */
    uint64_t parse_err;      /* DROP_PARSE (kni_interface_stats.parse_err) */
    uint64_t no_port;        /* DROP_NO_PORT */
    uint64_t forward;        /* verdict FORWARD (coprocessor tx) */
    uint64_t route_hit;      /* route LPM hits */
    uint64_t rx;             /* packets submitted */
    uint64_t _rsvd[7];
} cop_counters;
#define COP_N_COUNTERS 16
#define COP_COUNTER_SHARDS 256

int  cop_counters_read(cop_ctx *ctx, cop_counters *out, int reset);
/* Device address of the COP_COUNTER_SHARDS x COP_N_COUNTERS u64 counter
 * shards (an element-wise sum over GPUs preserves the per-shard layout). */
void *cop_counters_device_ptr(cop_ctx *ctx);

/* Per-port statistics (COP_CFG_PORT_STATS), mirroring struct
 * coprocessor_stats (switch.h:33-38) of the NF serving each vport:
 * rx_packets = packets routed to the port (enqueue_nf_rx), tx_packets =
 * packets its NF forwarded, nf_dropped = rx - tx (freed by the NF). The
 * ring-overflow drops (rx_dropped / tx_dropped) cannot occur on the device
 * path and read 0. With stage P off every packet counts as port 0. */
typedef struct cop_port_stats {
    uint64_t rx_packets;
    uint64_t rx_dropped;
    uint64_t tx_packets;
    uint64_t tx_dropped;
    uint64_t nf_dropped;
} cop_port_stats;
/* Synchronous read of min(n, n_ports) ports; returns n_ports or -errno. */
int  cop_port_stats_read(cop_ctx *ctx, cop_port_stats *out, uint32_t n, int reset);
/* Live telemetry, the read-and-zero of print_stats (switch.c:33-90), safe
 * while launches are in flight: counters (and port stats) are read — or
 * atomically exchanged with 0 when reset — by a small kernel on a separate
 * stream; no increment is lost or counted twice across snapshots. Does not
 * wait for submitted work. */
int  cop_counters_snapshot(cop_ctx *ctx, cop_counters *total, cop_port_stats *ports, uint32_t n_ports,
                           int reset);

/* Per-rule firewall hit counters (COP_CFG_RULE_COUNTERS): one u64 per rule
 * id of the firewall table (cop_lpm_export_rules order), incremented for
 * every IPv4 packet whose source matches that rule in the FW stage (the
 * rule rte_lpm_lookup resolved at firewall.c:194). Zeroed by
 * cop_set_fw_table. read: copies min(cap, n_rules) words, returns n_rules
 * (or -errno); reset != 0 zeroes them after the copy. */
int  cop_rule_counters_read(cop_ctx *ctx, uint64_t *out, uint32_t cap, int reset);
/* Device address and length of the per-rule counters. One allocation holds
 * the COP_COUNTER_SHARDS x COP_N_COUNTERS shard words, then the port-stat
 * shards (COP_COUNTER_SHARDS x 16), then the per-rule words, so one
 * element-wise u64 sum covers all three. */
int  cop_rule_counters_device_ptr(cop_ctx *ctx, void **dptr, uint32_t *n_rules);

/* Cross-GPU counter reduction over RCCL (xGMI): one communicator per
 * context, one rank per GPU. The 128-byte unique id comes from rank 0's
 * cop_coll_unique_id and is distributed by the caller (any transport).
 * librccl is loaded on first use; -ENOSYS when it is absent. */
#define COP_COLL_ID_BYTES 128
int  cop_coll_unique_id(uint8_t id[COP_COLL_ID_BYTES]);
int  cop_coll_init(cop_ctx *ctx, const uint8_t id[COP_COLL_ID_BYTES], int rank, int nranks);
/* All-reduce (u64 sum) of the counter shards and per-rule counters of every
 * rank, on the context's stream; synchronous. The sums are written to
 * *total and rule_hits[0..min(cap, n_rules)) when non-NULL (cap = 0 skips
 * the per-rule copy). reset != 0 zeroes this rank's local counters after
 * the reduction (the read-and-zero of print_stats, switch.c:33-90). */
int  cop_coll_reduce_counters(cop_ctx *ctx, cop_counters *total, uint64_t *rule_hits, uint32_t cap,
                              int reset);

/* Device memory helpers so C callers need no HIP headers. */
int  cop_dev_alloc(cop_ctx *ctx, size_t bytes, void **dptr);
/* HBM with another cache policy, for a poll-mode ring's outputs (records,
 * lists, counts) that the host or another agent reads while the kernel runs:
 * COP_ALLOC_UNCACHED (no GPU cache holds a line: a store is in memory once
 * it has drained) or COP_ALLOC_FINEGRAINED (coherent fine-grained memory).
 * Free with cop_dev_free. 0, or -errno. */
#define COP_ALLOC_UNCACHED 1u
#define COP_ALLOC_FINEGRAINED 2u
int  cop_dev_alloc_ex(cop_ctx *ctx, size_t bytes, uint32_t flags, void **dptr);
int  cop_dev_free(cop_ctx *ctx, void *dptr);
int  cop_host_alloc_pinned(cop_ctx *ctx, size_t bytes, void **hptr);
int  cop_host_free_pinned(cop_ctx *ctx, void *hptr);
/* Pinned host memory the device reads and writes coherently (mapped into
 * the device's address space; *dptr is the device's pointer to it): rings a
 * poll-mode kernel serves from host memory. Free with cop_host_free_pinned. */
int  cop_host_alloc_mapped(cop_ctx *ctx, size_t bytes, void **hptr, void **dptr);
int  cop_memcpy_h2d(cop_ctx *ctx, void *dst, const void *src, size_t bytes);
int  cop_memcpy_d2h(cop_ctx *ctx, void *dst, const void *src, size_t bytes);
int  cop_memcpy_d2d(cop_ctx *ctx, void *dst, const void *src, size_t bytes);
int  cop_memset_d(cop_ctx *ctx, void *dst, int value, size_t bytes);

/* Timing with HIP events: start/stop join every lane of the context. */
int  cop_timer_start(cop_ctx *ctx);
int  cop_timer_stop(cop_ctx *ctx, double *ms);
/* When on, every cop_submit is bracketed by an event pair; the mean kernel
 * duration of the launches since the last reset is returned in ms. */
int  cop_launch_timing(cop_ctx *ctx, int enable);
int  cop_launch_timing_read(cop_ctx *ctx, double *mean_ms, uint64_t *n, int reset);

/* ------------------------------------------------------------------------ */
/* SPSC ring with rte_ring bulk/burst semantics (init.c:74-75, switch.c)    */
/* ------------------------------------------------------------------------ */

typedef struct cop_ring cop_ring;
/* count must be a power of two; capacity is count - 1 (rte_ring default). */
cop_ring *cop_ring_create(uint32_t count);
void      cop_ring_free(cop_ring *r);
/* All-or-nothing: returns n or 0 (rte_ring_enqueue_bulk, switch.c:225,268). */
uint32_t  cop_ring_enqueue_bulk(cop_ring *r, void *const *objs, uint32_t n, uint32_t *free_space);
/* Up to n (rte_ring_dequeue_burst, switch.c:430,463). */
uint32_t  cop_ring_dequeue_burst(cop_ring *r, void **objs, uint32_t n, uint32_t *available);
uint32_t  cop_ring_count(const cop_ring *r);

/* ------------------------------------------------------------------------ */
/* Drop-in coprocessor API (coprocessor.h:23-30)                            */
/* ------------------------------------------------------------------------ */

/* rte_mbuf is opaque; the packet data address is
 * *(void **)(m + buf_addr_off) + *(uint16_t *)(m + data_off_off)
 * (rte_pktmbuf_mtod). Defaults match DPDK 17.11-19.05: 0 and 16. */
struct rte_mbuf;
void cop_set_mbuf_layout(uint32_t buf_addr_off, uint32_t data_off_off);
/* Rule file used by coprocessor_setup (coprocessor.c:19); default
 * "./nfs/firewall/rules.json", or $COP_RULE_FILE when set. */
void cop_set_rule_file(const char *path);

/* Per calling thread: create a GPU context (device = $COP_DEVICE or 0),
 * load the rule file with the reference limits. 0 or non-zero. Runs the
 * drop-in stage mask (cop_dropin_stages(), COP_STAGE_FW unless set). */
int coprocessor_setup(void);
/* The drop-in NF chain for contexts set up afterwards and for the drop-in
 * calls: COP_STAGE_FW or 0 (no NF: every packet forwards). 0 or -EINVAL. */
int cop_set_dropin_stages(uint32_t stages);
uint32_t cop_dropin_stages(void);
/* cop_set_dropin_stages(stages), then coprocessor_setup(). */
int cop_coprocessor_setup_stages(uint32_t stages);
/* coprocessor_setup() with a fixed chain: the firewall (ENABLE_FW_NF), or
 * none (DISABLE_NF). Same signature as coprocessor_setup. */
int cop_coprocessor_setup_fw(void);
int cop_coprocessor_setup_no_nf(void);
#ifndef COP_NO_DROPIN_MACROS
/* The caller's ENABLE_FW_NF / DISABLE_NF select the chain (see
 * COP_DROPIN_STAGES). An object-like alias: the reference's own declaration
 * `int coprocessor_setup(void);` (coprocessor.h:30) after this header still
 * compiles, and &coprocessor_setup is a function pointer. */
#if defined(DISABLE_NF) || defined(COP_DROPIN_NO_NF)
#define coprocessor_setup cop_coprocessor_setup_no_nf
#else
#define coprocessor_setup cop_coprocessor_setup_fw
#endif
#endif
int coprocessor_teardown(void);
/* 0 = forward, -1 = drop (coprocessor.c:50-65). One-packet GPU batch:
 * correct but latency-bound; use process_burst / cop_coprocessor_poll. */
int process_packet(struct rte_mbuf *pkt);
/* Burst form: ret[i] = process_packet(pkts[i]) for all i, one GPU batch. */
int process_burst(struct rte_mbuf **pkts, uint32_t n, int *ret);

/* Per-coprocessor counters (struct coprocessor_stats, switch.h:33-38). */
typedef struct cop_nf_stats {
    uint64_t rx_packets;
    uint64_t rx_dropped;
    uint64_t tx_packets;
    uint64_t tx_dropped;
} cop_nf_stats;

/* GPU replacement for one call of coprocessor() (switch.c:443-474): drain up
 * to max_pkts mbufs from rx in bursts of PKT_BURST_SZ, run them as one GPU
 * batch, enqueue forwarded mbufs to tx in arrival order in bulk bursts of
 * PKT_BURST_SZ (a burst that does not fit is freed and counted tx_dropped),
 * and free dropped mbufs with free_fn. Returns packets processed or -errno. */
typedef void (*cop_free_fn)(struct rte_mbuf *m, void *arg);
int cop_coprocessor_poll(cop_ctx *ctx, cop_ring *rx, cop_ring *tx, uint32_t max_pkts,
                         cop_free_fn free_fn, void *free_arg, cop_nf_stats *stats);
/* Pipelined form of cop_coprocessor_poll: each call drains up to max_pkts
 * and submits them as a GPU batch without waiting, then completes the
 * previous call's batch, forwarding and freeing exactly as
 * cop_coprocessor_poll does. So the host drains and gathers one batch while
 * the GPU runs the other. Packets leave in arrival order. Returns packets
 * completed by this call or -errno. When rx is empty, a call completes the
 * batch in flight. cop_coprocessor_flush completes everything in flight
 * (e.g. before coprocessor_teardown). */
int cop_coprocessor_poll_async(cop_ctx *ctx, cop_ring *rx, cop_ring *tx, uint32_t max_pkts,
                               cop_free_fn free_fn, void *free_arg, cop_nf_stats *stats);
int cop_coprocessor_flush(cop_ctx *ctx, cop_ring *tx, cop_free_fn free_fn, void *free_arg, cop_nf_stats *stats);
/* The calling thread's context created by coprocessor_setup (or NULL). */
cop_ctx *coprocessor_ctx(void);

/* The ring loop of several coprocessor threads on ONE poll-mode kernel (the
 * reference's five coprocessor lcores, each with its own rx ring,
 * main.c:92-94): cop_pmd_host_create starts a kernel on ctx serving n_rings
 * rings of n_slots batches of up to max_pkts packets each, whose 16-byte
 * header records and result records live in mapped pinned host memory (no
 * launch and no copy per batch), running the drop-in NF chain. Thread r then
 * calls cop_coprocessor_poll_pmd(h, r, ...) in its loop: it drains up to
 * max_pkts mbufs from rx, gathers their headers into ring r's next slot and
 * posts it; it completes (forwards to tx in arrival order, frees drops, as
 * cop_coprocessor_poll) every batch of the ring already done, oldest first,
 * and, when rx was empty or every slot is in flight, waits for the oldest.
 * Returns packets completed or -errno. cop_coprocessor_flush_pmd completes
 * everything ring r has in flight; cop_pmd_host_destroy (after every ring's
 * flush) stops the kernel. Ring r is used by one thread. */
typedef struct cop_pmd_host cop_pmd_host;
int cop_pmd_host_create(cop_ctx *ctx, uint32_t n_rings, uint32_t max_pkts, uint32_t n_slots, cop_pmd_host **out);
int cop_coprocessor_poll_pmd(cop_pmd_host *h, uint32_t ring, cop_ring *rx, cop_ring *tx, uint32_t max_pkts,
                             cop_free_fn free_fn, void *free_arg, cop_nf_stats *stats);
int cop_coprocessor_flush_pmd(cop_pmd_host *h, uint32_t ring, cop_ring *tx, cop_free_fn free_fn, void *free_arg,
                              cop_nf_stats *stats);
int cop_pmd_host_destroy(cop_pmd_host *h);

/* ------------------------------------------------------------------------ */
/* Deterministic synthetic workload (SURVEY.md §8d generator)               */
/* ------------------------------------------------------------------------ */

#define COP_GEN_FW     0  /* 1k-style firewall rule mix */
#define COP_GEN_ROUTES 1  /* BGP-like route prefix mix  */

/* Rules: splitmix64(seed). FW: 60% /24, 20% /16-23, 10% /8-15, 10% /25-32
 * confined to n_long_parents /24s; action 0 w.p. 0.5 else 1..255.
 * Routes: 55% /24, 25% /17-23, 10% /8-16, 10% /25-32; nh 1..2^24-1. */
int cop_gen_rules(uint64_t seed, uint32_t n, int kind, uint32_t n_long_parents,
                  cop_prefix *out);

typedef struct cop_trace_opts {
    uint32_t n_ports;         /* vports 192.167.10.1..n (default 5) */
    uint32_t pct_non_ipv4;    /* EtherType 0x86DD percentage (default 2) */
    uint32_t pct_bad_version; /* IPv4 EtherType, version != 4 (default 0) */
    uint32_t pct_unknown_dst; /* dst low16 in 0..4 (default 5) */
    uint32_t pct_vport_dst;   /* dst 192.167.10.x (default 60) */
    uint32_t pct_src_in_rule; /* src inside a FW rule prefix (default 50) */
} cop_trace_opts;
void cop_trace_opts_default(cop_trace_opts *o);

/* n 64-byte frames written at out + i*stride (stride >= 64). */
int cop_gen_trace(uint64_t seed, uint32_t n, const cop_trace_opts *opts,
                  const cop_prefix *fw, uint32_t n_fw,
                  const cop_prefix *routes, uint32_t n_routes,
                  uint8_t *out, uint32_t stride);
/* Simple IMIX 64/594/1518 at 7:4:1 packed into a slab at 64-byte aligned
 * offsets. Call with slab == NULL to get the slab size in *slab_bytes. */
int cop_gen_imix(uint64_t seed, uint32_t n, const cop_trace_opts *opts,
                 const cop_prefix *fw, uint32_t n_fw,
                 const cop_prefix *routes, uint32_t n_routes,
                 uint8_t *slab, uint64_t *slab_bytes, uint32_t *offsets);

#ifdef __cplusplus
}
#endif
#endif /* COP_GPU_H */
