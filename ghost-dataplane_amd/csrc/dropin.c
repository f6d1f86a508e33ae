/*
 * dropin.c — the reference's coprocessor API on top of the GPU context.
 *
 *   coprocessor_setup    coprocessor.c:21-35  (setup_rules + lpm_setup)
 *   coprocessor_teardown coprocessor.c:37-49
 *   process_packet       coprocessor.c:50-65  (0 forward / -1 drop)
 *   cop_coprocessor_poll switch.c:443-474     (coprocessor() loop body)
 *
 * All of them run the drop-in stage mask, the NF chain of process_packet:
 * the firewall (fw_packet_handler under ENABLE_FW_NF, coprocessor.c:59-62),
 * or nothing (coprocessor.c:59-64 without it: every packet forwards);
 * cop_set_dropin_stages / the COP_DROPIN_STAGES macro of the caller's build
 * choose. get_next_hop's parse/route drop belongs to the fast path
 * (switch.c:406-415), which has already routed every packet it enqueues to
 * a coprocessor ring.
 *
 * The reference calls setup/teardown once per coprocessor lcore, five
 * threads at once (main.c:92-94, switch.c:525,537), with NF state in
 * process globals (firewall.h:107-110). Here every calling thread gets its
 * own context in thread-local storage, so the threads share nothing.
 */
#define _POSIX_C_SOURCE 199309L   /* clock_gettime (diagnostic profile) */
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define COP_NO_DROPIN_MACROS 1   /* this file defines the functions the macros call */
#include "cop_gpu.h"
#include "cop_internal.h"

static uint32_t g_buf_addr_off = 0;   /* rte_mbuf.buf_addr (DPDK 17.11-19.05) */
static uint32_t g_data_off_off = 16;  /* rte_mbuf.data_off */
static char g_rule_file[4096] = "./nfs/firewall/rules.json"; /* coprocessor.c:19 */
static volatile uint32_t g_dropin_stages = COP_STAGE_FW;       /* ENABLE_FW_NF, coprocessor.h:21 */
static int g_rule_file_set = 0;

static __thread cop_ctx *tl_ctx = NULL;
/* Pipelined ring loop: per thread, up to COP_HOST_SLOTS batches in flight,
 * completed oldest first, so packets leave in arrival order. */
static __thread struct {
    void **objs[COP_HOST_SLOTS];
    uint32_t cap[COP_HOST_SLOTS];
    const void **data;
    uint32_t data_cap;
    uint32_t fifo[COP_HOST_SLOTS];   /* slots in flight, oldest first */
    uint32_t n[COP_HOST_SLOTS];      /* mbufs held by each slot in flight */
    uint32_t depth;
    cop_ctx *ctx;                    /* the context the slots were submitted on */
} tl_async;

static __thread struct {
    void **objs;
    const void **data;
    cop_result *res;
    uint32_t cap;
} tl_buf;

/* forward_batch's list of the mbufs to free (per thread) */
static __thread struct {
    void **drop;
    uint32_t cap;
} tl_fwd;

/* Diagnostic per-op host time of this thread's ring loop ($COP_HOST_PROF=1,
 * cop_debug_dropin_prof): ns in drain (dequeue + mbuf data addresses),
 * batch (cop_process_host_stages: gather, launch, wait, copy-out; or the
 * async submit: gather + launch), wait (async completion), forward (tx
 * enqueue + frees); then calls, calls that found packets, packets. */
enum { PROF_DRAIN, PROF_BATCH, PROF_WAIT, PROF_FWD, PROF_CALLS, PROF_BUSY_CALLS, PROF_PKTS, PROF_N };
static __thread uint64_t tl_prof[PROF_N];
static int g_prof = -1;

static inline int prof_on(void)
{
    if (g_prof < 0) {
        const char *e = getenv("COP_HOST_PROF");
        g_prof = e && atoi(e) ? 1 : 0;
    }
    return g_prof;
}

static inline uint64_t prof_ns(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

int cop_debug_dropin_prof(uint64_t *out, uint32_t n, int reset)
{
    if (!out) return -EINVAL;
    for (uint32_t i = 0; i < n && i < PROF_N; i++) out[i] = tl_prof[i];
    if (reset) memset(tl_prof, 0, sizeof(tl_prof));
    return PROF_N;
}

void cop_set_mbuf_layout(uint32_t buf_addr_off, uint32_t data_off_off)
{
    g_buf_addr_off = buf_addr_off;
    g_data_off_off = data_off_off;
}

void cop_set_rule_file(const char *path)
{
    if (!path) return;
    snprintf(g_rule_file, sizeof(g_rule_file), "%s", path);
    g_rule_file_set = 1;
}

static inline const void *mbuf_data(const struct rte_mbuf *m)
{
    const uint8_t *b = (const uint8_t *)m;
    void *addr;
    uint16_t off;
    memcpy(&addr, b + g_buf_addr_off, sizeof(addr));
    memcpy(&off, b + g_data_off_off, sizeof(off));
    return (const uint8_t *)addr + off;   /* rte_pktmbuf_mtod */
}

int cop_set_dropin_stages(uint32_t stages)
{
    if (stages & ~COP_STAGE_FW) return -EINVAL;   /* process_packet's chain: the firewall or nothing */
    g_dropin_stages = stages;
    return 0;
}

uint32_t cop_dropin_stages(void)
{
    return g_dropin_stages;
}

int cop_coprocessor_setup_stages(uint32_t stages)
{
    int rc = cop_set_dropin_stages(stages);
    if (rc) return 1;
    return coprocessor_setup();
}

int cop_coprocessor_setup_fw(void)
{
    return cop_coprocessor_setup_stages(COP_STAGE_FW);
}

int cop_coprocessor_setup_no_nf(void)
{
    return cop_coprocessor_setup_stages(0u);
}

cop_ctx *coprocessor_ctx(void)
{
    return tl_ctx;
}

int coprocessor_setup(void)
{
    if (tl_ctx) return 0;
    cop_config cfg;
    cop_config_default(&cfg);
    cfg.stages = g_dropin_stages;
    const char *dev = getenv("COP_DEVICE");
    if (dev) cfg.device = atoi(dev);
    int rc = cop_create(&cfg, &tl_ctx);
    if (rc) {
        fprintf(stderr, "coprocessor_setup: no GPU context (%d)\n", rc);
        tl_ctx = NULL;
        return 1;
    }
    const char *path = g_rule_file;
    const char *env = getenv("COP_RULE_FILE");
    if (env && !g_rule_file_set) path = env;
    /* lpm_setup's fixed limits and its stop-at-first-error behaviour */
    cop_lpm_config lc = {COP_FW_MAX_RULES, COP_FW_NUMBER_TBL8S, COP_LPM_STOP_AT_FIRST_ERROR};
    cop_lpm_report rep;
    rc = cop_load_fw_rules_file(tl_ctx, path, &lc, &rep);
    if (rc) {
        /* setup_rules rte_exits when the file cannot be parsed (firewall.c:291-296) */
        fprintf(stderr, "coprocessor_setup: %s\n", cop_last_error(tl_ctx));
        cop_destroy(tl_ctx);
        tl_ctx = NULL;
        return 1;
    }
    if (rep.n_failed)
        fprintf(stderr, "coprocessor_setup: rule %u failed (%d); %u later rules dropped\n",
                rep.first_error_idx, rep.first_error, rep.n_skipped);
    return 0;
}

/* Free n dequeued mbufs that will never be forwarded (an error after the
 * dequeue): the reference never loses a dequeued packet, it enqueues or
 * frees each one (switch.c:464-470). Counted as tx_dropped. */
static void drop_all(void *const *objs, uint32_t n, cop_free_fn free_fn, void *free_arg, cop_nf_stats *stats)
{
    if (free_fn)
        for (uint32_t i = 0; i < n; i++) free_fn((struct rte_mbuf *)objs[i], free_arg);
    if (stats) stats->tx_dropped += n;
}

int coprocessor_teardown(void)
{
    int rc = 0;
    if (tl_async.depth) {
        /* batches still in flight (cop_coprocessor_flush was not called):
         * wait for their kernels before the context goes away; their mbufs
         * were never forwarded or freed, so say so */
        uint32_t held = 0;
        for (uint32_t i = 0; i < tl_async.depth; i++) {
            (void)cop_host_batch_wait(tl_async.ctx, tl_async.fifo[i], NULL, NULL);
            held += tl_async.n[tl_async.fifo[i]];
        }
        fprintf(stderr, "coprocessor_teardown: %u batch(es) in flight, %u mbufs neither forwarded nor freed "
                        "(call cop_coprocessor_flush first)\n", tl_async.depth, held);
        tl_async.depth = 0;
        rc = 1;
    }
    if (tl_ctx) cop_destroy(tl_ctx);
    tl_ctx = NULL;
    for (uint32_t s = 0; s < COP_HOST_SLOTS; s++) {
        free(tl_async.objs[s]);
        tl_async.objs[s] = NULL;
        tl_async.cap[s] = 0;
    }
    free((void *)tl_async.data);
    tl_async.data = NULL;
    tl_async.data_cap = 0;
    tl_async.ctx = NULL;
    free(tl_buf.objs);
    free(tl_buf.data);
    free(tl_buf.res);
    memset(&tl_buf, 0, sizeof(tl_buf));
    free(tl_fwd.drop);
    tl_fwd.drop = NULL;
    tl_fwd.cap = 0;
    return rc;
}

static int ensure_buf(uint32_t n)
{
    if (tl_buf.cap >= n) return 0;
    uint32_t cap = n < 1024 ? 1024 : n;
    void **o = (void **)realloc(tl_buf.objs, cap * sizeof(void *));
    if (o) tl_buf.objs = o;
    const void **d = (const void **)realloc((void *)tl_buf.data, cap * sizeof(void *));
    if (d) tl_buf.data = d;
    cop_result *r = (cop_result *)realloc(tl_buf.res, cap * sizeof(cop_result));
    if (r) tl_buf.res = r;
    if (!o || !d || !r) return -ENOMEM;
    tl_buf.cap = cap;
    return 0;
}

int process_burst(struct rte_mbuf **pkts, uint32_t n, int *ret)
{
    if (!tl_ctx || (n && (!pkts || !ret))) return -EINVAL;
    if (ensure_buf(n)) return -ENOMEM;
    for (uint32_t i = 0; i < n; i++) tl_buf.data[i] = mbuf_data(pkts[i]);
    int rc = cop_process_host_stages(tl_ctx, g_dropin_stages, tl_buf.data, n, tl_buf.res, NULL, NULL);
    if (rc) return rc;
    for (uint32_t i = 0; i < n; i++) ret[i] = tl_buf.res[i].verdict == COP_FORWARD ? 0 : -1;
    return 0;
}

int process_packet(struct rte_mbuf *pkt)
{
    int r = -1;
    if (process_burst(&pkt, 1, &r)) return -1;
    return r;
}

/* forward in arrival order through a PKT_BURST_SZ tx buffer flushed with
 * an all-or-nothing bulk enqueue (enqueue_nf_tx / flush_nf_tx_queue,
 * switch.c:240-280,329-351); drops are freed (switch.c:469). The verdicts
 * are split without branches (a forward/drop branch mispredicts on every
 * third packet): the forwarded mbufs go to the tx bursts in order, the
 * dropped ones to a list freed after. */
static void forward_batch(cop_ring *tx, void *const *objs, const cop_result *res, uint32_t n, cop_free_fn free_fn,
                          void *free_arg, cop_nf_stats *stats)
{
    if (tl_fwd.cap < n) {
        void **d = (void **)realloc(tl_fwd.drop, (n < 1024 ? 1024 : n) * sizeof(void *));
        if (!d) {   /* no scratch: free nothing lost, forward nothing (counted) */
            drop_all(objs, n, free_fn, free_arg, stats);
            return;
        }
        tl_fwd.drop = d;
        tl_fwd.cap = n < 1024 ? 1024 : n;
    }
    void **drop = tl_fwd.drop;
    void *txb[COP_PKT_BURST_SZ + 1];
    uint32_t cnt = 0, nd = 0;
    for (uint32_t i = 0; i < n; i++) {
        void *m = objs[i];
        const uint32_t f = res[i].verdict == COP_FORWARD;
        txb[cnt] = m;
        drop[nd] = m;
        cnt += f;
        nd += 1u - f;
        if (cnt == COP_PKT_BURST_SZ || (i + 1 == n && cnt)) {
            uint32_t sent = cop_ring_enqueue_bulk(tx, txb, cnt, NULL);
            for (uint32_t k = sent; k < cnt; k++) drop[nd++] = txb[k];   /* a burst that does not fit */
            if (stats) {
                stats->tx_packets += sent;
                stats->tx_dropped += cnt - sent;
            }
            cnt = 0;
        }
    }
    if (free_fn)
        for (uint32_t k = 0; k < nd; k++) free_fn((struct rte_mbuf *)drop[k], free_arg);
}

/* dequeue up to max_pkts from rx (switch.c:463 dequeues PKT_BURST_SZ per
 * coprocessor() call; one GPU batch takes many such bursts, so dequeue
 * POLL_BURST at a time: the same packets in the same order, fewer
 * ring-index exchanges) and resolve each mbuf's data address */
static uint32_t drain_rx(cop_ring *rx, void **objs, const void **data, uint32_t max_pkts)
{
    enum { POLL_BURST = 8 * COP_PKT_BURST_SZ };
    uint32_t n = 0;
    while (n < max_pkts) {
        uint32_t want = max_pkts - n < POLL_BURST ? max_pkts - n : POLL_BURST;
        uint32_t got = cop_ring_dequeue_burst(rx, objs + n, want, NULL);
        n += got;
        if (got < want) break;
    }
    for (uint32_t i = 0; i < n; i++) {
        if (i + 16 < n) __builtin_prefetch((const uint8_t *)objs[i + 16] + g_buf_addr_off);
        data[i] = mbuf_data((struct rte_mbuf *)objs[i]);
    }
    return n;
}

int cop_coprocessor_poll(cop_ctx *ctx, cop_ring *rx, cop_ring *tx, uint32_t max_pkts,
                         cop_free_fn free_fn, void *free_arg, cop_nf_stats *stats)
{
    if (!ctx || !rx || !tx) return -EINVAL;
    if (max_pkts == 0) max_pkts = COP_PKT_BURST_SZ;
    /* refuse before dequeuing anything: a batch the context cannot take
     * would strand every mbuf it dequeued */
    if (max_pkts > cop_ctx_max_batch(ctx)) return -EINVAL;
    if (ensure_buf(max_pkts)) return -ENOMEM;
    const int prof = prof_on();
    uint64_t t0 = prof ? prof_ns() : 0;
    const uint32_t n = drain_rx(rx, tl_buf.objs, tl_buf.data, max_pkts);
    if (prof) {
        const uint64_t t1 = prof_ns();
        tl_prof[PROF_DRAIN] += t1 - t0;
        tl_prof[PROF_CALLS]++;
        t0 = t1;
    }
    if (n == 0) return 0;
    int rc = cop_process_host_stages(ctx, g_dropin_stages, tl_buf.data, n, tl_buf.res, NULL, NULL);
    if (rc) {
        drop_all(tl_buf.objs, n, free_fn, free_arg, stats);
        return rc;
    }
    if (prof) {
        const uint64_t t1 = prof_ns();
        tl_prof[PROF_BATCH] += t1 - t0;
        t0 = t1;
    }
    forward_batch(tx, tl_buf.objs, tl_buf.res, n, free_fn, free_arg, stats);
    if (prof) {
        tl_prof[PROF_FWD] += prof_ns() - t0;
        tl_prof[PROF_BUSY_CALLS]++;
        tl_prof[PROF_PKTS] += n;
    }
    return (int)n;
}

static int async_complete_oldest(cop_ctx *ctx, cop_ring *tx, cop_free_fn free_fn, void *free_arg,
                                 cop_nf_stats *stats)
{
    const uint32_t s = tl_async.fifo[0];
    const cop_result *res = NULL;
    uint32_t n = 0;
    const int prof = prof_on();
    uint64_t t0 = prof ? prof_ns() : 0;
    int rc = cop_host_batch_wait(ctx, s, &res, &n);
    if (prof) {
        const uint64_t t1 = prof_ns();
        tl_prof[PROF_WAIT] += t1 - t0;
        t0 = t1;
    }
    for (uint32_t i = 1; i < tl_async.depth; i++) tl_async.fifo[i - 1] = tl_async.fifo[i];
    tl_async.depth--;
    if (rc) {
        /* no verdicts for this batch: its mbufs are freed, never leaked */
        drop_all(tl_async.objs[s], tl_async.n[s], free_fn, free_arg, stats);
        tl_async.n[s] = 0;
        return rc;
    }
    forward_batch(tx, tl_async.objs[s], res, n, free_fn, free_arg, stats);
    tl_async.n[s] = 0;
    if (prof) {
        tl_prof[PROF_FWD] += prof_ns() - t0;
        tl_prof[PROF_PKTS] += n;
    }
    return (int)n;
}

int cop_coprocessor_poll_async(cop_ctx *ctx, cop_ring *rx, cop_ring *tx, uint32_t max_pkts,
                               cop_free_fn free_fn, void *free_arg, cop_nf_stats *stats)
{
    if (!ctx || !rx || !tx) return -EINVAL;
    if (max_pkts == 0) max_pkts = COP_PKT_BURST_SZ;
    if (max_pkts > cop_ctx_max_batch(ctx)) return -EINVAL;   /* before any dequeue */
    if (tl_async.depth && tl_async.ctx != ctx) return -EBUSY; /* flush the other context first */
    int done = 0;
    /* a free slot: complete the oldest batch if every slot is in flight */
    if (tl_async.depth == COP_HOST_SLOTS) {
        int r = async_complete_oldest(ctx, tx, free_fn, free_arg, stats);
        if (r < 0) return r;
        done += r;
    }
    uint32_t s = 0;
    for (; s < COP_HOST_SLOTS; s++) {
        int used = 0;
        for (uint32_t i = 0; i < tl_async.depth; i++) used |= tl_async.fifo[i] == s;
        if (!used) break;
    }
    if (tl_async.cap[s] < max_pkts) {
        void **o = (void **)realloc(tl_async.objs[s], max_pkts * sizeof(void *));
        if (!o) return -ENOMEM;
        tl_async.objs[s] = o;
        tl_async.cap[s] = max_pkts;
    }
    if (tl_async.data_cap < max_pkts) {
        const void **d = (const void **)realloc((void *)tl_async.data, max_pkts * sizeof(void *));
        if (!d) return -ENOMEM;
        tl_async.data = d;
        tl_async.data_cap = max_pkts;
    }
    const int prof = prof_on();
    uint64_t t0 = prof ? prof_ns() : 0;
    const uint32_t n = drain_rx(rx, tl_async.objs[s], tl_async.data, max_pkts);
    if (prof) {
        const uint64_t t1 = prof_ns();
        tl_prof[PROF_DRAIN] += t1 - t0;
        tl_prof[PROF_CALLS]++;
        tl_prof[PROF_BUSY_CALLS] += n != 0;
        t0 = t1;
    }
    if (n) {
        int rc = cop_host_batch_submit_stages(ctx, g_dropin_stages, s, tl_async.data, n);
        if (rc) {
            drop_all(tl_async.objs[s], n, free_fn, free_arg, stats);
            return rc;
        }
        if (prof) tl_prof[PROF_BATCH] += prof_ns() - t0;
        tl_async.n[s] = n;
        tl_async.ctx = ctx;
        tl_async.fifo[tl_async.depth++] = s;
    }
    /* complete the previous batch now (it ran while this one was gathered),
     * or the only one in flight when rx had nothing new */
    if (tl_async.depth > 1 || (n == 0 && tl_async.depth == 1)) {
        int r = async_complete_oldest(ctx, tx, free_fn, free_arg, stats);
        if (r < 0) return r;
        done += r;
    }
    return done;
}

int cop_coprocessor_flush(cop_ctx *ctx, cop_ring *tx, cop_free_fn free_fn, void *free_arg, cop_nf_stats *stats)
{
    if (!ctx || !tx) return -EINVAL;
    if (tl_async.depth && tl_async.ctx != ctx) return -EINVAL;
    int done = 0, err = 0;
    while (tl_async.depth) {
        int r = async_complete_oldest(ctx, tx, free_fn, free_arg, stats);
        if (r < 0) {
            if (!err) err = r;   /* keep completing: every held mbuf is forwarded or freed */
            continue;
        }
        done += r;
    }
    return err ? err : done;
}

/* ---- the drop-in ring loop on one shared poll-mode kernel ---------------
 * The reference runs one coprocessor lcore per vport, each polling its own
 * rx ring (main.c:92-94, switch.c:463). Here ONE poll-mode kernel serves
 * every such thread's ring: ring r's batches are the 16-byte header records
 * of one drain of rx ring r, gathered into mapped pinned host memory (the
 * kernel reads them over PCIe and writes its records back there), posted
 * with their packet count; no launch per batch. */
struct cop_pmd_host {
    cop_ctx *ctx;
    cop_pmd *pmd;
    uint32_t n_rings, n_slots, max_pkts;
    uint32_t slot_pkts;       /* max_pkts rounded up to even: the slot stride (16-byte aligned record slots) */
    uint8_t *h_stage;         /* [ring][slot][slot_pkts] 16-byte header records (mapped) */
    cop_result *h_res;        /* [ring][slot][slot_pkts] result records (mapped) */
    struct {
        void **objs;          /* [slot][slot_pkts] the mbufs each slot in flight holds */
        const void **data;    /* [max_pkts] the data addresses of one drain */
        uint32_t *n;          /* [slot] mbufs held */
        uint64_t head;        /* the ring's oldest batch in flight (its sequence number) */
    } ring[COP_PMD_MAX_RINGS];
};

int cop_pmd_host_destroy(cop_pmd_host *h)
{
    if (!h) return -EINVAL;
    int rc = h->pmd ? cop_pmd_stop(h->pmd) : 0;
    if (h->h_stage) cop_host_free_pinned(h->ctx, h->h_stage);
    if (h->h_res) cop_host_free_pinned(h->ctx, h->h_res);
    for (uint32_t r = 0; r < COP_PMD_MAX_RINGS; r++) {
        free(h->ring[r].objs);
        free((void *)h->ring[r].data);
        free(h->ring[r].n);
    }
    free(h);
    return rc;
}

int cop_pmd_host_create(cop_ctx *ctx, uint32_t n_rings, uint32_t max_pkts, uint32_t n_slots, cop_pmd_host **out)
{
    if (!ctx || !out || n_rings < 1 || n_rings > COP_PMD_MAX_RINGS || max_pkts < 1 || n_slots < 1) return -EINVAL;
    if (max_pkts > cop_ctx_max_batch(ctx)) return -EINVAL;
    *out = NULL;
    cop_pmd_host *h = (cop_pmd_host *)calloc(1, sizeof(*h));
    if (!h) return -ENOMEM;
    h->ctx = ctx;
    h->n_rings = n_rings;
    h->n_slots = n_slots;
    /* the ring's batches hold at most max_pkts (<= max_batch); its slots are
     * an even number of records apart (16-byte aligned record slots) */
    h->max_pkts = max_pkts;
    const uint32_t sp = h->slot_pkts = (max_pkts + 1u) & ~1u;
    const size_t recs = (size_t)n_rings * n_slots * sp;
    void *d_stage = NULL, *d_res = NULL;
    int rc = cop_host_alloc_mapped(ctx, recs * COP_HDR16_STRIDE, (void **)&h->h_stage, &d_stage);
    if (!rc) rc = cop_host_alloc_mapped(ctx, recs * sizeof(cop_result), (void **)&h->h_res, &d_res);
    cop_batch_ring rings[COP_PMD_MAX_RINGS];
    for (uint32_t r = 0; !rc && r < n_rings; r++) {
        h->ring[r].objs = (void **)calloc((size_t)n_slots * sp, sizeof(void *));
        h->ring[r].data = (const void **)calloc(max_pkts, sizeof(void *));
        h->ring[r].n = (uint32_t *)calloc(n_slots, sizeof(uint32_t));
        if (!h->ring[r].objs || !h->ring[r].data || !h->ring[r].n) rc = -ENOMEM;
        memset(&rings[r], 0, sizeof(rings[r]));
        rings[r].pkts = (uint8_t *)d_stage + (size_t)r * n_slots * sp * COP_HDR16_STRIDE;
        rings[r].n_slots = n_slots;
        rings[r].n = max_pkts;
        rings[r].stride = COP_HDR16_STRIDE;
        rings[r].pkts_slot_bytes = (uint64_t)sp * COP_HDR16_STRIDE;
        rings[r].results = (cop_result *)d_res + (size_t)r * n_slots * sp;
        rings[r].results_slot = sp;
    }
    if (!rc) rc = cop_pmd_start_rings_stages(ctx, rings, n_rings, COP_PMD_VARIABLE_N, g_dropin_stages, &h->pmd);
    if (rc) {
        cop_pmd_host_destroy(h);
        return rc;
    }
    *out = h;
    return 0;
}

/* complete ring r's oldest batch in flight: forward / free its mbufs */
static int pmd_host_complete(cop_pmd_host *h, uint32_t r, cop_ring *tx, cop_free_fn free_fn, void *free_arg,
                             cop_nf_stats *stats)
{
    const uint64_t b = h->ring[r].head;
    const uint32_t slot = (uint32_t)(b % h->n_slots);
    void **objs = h->ring[r].objs + (size_t)slot * h->slot_pkts;
    const uint32_t n = h->ring[r].n[slot];
    const int prof = prof_on();
    uint64_t t0 = prof ? prof_ns() : 0;
    int rc = cop_pmd_wait_ring(h->pmd, r, b + 1);
    if (prof) {
        const uint64_t t1 = prof_ns();
        tl_prof[PROF_WAIT] += t1 - t0;
        t0 = t1;
    }
    h->ring[r].head = b + 1;
    h->ring[r].n[slot] = 0;
    if (rc) {
        drop_all(objs, n, free_fn, free_arg, stats);   /* no verdicts: freed, never leaked */
        return rc;
    }
    const cop_result *res = h->h_res + ((size_t)r * h->n_slots + slot) * h->slot_pkts;
    forward_batch(tx, objs, res, n, free_fn, free_arg, stats);
    if (prof) {
        tl_prof[PROF_FWD] += prof_ns() - t0;
        tl_prof[PROF_PKTS] += n;
    }
    return (int)n;
}

int cop_coprocessor_poll_pmd(cop_pmd_host *h, uint32_t r, cop_ring *rx, cop_ring *tx, uint32_t max_pkts,
                             cop_free_fn free_fn, void *free_arg, cop_nf_stats *stats)
{
    if (!h || r >= h->n_rings || !rx || !tx) return -EINVAL;
    if (max_pkts == 0) max_pkts = COP_PKT_BURST_SZ;
    if (max_pkts > h->max_pkts) return -EINVAL;   /* before any dequeue */
    int done = 0;
    uint64_t posted = cop_pmd_posted_ring(h->pmd, r);
    /* a free slot: complete the oldest batch if every slot is in flight */
    if (posted - h->ring[r].head == h->n_slots) {
        int c = pmd_host_complete(h, r, tx, free_fn, free_arg, stats);
        if (c < 0) return c;
        done += c;
    }
    const uint32_t slot = (uint32_t)(posted % h->n_slots);
    void **objs = h->ring[r].objs + (size_t)slot * h->slot_pkts;
    const int prof = prof_on();
    uint64_t t0 = prof ? prof_ns() : 0;
    const uint32_t n = drain_rx(rx, objs, h->ring[r].data, max_pkts);
    if (prof) {
        const uint64_t t1 = prof_ns();
        tl_prof[PROF_DRAIN] += t1 - t0;
        tl_prof[PROF_CALLS]++;
        tl_prof[PROF_BUSY_CALLS] += n != 0;
        t0 = t1;
    }
    if (n) {
        cop_pack_headers(h->ring[r].data, n,
                         h->h_stage + (((size_t)r * h->n_slots + slot) * h->slot_pkts) * COP_HDR16_STRIDE);
        int rc = cop_pmd_post_batch(h->pmd, r, n);
        if (rc) {
            drop_all(objs, n, free_fn, free_arg, stats);
            return rc;
        }
        h->ring[r].n[slot] = n;
        posted++;
        if (prof) tl_prof[PROF_BATCH] += prof_ns() - t0;
    }
    /* complete, oldest first, every batch already done; with rx empty, the
     * oldest in flight too (waiting for it) */
    while (posted > h->ring[r].head) {
        if (cop_pmd_completed_ring(h->pmd, r) <= h->ring[r].head && n != 0) break;
        int c = pmd_host_complete(h, r, tx, free_fn, free_arg, stats);
        if (c < 0) return c;
        done += c;
        if (n == 0) break;
    }
    return done;
}

int cop_coprocessor_flush_pmd(cop_pmd_host *h, uint32_t r, cop_ring *tx, cop_free_fn free_fn, void *free_arg,
                              cop_nf_stats *stats)
{
    if (!h || r >= h->n_rings || !tx) return -EINVAL;
    int done = 0, err = 0;
    while (cop_pmd_posted_ring(h->pmd, r) > h->ring[r].head) {
        int c = pmd_host_complete(h, r, tx, free_fn, free_arg, stats);
        if (c < 0) {
            if (!err) err = c;   /* keep completing: every held mbuf is forwarded or freed */
            continue;
        }
        done += c;
    }
    return err ? err : done;
}
