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
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

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
 * switch.c:240-280,329-351); drops are freed (switch.c:469). */
static void forward_batch(cop_ring *tx, void *const *objs, const cop_result *res, uint32_t n, cop_free_fn free_fn,
                          void *free_arg, cop_nf_stats *stats)
{
    void *txb[COP_PKT_BURST_SZ];
    uint32_t cnt = 0;
    for (uint32_t i = 0; i <= n; i++) {
        int flush = (i == n) ? cnt > 0 : 0;
        if (i < n) {
            struct rte_mbuf *m = (struct rte_mbuf *)objs[i];
            if (res[i].verdict == COP_FORWARD) {
                txb[cnt++] = m;
                flush = cnt == COP_PKT_BURST_SZ;
            } else if (free_fn) {
                free_fn(m, free_arg);
            }
        }
        if (flush) {
            uint32_t sent = cop_ring_enqueue_bulk(tx, txb, cnt, NULL);
            if (sent < cnt && free_fn)
                for (uint32_t k = sent; k < cnt; k++) free_fn((struct rte_mbuf *)txb[k], free_arg);
            if (stats) {
                stats->tx_packets += sent;
                stats->tx_dropped += cnt - sent;
            }
            cnt = 0;
        }
    }
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
    const uint32_t n = drain_rx(rx, tl_buf.objs, tl_buf.data, max_pkts);
    if (n == 0) return 0;
    int rc = cop_process_host_stages(ctx, g_dropin_stages, tl_buf.data, n, tl_buf.res, NULL, NULL);
    if (rc) {
        drop_all(tl_buf.objs, n, free_fn, free_arg, stats);
        return rc;
    }
    forward_batch(tx, tl_buf.objs, tl_buf.res, n, free_fn, free_arg, stats);
    return (int)n;
}

static int async_complete_oldest(cop_ctx *ctx, cop_ring *tx, cop_free_fn free_fn, void *free_arg,
                                 cop_nf_stats *stats)
{
    const uint32_t s = tl_async.fifo[0];
    const cop_result *res = NULL;
    uint32_t n = 0;
    int rc = cop_host_batch_wait(ctx, s, &res, &n);
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
    const uint32_t n = drain_rx(rx, tl_async.objs[s], tl_async.data, max_pkts);
    if (n) {
        int rc = cop_host_batch_submit_stages(ctx, g_dropin_stages, s, tl_async.data, n);
        if (rc) {
            drop_all(tl_async.objs[s], n, free_fn, free_arg, stats);
            return rc;
        }
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
