/*
 * dropin.c — the reference's coprocessor API on top of the GPU context.
 *
 *   coprocessor_setup    coprocessor.c:21-35  (setup_rules + lpm_setup)
 *   coprocessor_teardown coprocessor.c:37-49
 *   process_packet       coprocessor.c:50-65  (0 forward / -1 drop)
 *   cop_coprocessor_poll switch.c:443-474     (coprocessor() loop body)
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

#include "cop_gpu.h"

static uint32_t g_buf_addr_off = 0;   /* rte_mbuf.buf_addr (DPDK 17.11-19.05) */
static uint32_t g_data_off_off = 16;  /* rte_mbuf.data_off */
static char g_rule_file[4096] = "./nfs/firewall/rules.json"; /* coprocessor.c:19 */
static int g_rule_file_set = 0;

static __thread cop_ctx *tl_ctx = NULL;
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

cop_ctx *coprocessor_ctx(void)
{
    return tl_ctx;
}

int coprocessor_setup(void)
{
    if (tl_ctx) return 0;
    cop_config cfg;
    cop_config_default(&cfg);
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

int coprocessor_teardown(void)
{
    if (tl_ctx) cop_destroy(tl_ctx);
    tl_ctx = NULL;
    free(tl_buf.objs);
    free(tl_buf.data);
    free(tl_buf.res);
    memset(&tl_buf, 0, sizeof(tl_buf));
    return 0;
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
    int rc = cop_process_host(tl_ctx, tl_buf.data, n, tl_buf.res, NULL, NULL);
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

int cop_coprocessor_poll(cop_ctx *ctx, cop_ring *rx, cop_ring *tx, uint32_t max_pkts,
                         cop_free_fn free_fn, void *free_arg, cop_nf_stats *stats)
{
    if (!ctx || !rx || !tx) return -EINVAL;
    if (max_pkts == 0) max_pkts = COP_PKT_BURST_SZ;
    if (ensure_buf(max_pkts)) return -ENOMEM;
    /* drain rx_q in bursts of PKT_BURST_SZ (switch.c:463) */
    uint32_t n = 0;
    while (n < max_pkts) {
        uint32_t want = max_pkts - n < COP_PKT_BURST_SZ ? max_pkts - n : COP_PKT_BURST_SZ;
        uint32_t got = cop_ring_dequeue_burst(rx, tl_buf.objs + n, want, NULL);
        n += got;
        if (got < want) break;
    }
    if (n == 0) return 0;
    for (uint32_t i = 0; i < n; i++) tl_buf.data[i] = mbuf_data((struct rte_mbuf *)tl_buf.objs[i]);
    int rc = cop_process_host(ctx, tl_buf.data, n, tl_buf.res, NULL, NULL);
    if (rc) return rc;
    /* forward in arrival order through a PKT_BURST_SZ tx buffer flushed with
     * an all-or-nothing bulk enqueue (enqueue_nf_tx / flush_nf_tx_queue,
     * switch.c:240-280,329-351); drops are freed (switch.c:469). */
    void *txb[COP_PKT_BURST_SZ];
    uint32_t cnt = 0;
    for (uint32_t i = 0; i <= n; i++) {
        int flush = (i == n) ? cnt > 0 : 0;
        if (i < n) {
            struct rte_mbuf *m = (struct rte_mbuf *)tl_buf.objs[i];
            if (tl_buf.res[i].verdict == COP_FORWARD) {
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
    return (int)n;
}
