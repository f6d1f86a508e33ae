/*
 * ringbench.c — rate of the drop-in ring loop: the
 * reference's fast path -> coprocessor -> tx path with the GPU as the
 * coprocessor, through the C ABI only.
 *
 * Each of L independent loops has the reference's three roles, one thread
 * each (switch.c runs one coprocessor lcore per vport, main.c:92-94):
 *   fast path:    enqueues mbuf pointers into its rx_q in all-or-nothing
 *                 bursts of 32 (rte_ring_enqueue_bulk, switch.c:225-234),
 *                 retrying while the ring is full;
 *   coprocessor:  its own context (coprocessor_setup, thread-local);
 *                 cop_coprocessor_poll or the pipelined
 *                 cop_coprocessor_poll_async drains up to max_pkts, runs a
 *                 GPU batch, forwards FORWARD packets to tx_q in arrival
 *                 order and frees drops (coprocessor(), switch.c:443-474);
 *   tx:           drains tx_q in bursts of 32.
 * Rings have the reference's 16384 slots (NF_QUEUE_RINGSIZE, init.h:54).
 * mbufs are DPDK-shaped (buf_addr at 0, data_off at 16, 2176 B data room,
 * 128 B headroom, init.h:38-44), a pool of 131072 per loop.
 *
 * usage: ringbench <packets per loop> <max_pkts per poll> <loops> [async|pmd]
 *   pmd: every loop's coprocessor thread posts to its own ring of ONE
 *        poll-mode kernel (cop_pmd_host_create, cop_coprocessor_poll_pmd)
 *        instead of launching per batch on its own context
 * prints one line: the aggregate Mpkt/s, per-loop rate and batch size;
 * exit 0 when every packet came out of every loop (forwarded + freed).
 * Build: make -C tools ringbench
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "cop_gpu.h"

/* diagnostics of the library (not in the public header) */
int cop_debug_dropin_prof(uint64_t *out, uint32_t n, int reset);
int cop_debug_host_prof(cop_ctx *c, uint64_t *out, uint32_t n, int reset);

#define NB_MBUF 131072u
#define STRIDE 2176u
#define HEADROOM 128u
#define MAX_LOOPS 16

typedef struct fake_mbuf {
    void *buf_addr;     /* offset 0  */
    uint64_t buf_iova;  /* offset 8  */
    uint16_t data_off;  /* offset 16 */
    uint8_t pad[46];
} fake_mbuf;

typedef struct loop {
    cop_ring *rx, *tx;
    fake_mbuf *mb;
    uint8_t *data;
    uint64_t n_total, processed, polls, freed;
    uint64_t prof[7], hprof[6];   /* $COP_HOST_PROF=1: per-op host ns (cop_debug_*_prof) */
    _Alignas(64) _Atomic uint64_t n_tx;   /* the tx thread's: its own line */
    atomic_int done, ready;
    int rc;
    uint32_t id;
} loop;

static uint32_t g_max_pkts;
static int g_async;
static int g_pmd;                 /* loops share one poll-mode kernel, ring l per loop */
static cop_pmd_host *g_ph;
static char g_rules[64];
static atomic_int g_go;

static void pin_to(int k);

static void free_mbuf(struct rte_mbuf *m, void *arg)
{
    (void)m;
    ((loop *)arg)->freed++;   /* called on the coprocessor thread only */
}

static void *fastpath(void *arg)
{
    loop *L = arg;
    pin_to(3 * (int)L->id);
    void *burst[COP_PKT_BURST_SZ];
    while (!atomic_load(&g_go)) {
    }
    for (uint64_t i = 0; i < L->n_total; i += COP_PKT_BURST_SZ) {
        uint32_t k = (uint32_t)(L->n_total - i < COP_PKT_BURST_SZ ? L->n_total - i : COP_PKT_BURST_SZ);
        for (uint32_t j = 0; j < k; j++) burst[j] = &L->mb[(i + j) % NB_MBUF];
        while (cop_ring_enqueue_bulk(L->rx, burst, k, NULL) == 0) __builtin_ia32_pause();
    }
    return NULL;
}

static void *txdrain(void *arg)
{
    loop *L = arg;
    pin_to(3 * (int)L->id + 2);
    void *burst[COP_PKT_BURST_SZ];
    for (;;) {
        uint32_t got = cop_ring_dequeue_burst(L->tx, burst, COP_PKT_BURST_SZ, NULL);
        if (got) {
            atomic_fetch_add_explicit(&L->n_tx, got, memory_order_relaxed);
        } else if (atomic_load(&L->done)) {
            if (cop_ring_count(L->tx) == 0) break;
        } else {
            __builtin_ia32_pause();
        }
    }
    return NULL;
}

static int poll_once(cop_ctx *ctx, loop *L, cop_nf_stats *st)
{
    if (g_pmd) return cop_coprocessor_poll_pmd(g_ph, L->id, L->rx, L->tx, g_max_pkts, free_mbuf, L, st);
    return g_async ? cop_coprocessor_poll_async(ctx, L->rx, L->tx, g_max_pkts, free_mbuf, L, st)
                   : cop_coprocessor_poll(ctx, L->rx, L->tx, g_max_pkts, free_mbuf, L, st);
}

static void *coprocessor(void *arg)
{
    loop *L = arg;
    pin_to(3 * (int)L->id + 1);
    if (!g_pmd && coprocessor_setup() != 0) {
        L->rc = 4;
        atomic_store(&L->done, 1);
        atomic_store(&L->ready, 1);
        return NULL;
    }
    cop_ctx *ctx = coprocessor_ctx();   /* (pmd: unused, the loops share the main thread's kernel) */
    cop_nf_stats st;
    memset(&st, 0, sizeof(st));
    /* warm-up: one small batch through the loop (allocations, first launch) */
    void *w[COP_PKT_BURST_SZ];
    for (uint32_t j = 0; j < COP_PKT_BURST_SZ; j++) w[j] = &L->mb[j];
    cop_ring_enqueue_bulk(L->rx, w, COP_PKT_BURST_SZ, NULL);
    for (uint64_t warm = 0; warm < COP_PKT_BURST_SZ;) {
        int r = poll_once(ctx, L, &st);
        if (r < 0) {
            L->rc = 9;
            break;
        }
        warm += (uint64_t)r;
    }
    while (cop_ring_dequeue_burst(L->tx, w, COP_PKT_BURST_SZ, NULL)) {
    }
    L->freed = 0;
    atomic_store(&L->ready, 1);
    while (!atomic_load(&g_go)) {
    }
    while (L->rc == 0 && L->processed < L->n_total) {
        int r = poll_once(ctx, L, &st);
        if (r < 0) {
            fprintf(stderr, "poll: %d %s\n", r, cop_last_error(ctx));
            L->rc = 10;
            break;
        }
        if (r > 0) L->polls++;
        L->processed += (uint64_t)r;
    }
    if (g_async && L->rc == 0) cop_coprocessor_flush(ctx, L->tx, free_mbuf, L, &st);
    if (g_pmd && L->rc == 0) cop_coprocessor_flush_pmd(g_ph, L->id, L->tx, free_mbuf, L, &st);
    atomic_store(&L->done, 1);
    cop_debug_dropin_prof(L->prof, 7, 1);
    if (!g_pmd) {
        cop_debug_host_prof(ctx, L->hprof, 6, 1);
        coprocessor_teardown();
    }
    return NULL;
}

/* Pin the calling thread to the k-th CPU this process may use, counting
 * from the 5th (the first few also serve interrupts and the main thread):
 * DPDK lcores are pinned, and a loop's three threads on adjacent cores keep
 * the ring transfers between them inside one CCD ($RINGBENCH_PIN=0: off). */
static void pin_to(int k)
{
    const char *e = getenv("RINGBENCH_PIN");
    if (e && !atoi(e)) return;
    cpu_set_t all;
    if (sched_getaffinity(0, sizeof(all), &all)) return;
    int seen = 0;
    for (int c = 0; c < CPU_SETSIZE; c++) {
        if (!CPU_ISSET(c, &all)) continue;
        if (seen++ == k + 4) {
            cpu_set_t one;
            CPU_ZERO(&one);
            CPU_SET(c, &one);
            pthread_setaffinity_np(pthread_self(), sizeof(one), &one);
            return;
        }
    }
}

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

int main(int argc, char **argv)
{
    if (argc < 4) {
        fprintf(stderr, "usage: %s packets_per_loop max_pkts loops [async]\n", argv[0]);
        return 2;
    }
    const uint64_t per_loop = strtoull(argv[1], NULL, 0);
    g_max_pkts = (uint32_t)strtoul(argv[2], NULL, 0);
    const int nl = atoi(argv[3]);
    g_async = argc > 4 && strcmp(argv[4], "async") == 0;
    g_pmd = argc > 4 && strcmp(argv[4], "pmd") == 0;
    if (nl < 1 || nl > MAX_LOOPS || (g_pmd && nl > COP_PMD_MAX_RINGS)) return 2;

    /* rules.json in the reference format, read by the reference's setup path */
    cop_prefix *rules = calloc(1000, sizeof(cop_prefix));
    if (!rules || cop_gen_rules(0x5EED1002, 1000, COP_GEN_FW, 20, rules) != 0) return 3;
    snprintf(g_rules, sizeof(g_rules), "/tmp/ringbench_rules_%d.json", (int)getpid());
    if (cop_rules_write_json(g_rules, rules, 1000) != 0) return 3;
    cop_set_rule_file(g_rules);   /* process-wide, before any coprocessor thread */
    cop_set_mbuf_layout(0, 16);

    if (g_pmd) {
        /* one context (the main thread's) and one kernel for every loop */
        if (coprocessor_setup() != 0) return 4;
        int prc = cop_pmd_host_create(coprocessor_ctx(), (uint32_t)nl, g_max_pkts, 4, &g_ph);
        if (prc) {
            fprintf(stderr, "cop_pmd_host_create: %d %s\n", prc, cop_last_error(coprocessor_ctx()));
            return 4;
        }
    }
    uint8_t *trace = malloc((size_t)NB_MBUF * 64);
    if (!trace || cop_gen_trace(0x5EED0002, NB_MBUF, NULL, rules, 1000, NULL, 0, trace, 64) != 0) return 7;
    static loop loops[MAX_LOOPS];
    pthread_t th[MAX_LOOPS][3];
    for (int l = 0; l < nl; l++) {
        loop *L = &loops[l];
        L->n_total = per_loop;
        L->id = (uint32_t)l;
        L->data = malloc((size_t)NB_MBUF * STRIDE);
        L->mb = calloc(NB_MBUF, sizeof(fake_mbuf));
        L->rx = cop_ring_create(COP_NF_QUEUE_RINGSIZE);
        L->tx = cop_ring_create(COP_NF_QUEUE_RINGSIZE);
        if (!L->data || !L->mb || !L->rx || !L->tx) return 6;
        for (uint32_t i = 0; i < NB_MBUF; i++) {
            memcpy(L->data + (size_t)i * STRIDE + HEADROOM, trace + (size_t)i * 64, 64);
            L->mb[i].buf_addr = L->data + (size_t)i * STRIDE;
            L->mb[i].data_off = HEADROOM;
        }
        pthread_create(&th[l][0], NULL, coprocessor, L);
    }
    for (int l = 0; l < nl; l++)
        while (!atomic_load(&loops[l].ready)) usleep(1000);
    for (int l = 0; l < nl; l++) {
        pthread_create(&th[l][1], NULL, fastpath, &loops[l]);
        pthread_create(&th[l][2], NULL, txdrain, &loops[l]);
    }
    const double t0 = now();
    atomic_store(&g_go, 1);
    for (int l = 0; l < nl; l++) pthread_join(th[l][0], NULL);
    const double dt = now() - t0;
    int rc = 0;
    uint64_t total = 0, polls = 0;
    for (int l = 0; l < nl; l++) {
        loop *L = &loops[l];
        if (L->rc) {
            /* a loop that never started leaves its fast path waiting on a
             * full ring: report and exit without joining it */
            fprintf(stderr, "loop %d failed: %d\n", l, L->rc);
            remove(g_rules);
            return L->rc;
        }
        pthread_join(th[l][1], NULL);
        pthread_join(th[l][2], NULL);
        if (atomic_load(&L->n_tx) + L->freed != L->n_total) rc = 11;
        total += L->processed;
        polls += L->polls;
    }
    remove(g_rules);
    if (g_pmd) {
        cop_pmd_host_destroy(g_ph);
        coprocessor_teardown();
    }
    if (getenv("COP_HOST_PROF")) {
        /* loop 0's host time per packet, by op (ns/pkt), and per busy call (us) */
        loop *L = &loops[0];
        const double pk = L->prof[6] ? (double)L->prof[6] : 1.0;
        const double calls = L->prof[5] ? (double)L->prof[5] : 1.0;
        printf("prof loop0 %s: ns/pkt drain %.2f batch %.2f wait %.2f fwd %.2f | calls %llu busy %llu pkts %llu "
               "(%.0f pkts/busy call, %.1f us/busy call) | host batch ns/pkt gather %.2f launch %.2f wait %.2f "
               "copy %.2f (%llu batches, %.1f us launch/batch, %.1f us wait/batch)\n",
               g_pmd ? "pmd" : g_async ? "async" : "sync", L->prof[0] / pk, L->prof[1] / pk, L->prof[2] / pk, L->prof[3] / pk,
               (unsigned long long)L->prof[4], (unsigned long long)L->prof[5], (unsigned long long)L->prof[6],
               L->prof[6] / calls, (L->prof[0] + L->prof[1] + L->prof[2] + L->prof[3]) / calls / 1e3,
               L->hprof[0] / pk, L->hprof[1] / pk, L->hprof[2] / pk, L->hprof[3] / pk,
               (unsigned long long)L->hprof[4], L->hprof[4] ? L->hprof[1] / (double)L->hprof[4] / 1e3 : 0.0,
               L->hprof[4] ? L->hprof[2] / (double)L->hprof[4] / 1e3 : 0.0);
    }
    printf("%s loops %2d max_pkts %6u  %8.1f Mpkt/s aggregate (%.1f per loop), %.0f pkts per poll\n",
           g_pmd ? "pmd  " : g_async ? "async" : "sync ", nl, g_max_pkts, (double)total / dt / 1e6, (double)total / dt / 1e6 / nl,
           polls ? (double)total / (double)polls : 0.0);
    return rc;
}
