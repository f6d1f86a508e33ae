/*
 * switch_dropin.c — the reference engine's call pattern, in C, against
 * libcopgpu.so through include/cop_gpu.h only (no HIP, no DPDK).
 *
 * It plays switch.c's roles around the coprocessor:
 *   main_loop:    coprocessor_setup() / coprocessor_teardown()   (switch.c:525,537)
 *   coprocessor() per packet: process_packet(mbuf)               (switch.c:465)
 *   coprocessor() per burst:  process_burst(mbufs)               (batched variant)
 *   the ring loop: fast path enqueues rte_ring bulk bursts of 32 into rx_q,
 *                  cop_coprocessor_poll() drains, forwards to tx_q in order
 *                  and frees drops                               (switch.c:443-474)
 * mbufs are laid out like DPDK 17.11's (buf_addr at 0, data_off at 16) with
 * the 2176-byte data room of init.h:38-41.
 *
 * usage: switch_dropin <rules.json> <n_packets> <out.bin>
 * out.bin: n int32 process_packet results (first min(n, 512) packets), then
 * n int32 process_burst results, then the forwarded packet indices in tx_q
 * order, preceded by their count (uint32). Exit 0 on success.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cop_gpu.h"

#define STRIDE 2176
#define HEADROOM 128

typedef struct fake_mbuf {     /* the two rte_mbuf fields the path reads */
    void *buf_addr;            /* offset 0  */
    uint64_t buf_iova;         /* offset 8  */
    uint16_t data_off;         /* offset 16 */
    uint16_t refcnt;
    uint32_t index;            /* test bookkeeping */
    uint8_t pad[40];
} fake_mbuf;

static uint64_t n_freed;
static void free_mbuf(struct rte_mbuf *m, void *arg)
{
    (void)m;
    (void)arg;
    n_freed++;
}

int main(int argc, char **argv)
{
    if (argc != 4) {
        fprintf(stderr, "usage: %s rules.json n out.bin\n", argv[0]);
        return 2;
    }
    const uint32_t n = (uint32_t)strtoul(argv[2], NULL, 0);
    cop_set_rule_file(argv[1]);
    if (coprocessor_setup() != 0) {            /* switch.c:525-526: rte_exit on failure */
        fprintf(stderr, "coprocessor_setup failed: %s\n", cop_last_error(coprocessor_ctx()));
        return 3;
    }
    /* the rule file's rules, for the trace generator */
    cop_prefix *rules = NULL;
    uint32_t nr = 0;
    if (cop_rules_load_json(argv[1], &rules, &nr) != 0) return 4;

    uint8_t *trace = malloc((size_t)n * 64);
    uint8_t *bufs = malloc((size_t)n * STRIDE);
    fake_mbuf *mb = calloc(n, sizeof(fake_mbuf));
    struct rte_mbuf **ptr = malloc((size_t)n * sizeof(*ptr));
    int *ret1 = malloc((size_t)n * sizeof(int)), *ret2 = malloc((size_t)n * sizeof(int));
    uint32_t *fwd = malloc((size_t)n * sizeof(uint32_t));
    if (!trace || !bufs || !mb || !ptr || !ret1 || !ret2 || !fwd) return 5;
    if (cop_gen_trace(0x5EED0C00, n, NULL, rules, nr, NULL, 0, trace, 64) != 0) return 6;
    for (uint32_t i = 0; i < n; i++) {
        mb[i].buf_addr = bufs + (size_t)i * STRIDE;
        mb[i].data_off = HEADROOM;
        mb[i].index = i;
        memcpy(bufs + (size_t)i * STRIDE + HEADROOM, trace + (size_t)i * 64, 64);
        ptr[i] = (struct rte_mbuf *)&mb[i];
    }

    /* 1. per packet, as coprocessor() calls it */
    const uint32_t n1 = n < 512 ? n : 512;
    for (uint32_t i = 0; i < n1; i++) ret1[i] = process_packet(ptr[i]);
    /* 2. one burst */
    if (process_burst(ptr, n, ret2) != 0) return 7;
    /* 3. the ring loop: fast path enqueues bursts of 32, the GPU coprocessor
     *    drains rx_q and fills tx_q, the fast path drains tx_q */
    cop_ring *rx = cop_ring_create(16384), *tx = cop_ring_create(16384);   /* init.c:74-75 */
    cop_nf_stats st;
    memset(&st, 0, sizeof(st));
    uint32_t next = 0, nf = 0;
    while (next < n || cop_ring_count(rx)) {
        while (next < n) {
            uint32_t k = n - next < 32 ? n - next : 32;
            if (cop_ring_enqueue_bulk(rx, (void *const *)&ptr[next], k, NULL) != k) break;
            st.rx_packets += k;          /* counted by the producer, flush_nf_rx_queue switch.c:233 */
            next += k;
        }
        if (cop_coprocessor_poll(coprocessor_ctx(), rx, tx, 65536, free_mbuf, NULL, &st) < 0) return 8;
        void *out[32];
        uint32_t got;
        while ((got = cop_ring_dequeue_burst(tx, out, 32, NULL)) != 0)
            for (uint32_t q = 0; q < got; q++) fwd[nf++] = ((fake_mbuf *)out[q])->index;
    }
    if (st.rx_packets != n || st.tx_packets != nf || n_freed + nf != n) {
        fprintf(stderr, "stats mismatch: rx %llu tx %llu fwd %u freed %llu\n", (unsigned long long)st.rx_packets,
                (unsigned long long)st.tx_packets, nf, (unsigned long long)n_freed);
        return 9;
    }
    FILE *fp = fopen(argv[3], "wb");
    if (!fp) return 10;
    fwrite(ret1, sizeof(int), n1, fp);
    fwrite(ret2, sizeof(int), n, fp);
    fwrite(&nf, sizeof(nf), 1, fp);
    fwrite(fwd, sizeof(uint32_t), nf, fp);
    fclose(fp);
    cop_ring_free(rx);
    cop_ring_free(tx);
    cop_rules_free(rules);
    if (coprocessor_teardown() != 0) return 11;   /* switch.c:537 */
    printf("switch_dropin ok: %u packets, %u forwarded, %llu freed\n", n, nf, (unsigned long long)n_freed);
    return 0;
}
