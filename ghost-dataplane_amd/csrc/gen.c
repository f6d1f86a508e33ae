/*
 * gen.c — deterministic synthetic rules and packet traces.
 *
 * The reference has no traffic generator of its own (its traffic came from
 * CloudSuite containers over KNI, README.md:32), so every trace here is
 * synthetic: splitmix64 streams with fixed seeds, 64-byte Eth/IPv4/UDP
 * frames with the field offsets the reference reads (EtherType at 12,
 * version/IHL at 14, src at 26, dst at 30: switch.c:116-127,
 * firewall.c:131-156).
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include "cop_gpu.h"

static inline uint64_t sm64(uint64_t *s)
{
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static inline uint32_t rnd(uint64_t *s, uint32_t n) /* uniform-ish in [0,n) */
{
    return (uint32_t)(((sm64(s) >> 32) * (uint64_t)n) >> 32);
}

static inline uint32_t mask_of(uint32_t d)
{
    return d == 0 ? 0u : (uint32_t)(0xFFFFFFFFull << (32 - d));
}

int cop_gen_rules(uint64_t seed, uint32_t n, int kind, uint32_t n_long_parents, cop_prefix *out)
{
    if (!out && n) return -EINVAL;
    uint64_t s = seed;
    uint32_t *pool = NULL;
    if (n_long_parents) {
        pool = (uint32_t *)malloc(n_long_parents * sizeof(uint32_t));
        if (!pool) return -ENOMEM;
        for (uint32_t i = 0; i < n_long_parents; i++) pool[i] = (uint32_t)(sm64(&s) >> 40);
    }
    for (uint32_t i = 0; i < n; i++) {
        uint32_t r = rnd(&s, 100), depth;
        if (kind == COP_GEN_FW) {
            if (r < 60) depth = 24;
            else if (r < 80) depth = 16 + rnd(&s, 8);
            else if (r < 90) depth = 8 + rnd(&s, 8);
            else depth = 25 + rnd(&s, 8);
        } else {
            if (r < 55) depth = 24;
            else if (r < 80) depth = 17 + rnd(&s, 7);
            else if (r < 90) depth = 8 + rnd(&s, 9);
            else depth = 25 + rnd(&s, 8);
        }
        uint32_t ip = (uint32_t)sm64(&s);
        if (depth > 24) {
            uint32_t parent = pool ? pool[rnd(&s, n_long_parents)] : (ip >> 8);
            ip = (parent << 8) | (ip & 0xFFu);
        } else if (i > 0 && rnd(&s, 100) < 30) {
            /* nest inside an earlier, shorter prefix so the LPM has depth */
            const cop_prefix *o = &out[rnd(&s, i)];
            if (o->depth < depth) {
                uint32_t m = mask_of(o->depth);
                ip = (o->ip & m) | (ip & ~m);
            }
        }
        uint32_t nh;
        if (kind == COP_GEN_FW) nh = rnd(&s, 2) ? 1 + rnd(&s, 255) : 0;
        else nh = 1 + rnd(&s, 0xFFFFFFu);
        memset(&out[i], 0, sizeof(out[i]));
        out[i].ip = ip;
        out[i].depth = (uint8_t)depth;
        out[i].next_hop = nh;
    }
    free(pool);
    return 0;
}

void cop_trace_opts_default(cop_trace_opts *o)
{
    o->n_ports = COP_KNI_KTHREAD;
    o->pct_non_ipv4 = 2;
    o->pct_bad_version = 0;
    o->pct_unknown_dst = 5;
    o->pct_vport_dst = 60;
    o->pct_src_in_rule = 50;
}

static inline void put16(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}

static inline void put32(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t)(v >> 24);
    p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);
    p[3] = (uint8_t)v;
}

static void make_frame(uint64_t *s, const cop_trace_opts *o, const cop_prefix *fw, uint32_t n_fw,
                       const cop_prefix *rt, uint32_t n_rt, uint8_t *p, uint32_t len)
{
    /* payload first (random bytes), then the headers over it */
    for (uint32_t k = 0; k < len; k += 8) {
        uint64_t v = sm64(s);
        uint32_t c = len - k < 8 ? len - k : 8;
        memcpy(p + k, &v, c);
    }
    uint32_t et = rnd(s, 100) < o->pct_non_ipv4 ? 0x86DDu : 0x0800u;
    uint32_t ver = (et == 0x0800u && rnd(s, 100) < o->pct_bad_version) ? 0x65u : 0x45u;

    uint32_t src;
    if (n_fw && rnd(s, 100) < o->pct_src_in_rule) {
        const cop_prefix *r = &fw[rnd(s, n_fw)];
        uint32_t d = r->depth > 32 ? 32 : r->depth;
        uint32_t m = mask_of(d);
        src = (r->ip & m) | ((uint32_t)sm64(s) & ~m);
    } else {
        src = (uint32_t)sm64(s);
    }
    uint32_t dst, r = rnd(s, 100);
    uint32_t nports = o->n_ports ? o->n_ports : 1;
    if (r < o->pct_vport_dst) {
        dst = (192u << 24) | (167u << 16) | (10u << 8) | (1 + rnd(s, nports));
    } else if (r < o->pct_vport_dst + o->pct_unknown_dst) {
        dst = ((uint32_t)sm64(s) & 0xFFFF0000u) | rnd(s, 5);
    } else if (n_rt) {
        const cop_prefix *q = &rt[rnd(s, n_rt)];
        uint32_t d = q->depth > 32 ? 32 : q->depth;
        uint32_t m = mask_of(d);
        dst = (q->ip & m) | ((uint32_t)sm64(s) & ~m);
    } else {
        dst = (uint32_t)sm64(s);
    }

    put16(p + 12, et);
    p[14] = (uint8_t)ver;
    p[15] = 0;
    put16(p + 16, len - 14);
    put16(p + 18, (uint32_t)sm64(s));
    put16(p + 20, 0x4000);
    p[22] = 64;
    p[23] = 17;
    put16(p + 24, 0);
    put32(p + 26, src);
    put32(p + 30, dst);
    uint32_t sum = 0;
    for (int k = 0; k < 20; k += 2) sum += ((uint32_t)p[14 + k] << 8) | p[15 + k];
    while (sum >> 16) sum = (sum & 0xFFFF) + (sum >> 16);
    put16(p + 24, ~sum & 0xFFFF);
    uint32_t ports = (uint32_t)sm64(s);
    put16(p + 34, ports >> 16);
    put16(p + 36, ports & 0xFFFF);
    put16(p + 38, len - 34);
    put16(p + 40, 0);
}

int cop_gen_trace(uint64_t seed, uint32_t n, const cop_trace_opts *opts, const cop_prefix *fw,
                  uint32_t n_fw, const cop_prefix *routes, uint32_t n_routes, uint8_t *out,
                  uint32_t stride)
{
    cop_trace_opts d;
    if (!opts) {
        cop_trace_opts_default(&d);
        opts = &d;
    }
    if ((!out && n) || stride < 64) return -EINVAL;
    uint64_t s = seed;
    for (uint32_t i = 0; i < n; i++)
        make_frame(&s, opts, fw, n_fw, routes, n_routes, out + (size_t)i * stride, 64);
    return 0;
}

int cop_gen_imix(uint64_t seed, uint32_t n, const cop_trace_opts *opts, const cop_prefix *fw,
                 uint32_t n_fw, const cop_prefix *routes, uint32_t n_routes, uint8_t *slab,
                 uint64_t *slab_bytes, uint32_t *offsets)
{
    cop_trace_opts d;
    if (!opts) {
        cop_trace_opts_default(&d);
        opts = &d;
    }
    if (!slab_bytes) return -EINVAL;
    /* sizes from their own stream so the size layout is seed-stable */
    uint64_t ss = seed ^ 0x1D1Full;
    uint64_t off = 0;
    uint64_t s = seed;
    for (uint32_t i = 0; i < n; i++) {
        uint32_t r = rnd(&ss, 12);
        uint32_t len = r < 7 ? 64u : (r < 11 ? 594u : 1518u);
        if (slab) {
            if (off > 0xFFFFFFFFull) return -ERANGE;
            offsets[i] = (uint32_t)off;
            make_frame(&s, opts, fw, n_fw, routes, n_routes, slab + off, len);
        }
        off += (len + 63u) & ~63u;
    }
    *slab_bytes = off;
    return 0;
}
