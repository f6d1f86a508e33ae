/* Bucketed interval device form of an LPM table (COP_CFG_LPM_BKT): the
 * route stage's lookup for tables too large for the LDS interval form, kept
 * in global memory small enough to stay in L2 / the Infinity Cache.
 *
 * An LPM table flattens to sorted, merged (start, value) intervals (the form
 * the LDS search and the DIR-24-8 image are pinned to: rte_lpm_lookup
 * semantics, firewall.c:194). The answer for ip is the value of R(ip), the
 * last interval whose start <= ip. The address space is cut into 2^ib
 * buckets of its top ib bits (ib = ceil(log2 m) + xbits, 12..22); idx[b] = R(b << (32 - ib)) and idx[2^ib] =
 * m - 1. For ip in bucket b, R(ip) lies in [idx[b], idx[b + 1]]. With
 * 2^ib >= m a bucket holds about one boundary, so the kernel's two rounds
 * (cop_device.h bkt_issue / bkt_step) decide almost every lookup:
 *   1. one 8-byte load {idx[b], idx[b + 1]} = {k0, k1};
 *   2. one 64-byte read of pairs k0 .. k0 + 7: the answer when the bucket
 *      holds at most 7 boundaries (k1 <= k0 + 7) or ip lies below start
 *      k0 + 7;
 *   otherwise a scan on over pairs k0 + 8 .. k1, two (one 16-byte load) a round.
 * Pairs past the end are pads {0xFFFFFFFF, last value}: only ip 0xFFFFFFFF
 * reaches one, and its answer is the last interval's value. */
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include "cop_internal.h"

int cop_lpm_bkt_build(const uint32_t *s, const uint32_t *v, uint32_t m, uint32_t xbits, cop_lpm_bkt *out)
{
    memset(out, 0, sizeof(*out));
    if (!m || xbits > 8) return -EINVAL;
    uint32_t ib = 0;
    while (ib < 31 && (1u << ib) < m) ib++;
    ib += xbits;   /* 2^xbits buckets per interval: fewer wide buckets, a larger index */
    if (ib < COP_BKT_MIN_BITS) ib = COP_BKT_MIN_BITS;
    if (ib > COP_BKT_MAX_BITS) ib = COP_BKT_MAX_BITS;
    const uint32_t nb = 1u << ib;
    out->idx = (uint32_t *)malloc(((size_t)nb + 1) * 4);
    out->pairs = (uint32_t *)malloc(2 * ((size_t)m + COP_BKT_PADS) * 4);
    if (!out->idx || !out->pairs) {
        cop_lpm_bkt_free(out);
        return -ENOMEM;
    }
    for (uint32_t k = 0; k < m + COP_BKT_PADS; k++) {
        out->pairs[2 * (size_t)k] = k < m ? s[k] : 0xFFFFFFFFu;
        out->pairs[2 * (size_t)k + 1] = k < m ? v[k] : v[m - 1];
    }
    uint32_t k = 0, widest = 0;
    for (uint32_t b = 0; b <= nb; b++) {
        const uint64_t x = b == nb ? 0xFFFFFFFFull : (uint64_t)b << (32 - ib);
        while (k + 1 < m && s[k + 1] <= x) k++;
        out->idx[b] = k;
        if (b && out->idx[b] - out->idx[b - 1] > widest) widest = out->idx[b] - out->idx[b - 1];
    }
    uint32_t lv = 0;
    while ((1u << lv) <= widest) lv++;
    out->m = m;
    out->ib = ib;
    out->lv = lv;
    out->widest = widest;
    return 0;
}

void cop_lpm_bkt_free(cop_lpm_bkt *t)
{
    free(t->idx);
    free(t->pairs);
    memset(t, 0, sizeof(*t));
}

/* The kernel's rounds (cop_device.h bkt_step) on the host (tests); *rounds
 * += the wide-bucket rounds this lookup needed */
uint32_t cop_lpm_bkt_lookup(const cop_lpm_bkt *t, uint32_t ip, uint32_t *rounds)
{
    const uint32_t b = ip >> (32u - t->ib);
    const uint32_t k0 = t->idx[b], k1 = t->idx[b + 1];
    const uint32_t *q = t->pairs + 2 * (size_t)k0;
    uint32_t e = q[1];
    for (uint32_t i = 1; i < 8; i++)   /* pairs k0 .. k0 + 7: one 64-byte read */
        if (i <= k1 - k0 && ip >= q[2 * i]) e = q[2 * i + 1];
    if (!(k1 - k0 > 7u && ip >= q[14])) return e;
    for (uint32_t j = k0 + 8u;; j += 2u) {   /* the wide bucket: two pairs a round */
        const uint32_t *a = t->pairs + 2 * (size_t)j;
        if (rounds) (*rounds)++;
        for (uint32_t i = 0; i < 2; i++)
            if (j + i <= k1 && ip >= a[2 * i]) e = a[2 * i + 1];
        if (!(j + 1u < k1 && ip >= a[2])) return e;
    }
}

int cop_lpm_bkt_probe(const cop_lpm_table *tab, int form, uint32_t xbits, const uint32_t *ips, uint32_t n,
                      uint32_t *out, uint32_t *ref, uint32_t *info)
{
    uint32_t *s = NULL, *v = NULL;
    const uint32_t m = cop_lpm_form_intervals(tab, form, &s, &v);
    if (!s) return -ENOMEM;
    cop_lpm_bkt t;
    int rc = cop_lpm_bkt_build(s, v, m, xbits, &t);
    if (!rc && ref)   /* the same lookups by binary search over all intervals */
        for (uint32_t i = 0; i < n; i++) {
            uint32_t lo = 0, hi = m - 1;
            while (lo < hi) {
                const uint32_t mid = lo + (hi - lo + 1) / 2;
                if (s[mid] <= ips[i]) lo = mid;
                else hi = mid - 1;
            }
            ref[i] = v[lo];
        }
    free(s);
    free(v);
    if (rc) return rc;
    uint32_t lifted = 0, rounds = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t r0 = rounds;
        out[i] = cop_lpm_bkt_lookup(&t, ips[i], &rounds);
        lifted += rounds != r0;
    }
    if (info) {   /* m, ib, lv, widest bucket, lookups that needed a wide-bucket round, those rounds */
        info[0] = t.m;
        info[1] = t.ib;
        info[2] = t.lv;
        info[3] = t.widest;
        info[4] = lifted;
        info[5] = rounds;
    }
    cop_lpm_bkt_free(&t);
    return 0;
}
