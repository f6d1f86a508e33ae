/*
 * lpm_trie.c — the multibit-trie device form of an LPM table: a 12-bit top
 * level staged in LDS, then popcount-compressed 6-bit nodes that stay
 * resident in the XCD's L2 (the rte_lpm_lookup semantics of
 * firewall.c:194 over any table size; the DIR-24-8 form needs a 64 MiB
 * tbl24 that only the Infinity Cache holds).
 *
 * Built from the table's flattened step function (the sorted, merged
 * intervals of cop_lpm_form_intervals), so every form lookup returns
 * exactly the interval value the other forms return:
 *   level 0   l0[ip >> 20]: a value (bit 31 clear) when the /12 block holds
 *             one interval, else COP_TRIE_NODE | node index;
 *   nodes     6-bit strides over address bits 19..14, 13..8, 7..2, then a
 *             2-bit last level (bits 1..0). A node is six u32:
 *             vec (u64: bit c set = child c is a node), leafvec (u64: bit c
 *             set = leaf child c starts a new run of equal leaves; a child
 *             node ends a run), child_base, leaf_base. Child c is node
 *             child_base + popcount(vec & ((2 << c) - 1)) - 1, or leaf
 *             leaves[leaf_base + popcount(leafvec & ((2 << c) - 1)) - 1].
 * The children of a node are contiguous (breadth-first allocation), so one
 * base per node suffices (the Poptrie layout: Asai & Ohara, SIGCOMM 2015).
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include "cop_internal.h"

typedef struct {
    uint32_t lo;      /* first address of the node's range */
    uint32_t level;   /* 1..4 */
    uint32_t idx;     /* node index */
} trie_work;

static const uint32_t SHIFT[5] = {20, 14, 8, 2, 0};   /* child index = (ip >> SHIFT[l]) & mask */
static const uint32_t STRIDE[5] = {12, 6, 6, 6, 2};

/* index of the interval holding ip: the last start <= ip */
static uint32_t iv_find(const uint32_t *s, uint32_t m, uint32_t ip)
{
    uint32_t lo = 0, hi = m;   /* s[0] == 0 <= ip */
    while (hi - lo > 1) {
        const uint32_t mid = lo + (hi - lo) / 2;
        if (s[mid] <= ip) lo = mid;
        else hi = mid;
    }
    return lo;
}

/* the value of [a, a + len - 1] if the step function is constant there */
static int iv_const(const uint32_t *s, const uint32_t *v, uint32_t m, uint32_t a, uint64_t len, uint32_t *val)
{
    const uint32_t k = iv_find(s, m, a);
    *val = v[k];
    return k + 1 == m || (uint64_t)s[k + 1] > (uint64_t)a + len - 1;
}

static int grow(void **p, size_t *cap, size_t need, size_t elem)
{
    if (need <= *cap) return 0;
    size_t c = *cap ? *cap : 1024;
    while (c < need) c *= 2;
    void *q = realloc(*p, c * elem);
    if (!q) return -ENOMEM;
    *p = q;
    *cap = c;
    return 0;
}

int cop_lpm_trie_build(const uint32_t *starts, const uint32_t *vals, uint32_t m, cop_lpm_trie *out)
{
    if (!starts || !vals || !m || !out || starts[0] != 0) return -EINVAL;
    memset(out, 0, sizeof(*out));
    for (uint32_t k = 0; k < m; k++)
        if (vals[k] & COP_TRIE_NODE) return -ERANGE;   /* values use bits 0..30 */
    uint32_t *nodes = NULL, *leaves = NULL;
    trie_work *q = NULL;
    size_t cap_n = 0, cap_l = 0, cap_q = 0;
    uint32_t n_nodes = 0, n_leaves = 0;
    size_t qh = 0, qt = 0;
    int rc = 0;
    /* level 0: one entry per /12 block */
    for (uint32_t t = 0; t < COP_TRIE_L0; t++) {
        uint32_t val;
        if (iv_const(starts, vals, m, t << 20, 1ull << 20, &val)) {
            out->l0[t] = val;
        } else {
            if ((rc = grow((void **)&q, &cap_q, qt + 1, sizeof(*q)))) goto fail;
            q[qt++] = (trie_work){t << 20, 1, n_nodes};
            out->l0[t] = COP_TRIE_NODE | n_nodes;
            n_nodes++;
        }
    }
    /* nodes breadth-first: a node's child nodes take the next free indices */
    while (qh < qt) {
        const trie_work w = q[qh++];
        const uint32_t sb = STRIDE[w.level], sh = SHIFT[w.level];
        const uint64_t span = 1ull << sh;   /* addresses per child */
        uint64_t vec = 0, leafvec = 0;
        const uint32_t child_base = n_nodes, leaf_base = n_leaves;
        int prev_leaf = 0;
        uint32_t prev_val = 0;
        uint32_t k = iv_find(starts, m, w.lo);   /* advanced child by child */
        for (uint32_t c = 0; c < (1u << sb); c++) {
            const uint32_t a = w.lo + (uint32_t)(c * span);
            while (k + 1 < m && starts[k + 1] <= a) k++;
            const uint32_t val = vals[k];
            if (k + 1 == m || (uint64_t)starts[k + 1] > (uint64_t)a + span - 1) {
                if (!prev_leaf || val != prev_val) {
                    leafvec |= 1ull << c;
                    if ((rc = grow((void **)&leaves, &cap_l, (size_t)n_leaves + 1, 4))) goto fail;
                    leaves[n_leaves++] = val;
                }
                prev_leaf = 1;
                prev_val = val;
            } else {
                vec |= 1ull << c;
                if ((rc = grow((void **)&q, &cap_q, qt + 1, sizeof(*q)))) goto fail;
                q[qt++] = (trie_work){a, w.level + 1, n_nodes};
                n_nodes++;
                prev_leaf = 0;
            }
        }
        if ((rc = grow((void **)&nodes, &cap_n, (size_t)(w.idx + 1) * COP_TRIE_NODE_WORDS, 4))) goto fail;
        uint32_t *nd = nodes + (size_t)w.idx * COP_TRIE_NODE_WORDS;
        nd[0] = (uint32_t)vec;
        nd[1] = (uint32_t)(vec >> 32);
        nd[2] = (uint32_t)leafvec;
        nd[3] = (uint32_t)(leafvec >> 32);
        nd[4] = child_base;
        nd[5] = leaf_base;
        if (n_nodes >= COP_TRIE_NODE) { rc = -E2BIG; goto fail; }
    }
    free(q);
    out->n_nodes = n_nodes;
    out->n_leaves = n_leaves;
    out->nodes = nodes;
    out->leaves = leaves;
    if (!out->nodes) out->nodes = (uint32_t *)calloc(COP_TRIE_NODE_WORDS, 4);   /* a trie of level 0 only */
    if (!out->leaves) out->leaves = (uint32_t *)calloc(1, 4);
    if (!out->nodes || !out->leaves) {
        cop_lpm_trie_free(out);
        return -ENOMEM;
    }
    return 0;
fail:
    free(q);
    free(nodes);
    free(leaves);
    memset(out, 0, sizeof(*out));
    return rc;
}

void cop_lpm_trie_free(cop_lpm_trie *t)
{
    if (!t) return;
    free(t->nodes);
    free(t->leaves);
    t->nodes = t->leaves = NULL;
    t->n_nodes = t->n_leaves = 0;
}

static inline uint32_t popc64(uint64_t x) { return (uint32_t)__builtin_popcountll(x); }

/* The device walk, on the host (tests): the value of ip. */
uint32_t cop_lpm_trie_lookup(const cop_lpm_trie *t, uint32_t ip)
{
    uint32_t e = t->l0[ip >> 20];
    for (uint32_t l = 1; l <= 4 && (e & COP_TRIE_NODE); l++) {
        const uint32_t *nd = t->nodes + (size_t)(e & ~COP_TRIE_NODE) * COP_TRIE_NODE_WORDS;
        const uint64_t vec = nd[0] | (uint64_t)nd[1] << 32, lv = nd[2] | (uint64_t)nd[3] << 32;
        const uint32_t c = (ip >> SHIFT[l]) & ((1u << STRIDE[l]) - 1u);
        const uint64_t upto = c == 63 ? ~0ull : (2ull << c) - 1ull;
        if ((vec >> c) & 1ull) e = COP_TRIE_NODE | (nd[4] + popc64(vec & upto) - 1u);
        else e = t->leaves[nd[5] + popc64(lv & upto) - 1u];
    }
    return e;
}

/* Build the trie of a table's device form and run lookups (tests: the host
 * walk against the interval values, and the sizes). Returns 0 or -errno. */
int cop_lpm_trie_probe(const cop_lpm_table *tab, int form, const uint32_t *ips, uint32_t n, uint32_t *out,
                       uint32_t *ref, uint32_t *n_nodes, uint32_t *n_leaves)
{
    uint32_t *s = NULL, *v = NULL;
    const uint32_t m = cop_lpm_form_intervals(tab, form, &s, &v);
    if (!s) return -ENOMEM;
    cop_lpm_trie t;
    int rc = cop_lpm_trie_build(s, v, m, &t);
    if (!rc && ref)   /* the same lookups by binary search over the intervals */
        for (uint32_t i = 0; i < n; i++) ref[i] = v[iv_find(s, m, ips[i])];
    free(s);
    free(v);
    if (rc) return rc;
    for (uint32_t i = 0; i < n; i++) out[i] = cop_lpm_trie_lookup(&t, ips[i]);
    if (n_nodes) *n_nodes = t.n_nodes;
    if (n_leaves) *n_leaves = t.n_leaves;
    cop_lpm_trie_free(&t);
    return 0;
}
