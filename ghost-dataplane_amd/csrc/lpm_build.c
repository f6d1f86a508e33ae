/*
 * lpm_build.c — host-side LPM table builder with DPDK rte_lpm semantics.
 *
 * The reference builds its firewall table in lpm_setup (firewall.c:215-255)
 * by calling rte_lpm_create(max_rules=1024, number_tbl8s=24) and then
 * rte_lpm_add(ip, depth, action) per rule, in file order. DPDK is not
 * vendored; the semantics restated here are those of
 * DPDK 17.11 librte_lpm (v1604 ABI, the range the reference's API usage
 * pins: 17.11 <= v <= 19.05):
 *
 *   - depth outside 1..32                       -> -EINVAL, table unchanged
 *   - ip is masked to depth
 *   - (masked ip, depth) already held           -> next hop overwritten
 *                                                  (last write wins), 0
 *   - new rule when max_rules distinct held     -> -ENOSPC
 *   - new depth>24 rule whose /24 has no tbl8
 *     group yet when all groups are in use     -> -ENOSPC, table unchanged
 *   - lookups: exact longest-prefix match over the held rules; miss -> nh 0
 *
 * DPDK adds one rule at a time into its DIR-24-8 image and scans rule
 * groups linearly (O(n^2) at 1M rules). This builder instead decides
 * acceptance with a hash table, then flattens the accepted set into
 * disjoint address intervals with one sorted sweep (O(n log n)), and
 * paints the DIR-24-8 image from the intervals in one pass over 2^24
 * entries. The result is the same lookup function (nh, hit) as DPDK's
 * incremental image; tests/test_lpm_host.py checks it against the
 * oracle's incremental restatement.
 */
#include <errno.h>
#include <stdlib.h>
#include <string.h>

#include "cop_internal.h"

static inline uint32_t depth_mask(uint32_t depth)
{
    return depth == 0 ? 0u : (uint32_t)(0xFFFFFFFFull << (32 - depth));
}

static inline uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* open-addressing map: key (u64, never ~0) -> u32 */
typedef struct {
    uint64_t *keys;
    uint32_t *vals;
    uint64_t  cap; /* power of two */
} umap;

#define UMAP_EMPTY (~0ull)

static int umap_init(umap *m, uint64_t want)
{
    uint64_t cap = 16;
    while (cap < want * 2) cap <<= 1;
    m->keys = (uint64_t *)malloc(cap * sizeof(uint64_t));
    m->vals = (uint32_t *)malloc(cap * sizeof(uint32_t));
    if (!m->keys || !m->vals) {
        free(m->keys);
        free(m->vals);
        return -ENOMEM;
    }
    memset(m->keys, 0xFF, cap * sizeof(uint64_t));
    m->cap = cap;
    return 0;
}

static void umap_free(umap *m)
{
    free(m->keys);
    free(m->vals);
}

/* returns pointer to value slot; *found tells whether the key existed */
static uint32_t *umap_slot(umap *m, uint64_t key, int *found)
{
    uint64_t i = mix64(key) & (m->cap - 1);
    for (;;) {
        if (m->keys[i] == key) {
            *found = 1;
            return &m->vals[i];
        }
        if (m->keys[i] == UMAP_EMPTY) {
            *found = 0;
            return &m->vals[i];
        }
        i = (i + 1) & (m->cap - 1);
    }
}

static void umap_commit(umap *m, uint32_t *slot, uint64_t key)
{
    m->keys[slot - m->vals] = key;
}

typedef struct {
    uint32_t ip;
    uint32_t val;
    uint32_t rule;
    uint8_t  depth;
} srule;

static int srule_cmp(const void *a, const void *b)
{
    const srule *x = (const srule *)a, *y = (const srule *)b;
    if (x->ip != y->ip) return x->ip < y->ip ? -1 : 1;
    return (int)x->depth - (int)y->depth;
}

typedef struct {
    uint32_t *start;
    uint32_t *val;
    uint32_t  n;
} ivbuf;

static void iv_emit(ivbuf *b, uint64_t pos, uint32_t val)
{
    if (pos >= (1ull << 32)) return;
    if (b->n && b->start[b->n - 1] == (uint32_t)pos) {
        b->val[b->n - 1] = val;
        if (b->n >= 2 && b->val[b->n - 2] == val) b->n--;
        return;
    }
    if (b->n && b->val[b->n - 1] == val) return;
    b->start[b->n] = (uint32_t)pos;
    b->val[b->n] = val;
    b->n++;
}

/* /24 blocks with an interval boundary strictly inside need a tbl8 group */
static uint32_t count_ext(const uint32_t *start, uint32_t n)
{
    uint32_t n_ext = 0, last_blk = 0xFFFFFFFFu;
    for (uint32_t k = 0; k < n; k++) {
        uint32_t st = start[k];
        if ((st & 0xFFu) != 0 && (st >> 8) != last_blk) {
            n_ext++;
            last_blk = st >> 8;
        }
    }
    return n_ext;
}

void cop_lpm_free(cop_lpm_table *t)
{
    if (!t) return;
    free(t->rule_ip);
    free(t->rule_depth);
    free(t->rule_nh);
    free(t->iv_start);
    free(t->iv_val);
    free(t->rv_start);
    free(t->rv_rule);
    free(t);
}

int cop_lpm_build(const cop_prefix *rules, uint32_t n, const cop_lpm_config *cfg,
                  cop_lpm_table **out, cop_lpm_report *report)
{
    cop_lpm_config dflt = {COP_FW_MAX_RULES, COP_FW_NUMBER_TBL8S, COP_LPM_STOP_AT_FIRST_ERROR};
    if (!out || (n && !rules)) return -EINVAL;
    if (!cfg) cfg = &dflt;
    *out = NULL;
    /* rte_lpm_create rejects max_rules == 0 (and number_tbl8s == 0 in 17.11) */
    if (cfg->max_rules == 0) return -EINVAL;

    cop_lpm_table *t = (cop_lpm_table *)calloc(1, sizeof(*t));
    if (!t) return -ENOMEM;
    cop_lpm_report *rep = &t->report;
    rep->n_in = n;

    uint32_t cap_rules = n < cfg->max_rules ? n : cfg->max_rules;
    t->rule_ip = (uint32_t *)malloc((size_t)(cap_rules ? cap_rules : 1) * sizeof(uint32_t));
    t->rule_depth = (uint8_t *)malloc((size_t)(cap_rules ? cap_rules : 1));
    t->rule_nh = (uint32_t *)malloc((size_t)(cap_rules ? cap_rules : 1) * sizeof(uint32_t));
    umap rmap, pmap;
    int rc = 0;
    if (!t->rule_ip || !t->rule_depth || !t->rule_nh) rc = -ENOMEM;
    if (!rc && (rc = umap_init(&rmap, cap_rules + 1)) == 0) {
        if ((rc = umap_init(&pmap, (cfg->number_tbl8s < cap_rules ? cfg->number_tbl8s : cap_rules) + 1)) != 0)
            umap_free(&rmap);
    }
    if (rc) {
        cop_lpm_free(t);
        return rc;
    }

    /* ---- acceptance: sequential rte_lpm_add semantics ---- */
    for (uint32_t i = 0; i < n; i++) {
        const cop_prefix *r = &rules[i];
        int err = 0;
        uint32_t depth = r->depth;
        if (depth < 1 || depth > COP_LPM_MAX_DEPTH) {
            err = -EINVAL;
        } else {
            uint32_t ipm = r->ip & depth_mask(depth);
            uint64_t key = ((uint64_t)depth << 32) | ipm;
            int found;
            uint32_t *slot = umap_slot(&rmap, key, &found);
            if (found) {
                /* rule_add: existing rule -> next_hop updated, then the
                 * table paint overwrites entries of this depth. */
                t->rule_nh[*slot] = r->next_hop & COP_LPM_NH_MASK;
                rep->n_updated++;
            } else if (t->n_rules >= cfg->max_rules) {
                err = -ENOSPC;
            } else {
                int need_group = 0;
                uint32_t *pslot = NULL;
                uint64_t pkey = ipm >> 8;
                if (depth > 24) {
                    int pfound;
                    pslot = umap_slot(&pmap, pkey, &pfound);
                    if (!pfound) {
                        if (t->tbl8_used >= cfg->number_tbl8s) err = -ENOSPC;
                        else need_group = 1;
                    }
                }
                if (!err) {
                    if (need_group) {
                        umap_commit(&pmap, pslot, pkey);
                        *pslot = t->tbl8_used++;
                    }
                    umap_commit(&rmap, slot, key);
                    *slot = t->n_rules;
                    t->rule_ip[t->n_rules] = ipm;
                    t->rule_depth[t->n_rules] = (uint8_t)depth;
                    t->rule_nh[t->n_rules] = r->next_hop & COP_LPM_NH_MASK;
                    t->n_rules++;
                }
            }
        }
        if (err) {
            rep->n_failed++;
            if (!rep->first_error) {
                rep->first_error = err;
                rep->first_error_idx = i;
            }
            if (cfg->flags & COP_LPM_STOP_AT_FIRST_ERROR) {
                rep->n_skipped = n - i - 1;
                break;
            }
        } else {
            rep->n_added++;
        }
    }
    umap_free(&rmap);
    umap_free(&pmap);
    rep->n_distinct = t->n_rules;
    rep->tbl8_used = t->tbl8_used;

    /* ---- flatten: sorted sweep over nested prefixes ---- */
    srule *s = (srule *)malloc((size_t)(t->n_rules ? t->n_rules : 1) * sizeof(srule));
    uint32_t ivcap = 2 * t->n_rules + 2;
    t->iv_start = (uint32_t *)malloc((size_t)ivcap * sizeof(uint32_t));
    t->iv_val = (uint32_t *)malloc((size_t)ivcap * sizeof(uint32_t));
    t->rv_start = (uint32_t *)malloc((size_t)ivcap * sizeof(uint32_t));
    t->rv_rule = (uint32_t *)malloc((size_t)ivcap * sizeof(uint32_t));
    if (!s || !t->iv_start || !t->iv_val || !t->rv_start || !t->rv_rule) {
        free(s);
        cop_lpm_free(t);
        return -ENOMEM;
    }
    for (uint32_t i = 0; i < t->n_rules; i++) {
        s[i].ip = t->rule_ip[i];
        s[i].depth = t->rule_depth[i];
        s[i].val = t->rule_nh[i] | COP_IV_HIT | ((uint32_t)t->rule_depth[i] << COP_IV_DEPTH_SH);
        s[i].rule = i;
    }
    qsort(s, t->n_rules, sizeof(srule), srule_cmp);

    /* one sweep feeds two interval sets: keyed by value (nh, hit, depth)
     * and keyed by the matching rule (the firewall's rule-id image) */
    ivbuf b = {t->iv_start, t->iv_val, 1};
    ivbuf br = {t->rv_start, t->rv_rule, 1};
    b.start[0] = br.start[0] = 0;
    b.val[0] = 0;
    br.val[0] = COP_NO_RULE;
    struct {
        uint64_t end;
        uint32_t val, rule;
    } stk[COP_LPM_MAX_DEPTH + 2];
    int sp = 0;
    for (uint32_t i = 0; i < t->n_rules; i++) {
        uint64_t st = s[i].ip;
        uint64_t en = st + (1ull << (32 - s[i].depth)) - 1;
        while (sp > 0 && stk[sp - 1].end < st) {
            sp--;
            iv_emit(&b, stk[sp].end + 1, sp ? stk[sp - 1].val : 0u);
            iv_emit(&br, stk[sp].end + 1, sp ? stk[sp - 1].rule : COP_NO_RULE);
        }
        iv_emit(&b, st, s[i].val);
        iv_emit(&br, st, s[i].rule);
        stk[sp].end = en;
        stk[sp].val = s[i].val;
        stk[sp].rule = s[i].rule;
        sp++;
    }
    while (sp > 0) {
        sp--;
        iv_emit(&b, stk[sp].end + 1, sp ? stk[sp - 1].val : 0u);
        iv_emit(&br, stk[sp].end + 1, sp ? stk[sp - 1].rule : COP_NO_RULE);
    }
    free(s);
    t->n_iv = b.n;
    t->n_rv = br.n;
    t->n_ext = count_ext(t->iv_start, t->n_iv);
    t->n_ext_rule = count_ext(t->rv_start, t->n_rv);

    uint32_t *ms = NULL, *mv = NULL;
    rep->n_intervals = cop_lpm_merged_intervals(t, &ms, &mv);
    free(ms);
    free(mv);
    if (report) *report = *rep;
    *out = t;
    return 0;
}

uint32_t cop_lpm_merged_intervals(const cop_lpm_table *t, uint32_t **starts, uint32_t **vals)
{
    uint32_t *s = (uint32_t *)malloc((size_t)t->n_iv * sizeof(uint32_t));
    uint32_t *v = (uint32_t *)malloc((size_t)t->n_iv * sizeof(uint32_t));
    uint32_t m = 0;
    if (!s || !v) {
        free(s);
        free(v);
        *starts = *vals = NULL;
        return 0;
    }
    for (uint32_t k = 0; k < t->n_iv; k++) {
        uint32_t val = t->iv_val[k] & COP_IV_NHHIT;
        if (m && v[m - 1] == val) continue;
        s[m] = t->iv_start[k];
        v[m] = val;
        m++;
    }
    *starts = s;
    *vals = v;
    return m;
}

static inline uint32_t dir_entry(uint32_t ival)
{
    if (!(ival & COP_IV_HIT)) return 0u;
    return ival & ~0x02000000u; /* nh | valid | depth<<26 */
}

static inline uint32_t rule_entry(const cop_lpm_table *t, uint32_t rule)
{
    if (rule == COP_NO_RULE) return 0u;
    return rule | COP_DIR_VALID | (t->rule_nh[rule] ? COP_RV_DROP : 0u);
}

/* Paint tbl24/tbl8 from intervals (start[], entry[]) in one pass over the
 * 2^24 /24 blocks; blocks with an interior boundary get the next tbl8 group. */
static void fill_dir24(const uint32_t *start, const uint32_t *entry, uint32_t niv, uint32_t *tbl24,
                       uint32_t *tbl8)
{
    uint32_t k = 0, g = 0;
    for (uint32_t blk = 0; blk < (1u << 24); blk++) {
        uint64_t lo = (uint64_t)blk << 8, hi = lo + 255;
        while (k + 1 < niv && start[k + 1] <= lo) k++;
        uint64_t next = (k + 1 < niv) ? start[k + 1] : (1ull << 32);
        if (next > hi) {
            tbl24[blk] = entry[k];
            continue;
        }
        /* extended: paint the 256 addresses of this /24 from the intervals */
        uint32_t kk = k;
        uint32_t *grp = tbl8 + (size_t)g * 256;
        for (uint32_t a = 0; a < 256; a++) {
            uint64_t addr = lo + a;
            while (kk + 1 < niv && start[kk + 1] <= addr) kk++;
            grp[a] = entry[kk];
        }
        tbl24[blk] = g | COP_DIR_VALID_EXT;
        g++;
    }
}

/* device entries of a form, one per (unmerged) interval */
static uint32_t *form_entries(const cop_lpm_table *t, int form, const uint32_t **start, uint32_t *n)
{
    uint32_t cnt = form == COP_FORM_RULE ? t->n_rv : t->n_iv;
    uint32_t *e = (uint32_t *)malloc((size_t)(cnt ? cnt : 1) * sizeof(uint32_t));
    if (!e) return NULL;
    for (uint32_t k = 0; k < cnt; k++)
        e[k] = form == COP_FORM_RULE ? rule_entry(t, t->rv_rule[k]) : dir_entry(t->iv_val[k]);
    *start = form == COP_FORM_RULE ? t->rv_start : t->iv_start;
    *n = cnt;
    return e;
}

void cop_lpm_fill_dir24(const cop_lpm_table *t, uint32_t *tbl24, uint32_t *tbl8)
{
    cop_lpm_form_fill_dir24(t, COP_FORM_NH, tbl24, tbl8);
}

void cop_lpm_form_fill_dir24(const cop_lpm_table *t, int form, uint32_t *tbl24, uint32_t *tbl8)
{
    const uint32_t *start;
    uint32_t n;
    uint32_t *e = form_entries(t, form, &start, &n);
    if (!e) {   /* allocation failure: a table of misses (callers check n_ext) */
        memset(tbl24, 0, sizeof(uint32_t) << 24);
        return;
    }
    fill_dir24(start, e, n, tbl24, tbl8);
    free(e);
}

uint32_t cop_lpm_form_n_ext(const cop_lpm_table *t, int form)
{
    return form == COP_FORM_RULE ? t->n_ext_rule : t->n_ext;
}

uint32_t cop_lpm_form_intervals(const cop_lpm_table *t, int form, uint32_t **starts, uint32_t **entries)
{
    if (form != COP_FORM_RULE) {
        /* NH form: merged (nh | hit) values, as the interval export */
        return cop_lpm_merged_intervals(t, starts, entries);
    }
    uint32_t *s = (uint32_t *)malloc((size_t)(t->n_rv ? t->n_rv : 1) * sizeof(uint32_t));
    uint32_t *v = (uint32_t *)malloc((size_t)(t->n_rv ? t->n_rv : 1) * sizeof(uint32_t));
    if (!s || !v) {
        free(s);
        free(v);
        *starts = *entries = NULL;
        return 0;
    }
    for (uint32_t k = 0; k < t->n_rv; k++) {
        s[k] = t->rv_start[k];
        v[k] = rule_entry(t, t->rv_rule[k]);
    }
    *starts = s;
    *entries = v;
    return t->n_rv;
}

int cop_lpm_lookup_rules(const cop_lpm_table *t, const uint32_t *ips, uint32_t n, int32_t *rule_id)
{
    if (!t || (n && (!ips || !rule_id))) return -EINVAL;
    for (uint32_t i = 0; i < n; i++) {
        /* last interval with start <= ip (rv_start[0] == 0) */
        uint32_t lo = 0, hi = t->n_rv;
        while (hi - lo > 1) {
            uint32_t mid = lo + (hi - lo) / 2;
            if (t->rv_start[mid] <= ips[i]) lo = mid;
            else hi = mid;
        }
        rule_id[i] = t->rv_rule[lo] == COP_NO_RULE ? -1 : (int32_t)t->rv_rule[lo];
    }
    return 0;
}

int cop_lpm_export_dir24(const cop_lpm_table *t, uint32_t *tbl24, uint32_t *tbl8,
                         uint32_t tbl8_cap_entries)
{
    if (!t || !tbl24) return -EINVAL;
    if ((uint64_t)t->n_ext * 256 > tbl8_cap_entries || (t->n_ext && !tbl8)) return -ENOSPC;
    cop_lpm_fill_dir24(t, tbl24, tbl8);
    return (int)t->n_ext;
}

int cop_lpm_export_intervals(const cop_lpm_table *t, uint32_t *starts, uint32_t *values,
                             uint32_t cap)
{
    if (!t) return -EINVAL;
    uint32_t *s, *v;
    uint32_t m = cop_lpm_merged_intervals(t, &s, &v);
    if (!s) return -ENOMEM;
    int rc = (int)m;
    if (m > cap) {
        rc = -ENOSPC;
    } else if (starts && values) {
        memcpy(starts, s, (size_t)m * sizeof(uint32_t));
        memcpy(values, v, (size_t)m * sizeof(uint32_t));
    }
    free(s);
    free(v);
    return rc;
}

int cop_lpm_export_rules(const cop_lpm_table *t, cop_prefix *out, uint32_t cap)
{
    if (!t) return -EINVAL;
    if (!out) return (int)t->n_rules;
    if (t->n_rules > cap) return -ENOSPC;
    for (uint32_t i = 0; i < t->n_rules; i++) {
        memset(&out[i], 0, sizeof(out[i]));
        out[i].ip = t->rule_ip[i];
        out[i].depth = t->rule_depth[i];
        out[i].next_hop = t->rule_nh[i];
    }
    return (int)t->n_rules;
}
