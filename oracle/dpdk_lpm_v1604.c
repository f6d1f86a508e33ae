/*
 * dpdk_lpm_v1604.c — a LITERAL restatement of DPDK 17.11 librte_lpm's
 * v1604-ABI add path: the rule table as DPDK keeps it, not as a hash.
 *
 * TEST INFRASTRUCTURE ONLY (see cop_oracle.c's header): loaded by tests/
 * as a second checker of the product's LPM builder (csrc/lpm_build.c) and
 * of cop_oracle.c's hash-based restatement. Never linked into the product.
 *
 * DPDK is a third-party dependency of the reference that is neither
 * vendored nor pinned (its API usage bounds it to
 * 17.11..19.05; the v1604 functions below are the same across that range).
 * This file restates the published algorithm of lib/librte_lpm/rte_lpm.c,
 * function by function, in its own code:
 *
 *   dl_rule_add      rule_add_v1604      rules_tbl grouped by depth:
 *                    rule_info[depth-1] = {used_rules, first_rule}; groups
 *                    sit in depth order; a new rule goes at the end of its
 *                    group, and every deeper non-empty group is shifted by
 *                    one (its first rule copied past its end); -ENOSPC when
 *                    the insertion point or any deeper group's end is
 *                    max_rules. An empty group gets first_rule = the
 *                    insertion point BEFORE the deeper groups are checked,
 *                    so a -ENOSPC there leaves that stale first_rule behind
 *                    (it is never read while the group is empty).
 *   dl_rule_delete   rule_delete_v1604   the group's last rule fills the
 *                    hole; each deeper non-empty group moves its last rule
 *                    to just before its first and decrements first_rule.
 *   dl_tbl8_alloc    tbl8_alloc_v1604    first group whose first entry has
 *                    valid_group == 0; zeroed, valid_group set.
 *   dl_add_small     add_depth_small_v1604
 *   dl_add_big       add_depth_big_v1604 (the three tbl24 cases)
 *   dl_lpm_add       rte_lpm_add_v1604   -EINVAL for depth 0 or > 32; mask;
 *                    rule_add; paint; on a tbl8 failure, rule_delete of the
 *                    rule just added (or updated) and the error.
 *   dl_lpm_lookup    rte_lpm_lookup      tbl24, then tbl8 when valid+ext.
 *
 * Entries are the v1604 rte_lpm_tbl_entry bit-fields on a little-endian
 * host: next_hop:24 | valid:1 | valid_group:1 | depth:6.
 */
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define DL_MAX_DEPTH 32
#define DL_TBL24 (1u << 24)
#define DL_GRP 256u

typedef struct dl_entry {      /* rte_lpm_tbl_entry (v1604) */
    uint32_t next_hop : 24;
    uint32_t valid : 1;
    uint32_t valid_group : 1;
    uint32_t depth : 6;
} dl_entry;

typedef struct dl_rule {       /* rte_lpm_rule */
    uint32_t ip;
    uint32_t next_hop;
} dl_rule;

typedef struct dl_rule_info {  /* rte_lpm_rule_info */
    uint32_t used_rules;
    uint32_t first_rule;
} dl_rule_info;

typedef struct dl_lpm {
    uint32_t max_rules, number_tbl8s;
    dl_rule_info rule_info[DL_MAX_DEPTH];
    dl_entry *tbl24;
    dl_entry *tbl8;
    dl_rule *rules_tbl;
} dl_lpm;

static uint32_t depth_to_mask(uint32_t depth) { return (uint32_t)(0xFFFFFFFFull << (32 - depth)); }

dl_lpm *dl_lpm_create(uint32_t max_rules, uint32_t number_tbl8s)
{
    if (max_rules == 0) return NULL;
    dl_lpm *l = (dl_lpm *)calloc(1, sizeof(*l));
    if (!l) return NULL;
    l->max_rules = max_rules;
    l->number_tbl8s = number_tbl8s;
    l->tbl24 = (dl_entry *)calloc(DL_TBL24, sizeof(dl_entry));
    l->tbl8 = (dl_entry *)calloc((size_t)(number_tbl8s ? number_tbl8s : 1) * DL_GRP, sizeof(dl_entry));
    l->rules_tbl = (dl_rule *)calloc(max_rules, sizeof(dl_rule));
    if (!l->tbl24 || !l->tbl8 || !l->rules_tbl) {
        free(l->tbl24);
        free(l->tbl8);
        free(l->rules_tbl);
        free(l);
        return NULL;
    }
    return l;
}

void dl_lpm_free(dl_lpm *l)
{
    if (!l) return;
    free(l->tbl24);
    free(l->tbl8);
    free(l->rules_tbl);
    free(l);
}

static int32_t dl_rule_add(dl_lpm *l, uint32_t ip_masked, uint32_t depth, uint32_t next_hop)
{
    dl_rule_info *ri = l->rule_info;
    uint32_t rule_index;
    if (ri[depth - 1].used_rules > 0) {
        /* an existing rule of this (prefix, depth): last write wins */
        const uint32_t first = ri[depth - 1].first_rule, last = first + ri[depth - 1].used_rules;
        for (rule_index = first; rule_index < last; rule_index++) {
            if (l->rules_tbl[rule_index].ip == ip_masked) {
                l->rules_tbl[rule_index].next_hop = next_hop;
                return (int32_t)rule_index;
            }
        }
        if (rule_index == l->max_rules) return -ENOSPC;
    } else {
        /* the group starts where the nearest shallower non-empty one ends */
        rule_index = 0;
        for (int i = (int)depth - 1; i > 0; i--) {
            if (ri[i - 1].used_rules > 0) {
                rule_index = ri[i - 1].first_rule + ri[i - 1].used_rules;
                break;
            }
        }
        if (rule_index == l->max_rules) return -ENOSPC;
        ri[depth - 1].first_rule = rule_index;   /* stays set if the shift below fails */
    }
    /* make room: shift every deeper non-empty group up by one */
    for (int i = DL_MAX_DEPTH; i > (int)depth; i--) {
        if (ri[i - 1].first_rule + ri[i - 1].used_rules == l->max_rules) return -ENOSPC;
        if (ri[i - 1].used_rules > 0) {
            l->rules_tbl[ri[i - 1].first_rule + ri[i - 1].used_rules] = l->rules_tbl[ri[i - 1].first_rule];
            ri[i - 1].first_rule++;
        }
    }
    l->rules_tbl[rule_index].ip = ip_masked;
    l->rules_tbl[rule_index].next_hop = next_hop;
    ri[depth - 1].used_rules++;
    return (int32_t)rule_index;
}

static void dl_rule_delete(dl_lpm *l, int32_t rule_index, uint32_t depth)
{
    dl_rule_info *ri = l->rule_info;
    l->rules_tbl[rule_index] = l->rules_tbl[ri[depth - 1].first_rule + ri[depth - 1].used_rules - 1];
    for (uint32_t i = depth; i < DL_MAX_DEPTH; i++) {
        if (ri[i].used_rules > 0) {
            l->rules_tbl[ri[i].first_rule - 1] = l->rules_tbl[ri[i].first_rule + ri[i].used_rules - 1];
            ri[i].first_rule--;
        }
    }
    ri[depth - 1].used_rules--;
}

static int32_t dl_tbl8_alloc(dl_lpm *l)
{
    for (uint32_t g = 0; g < l->number_tbl8s; g++) {
        dl_entry *e = &l->tbl8[(size_t)g * DL_GRP];
        if (!e->valid_group) {
            memset(e, 0, DL_GRP * sizeof(*e));
            e->valid_group = 1;
            return (int32_t)g;
        }
    }
    return -ENOSPC;
}

static void dl_add_small(dl_lpm *l, uint32_t ip, uint32_t depth, uint32_t next_hop)
{
    const uint32_t tbl24_index = ip >> 8, tbl24_range = 1u << (24 - depth);
    for (uint32_t i = tbl24_index; i < tbl24_index + tbl24_range; i++) {
        dl_entry *e = &l->tbl24[i];
        if (!e->valid || (e->valid_group == 0 && e->depth <= depth)) {
            dl_entry n = {next_hop, 1, 0, depth};
            *e = n;
            continue;
        }
        if (e->valid_group == 1) {
            /* extended: paint the tbl8 entries this rule now covers */
            dl_entry *g = &l->tbl8[(size_t)e->next_hop * DL_GRP];
            for (uint32_t j = 0; j < DL_GRP; j++) {
                if (!g[j].valid || g[j].depth <= depth) {
                    dl_entry n = {next_hop, 1, 1, depth};
                    g[j] = n;
                }
            }
        }
    }
}

static int32_t dl_add_big(dl_lpm *l, uint32_t ip_masked, uint32_t depth, uint32_t next_hop)
{
    const uint32_t tbl24_index = ip_masked >> 8, tbl8_range = 1u << (32 - depth);
    dl_entry *t24 = &l->tbl24[tbl24_index];
    if (!t24->valid) {
        const int32_t g = dl_tbl8_alloc(l);
        if (g < 0) return g;
        const uint32_t idx = (uint32_t)g * DL_GRP + (ip_masked & 0xFF);
        for (uint32_t i = idx; i < idx + tbl8_range; i++) {
            l->tbl8[i].depth = depth;
            l->tbl8[i].next_hop = next_hop;
            l->tbl8[i].valid = 1;
        }
        dl_entry n = {(uint32_t)g, 1, 1, 0};
        *t24 = n;
    } else if (t24->valid_group == 0) {
        const int32_t g = dl_tbl8_alloc(l);
        if (g < 0) return g;
        const uint32_t start = (uint32_t)g * DL_GRP, idx = start + (ip_masked & 0xFF);
        for (uint32_t i = start; i < start + DL_GRP; i++) {   /* the /24's old value everywhere */
            l->tbl8[i].valid = 1;
            l->tbl8[i].depth = t24->depth;
            l->tbl8[i].next_hop = t24->next_hop;
        }
        for (uint32_t i = idx; i < idx + tbl8_range; i++) {
            l->tbl8[i].valid = 1;
            l->tbl8[i].depth = depth;
            l->tbl8[i].next_hop = next_hop;
        }
        dl_entry n = {(uint32_t)g, 1, 1, 0};
        *t24 = n;
    } else {
        const uint32_t idx = t24->next_hop * DL_GRP + (ip_masked & 0xFF);
        for (uint32_t i = idx; i < idx + tbl8_range; i++) {
            if (!l->tbl8[i].valid || l->tbl8[i].depth <= depth) {
                dl_entry n = {next_hop, 1, l->tbl8[i].valid_group, depth};
                l->tbl8[i] = n;
            }
        }
    }
    return 0;
}

int dl_lpm_add(dl_lpm *l, uint32_t ip, uint32_t depth, uint32_t next_hop)
{
    if (!l || depth < 1 || depth > DL_MAX_DEPTH) return -EINVAL;
    next_hop &= 0x00FFFFFFu;   /* the 24-bit next_hop field */
    const uint32_t ip_masked = ip & depth_to_mask(depth);
    const int32_t rule_index = dl_rule_add(l, ip_masked, depth, next_hop);
    if (rule_index < 0) return rule_index;
    if (depth <= 24) {
        dl_add_small(l, ip_masked, depth, next_hop);
    } else {
        const int32_t st = dl_add_big(l, ip_masked, depth, next_hop);
        if (st < 0) {
            dl_rule_delete(l, rule_index, depth);
            return st;
        }
    }
    return 0;
}

int dl_lpm_lookup(const dl_lpm *l, uint32_t ip, uint32_t *next_hop)
{
    dl_entry e = l->tbl24[ip >> 8];
    if (e.valid && e.valid_group) e = l->tbl8[(size_t)e.next_hop * DL_GRP + (ip & 0xFF)];
    *next_hop = e.next_hop;
    return e.valid ? 0 : -ENOENT;
}

void dl_lpm_lookup_batch(const dl_lpm *l, const uint32_t *ips, uint64_t n, uint32_t *nh, uint8_t *hit)
{
    for (uint64_t i = 0; i < n; i++) hit[i] = dl_lpm_lookup(l, ips[i], &nh[i]) == 0;
}

/* lpm_setup's loop (firewall.c:243-252) over this table: returns the index
 * of the first failed add (or -1) and its errno in *err; every add's return
 * code in rc[] when non-NULL (-9999 for rules never presented). */
int64_t dl_lpm_setup(dl_lpm *l, const uint32_t *ip, const uint8_t *depth, const uint32_t *nh, uint64_t n,
                     int stop_at_error, int32_t *err, int32_t *rc)
{
    int64_t first = -1;
    *err = 0;
    for (uint64_t i = 0; i < n; i++) {
        const int r = dl_lpm_add(l, ip[i], depth[i], nh[i]);
        if (rc) rc[i] = r;
        if (r < 0 && first < 0) {
            first = (int64_t)i;
            *err = r;
            if (stop_at_error) {
                if (rc)
                    for (uint64_t k = i + 1; k < n; k++) rc[k] = -9999;
                break;
            }
        }
    }
    return first;
}

uint32_t dl_lpm_n_rules(const dl_lpm *l)
{
    uint32_t n = 0;
    for (int d = 0; d < DL_MAX_DEPTH; d++) n += l->rule_info[d].used_rules;
    return n;
}

uint32_t dl_lpm_tbl8_used(const dl_lpm *l)
{
    uint32_t u = 0;
    for (uint32_t g = 0; g < l->number_tbl8s; g++) u += l->tbl8[(size_t)g * DL_GRP].valid_group;
    return u;
}

/* rule_info (32 x {used_rules, first_rule}) and the rules_tbl prefix in use */
void dl_lpm_rule_info(const dl_lpm *l, uint32_t *used, uint32_t *first)
{
    for (int d = 0; d < DL_MAX_DEPTH; d++) {
        used[d] = l->rule_info[d].used_rules;
        first[d] = l->rule_info[d].first_rule;
    }
}

int dl_lpm_rules(const dl_lpm *l, uint32_t *ip, uint8_t *depth, uint32_t *nh, uint32_t cap)
{
    uint32_t k = 0;
    for (uint32_t d = 1; d <= DL_MAX_DEPTH; d++) {
        const dl_rule_info *ri = &l->rule_info[d - 1];
        for (uint32_t r = ri->first_rule; r < ri->first_rule + ri->used_rules; r++) {
            if (k == cap) return -ENOSPC;
            ip[k] = l->rules_tbl[r].ip;
            depth[k] = (uint8_t)d;
            nh[k] = l->rules_tbl[r].next_hop;
            k++;
        }
    }
    return (int)k;
}
