/*
 * cop_oracle.c — CPU restatement of the reference coprocessor path.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the
 * checker or as the timed CPU baseline. The product (libcopgpu.so) never
 * links or calls it.
 *
 * Parity status: PARTIALLY PINNED. The reference has no tests and no
 * golden vectors; its only fixture is
 * engine/nfs/firewall/rules.json (two accept rules), pinned in
 * tests/golden/. The reference cannot be built here (DPDK absent; building
 * it would need stand-in DPDK headers, which this project does not write),
 * so everything beyond that fixture is "parity unpinned": a restatement of
 * the reference's source, cross-checked against a second independent
 * restatement (brute-force LPM) and against the product.
 *
 * What is restated, with the reference lines it follows:
 *   orc_route_table_default  read_config          init.c:40-84
 *   orc_get_next_hop         get_next_hop         switch.c:93-136
 *   orc_fw_packet_handler    fw_packet_handler    firewall.c:170-213
 *                            (+ fw_pkt_ipv4_hdr / fw_pkt_is_ipv4 :131-168;
 *                             version != 4 is UB in the reference (NULL
 *                             deref at :193-194); defined here as a drop)
 *   orc_lpm_setup            lpm_setup            firewall.c:215-255
 *   orc_lpm_*                DPDK librte_lpm 17.11 (v1604 ABI): third-party,
 *                            not vendored, version pinned by API usage to
 *                            17.11..19.05. Restated from its
 *                            published algorithm: rule table with
 *                            last-write-wins, max_rules, DIR-24-8 with
 *                            add_depth_small / add_depth_big and first-free
 *                            tbl8 group allocation, lookup via tbl24 then tbl8.
 *   orc_process              process_packet + coprocessor() ordering
 *                            coprocessor.c:50-65, switch.c:443-474,
 *                            fast-path drop switch.c:406-410,
 *                            enqueue_nf_rx port bound switch.c:316-319
 *   orc_coprocessor_bench    the coprocessor() loop over a 16384-slot ring
 *                            of mbuf descriptors in bursts of 32
 *                            (init.h:38-54, init.c:74-75) — the timed CPU
 *                            baseline.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ---------------------------------------------------------------------- */
/* init.c:40-84 and switch.c:93-136                                        */
/* ---------------------------------------------------------------------- */

void orc_route_table_default(uint16_t *rt, uint32_t n_ports)
{
    for (uint32_t i = 0; i < 65536; i++) rt[i] = 0;
    for (uint32_t i = 0; i < n_ports; i++) rt[i] = 0xFFFF;           /* init.c:51-53 */
    for (uint32_t i = 0; i < n_ports; i++) {                          /* init.c:56-60,79-81 */
        uint32_t ip = (192u << 24) | (167u << 16) | (10u << 8) | ((i + 1) & 0xff);
        rt[ip & 0xFFFF] = (uint16_t)i;
    }
}

static inline uint32_t be16at(const uint8_t *p) { return ((uint32_t)p[0] << 8) | p[1]; }
static inline uint32_t be32at(const uint8_t *p)
{
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

uint32_t orc_get_next_hop(const uint8_t *pkt, const uint16_t *rt)
{
    if (be16at(pkt + 12) != 0x0800) return 0xFFFF;   /* ETHER_TYPE_IPv4, switch.c:117-120 */
    uint32_t dst = be32at(pkt + 14 + 16);             /* ipv4_hdr.dst_addr, switch.c:125-127 */
    return rt[dst & 0xFFFF];                          /* switch.c:133 */
}

/* ---------------------------------------------------------------------- */
/* DPDK rte_lpm (17.11, v1604): incremental DIR-24-8                       */
/* ---------------------------------------------------------------------- */

#define E_VALID 0x01000000u
#define E_GROUP 0x02000000u
#define E_DEPTH(e) ((e) >> 26)
#define E_NH(e) ((e) & 0x00FFFFFFu)
#define MK(nh, depth, grp) (((nh) & 0x00FFFFFFu) | E_VALID | ((grp) ? E_GROUP : 0u) | ((uint32_t)(depth) << 26))

typedef struct orc_lpm {
    uint32_t max_rules, number_tbl8s;
    uint32_t n_rules;
    /* rule table as a hash: key = depth<<32 | masked ip; rid = rule id
     * (order in which distinct rules were first accepted) */
    uint64_t *rkey;
    uint32_t *rnh;
    uint32_t *rid;
    uint64_t rcap;
    uint32_t *tbl24;
    uint32_t *tbl8;
    uint8_t *grp_used;
    /* rules-only mode (no DIR-24-8 image, for 1M-rule tables): tbl8 group
     * accounting by the set of /24 parents holding a depth > 24 rule, and
     * lookups by hash probes from depth 32 down */
    int rules_only;
    uint64_t *parents;
    uint64_t pcap;
    uint32_t n_groups;
} orc_lpm;

#define RK_EMPTY (~0ull)

static uint64_t rk_hash(uint64_t k)
{
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

static int64_t rk_find(const orc_lpm *l, uint64_t key, uint64_t *slot_out)
{
    uint64_t i = rk_hash(key) & (l->rcap - 1);
    while (l->rkey[i] != RK_EMPTY) {
        if (l->rkey[i] == key) {
            *slot_out = i;
            return 1;
        }
        i = (i + 1) & (l->rcap - 1);
    }
    *slot_out = i;
    return 0;
}

static void rk_erase(orc_lpm *l, uint64_t slot)
{
    /* backward-shift deletion for linear probing */
    uint64_t i = slot, j = slot;
    l->rkey[i] = RK_EMPTY;
    for (;;) {
        j = (j + 1) & (l->rcap - 1);
        if (l->rkey[j] == RK_EMPTY) return;
        uint64_t h = rk_hash(l->rkey[j]) & (l->rcap - 1);
        int move = (i <= j) ? (h <= i || h > j) : (h <= i && h > j);
        if (move) {
            l->rkey[i] = l->rkey[j];
            l->rnh[i] = l->rnh[j];
            l->rid[i] = l->rid[j];
            l->rkey[j] = RK_EMPTY;
            i = j;
        }
    }
}

void orc_lpm_free(orc_lpm *l)
{
    if (!l) return;
    free(l->rkey);
    free(l->rnh);
    free(l->rid);
    free(l->tbl24);
    free(l->tbl8);
    free(l->grp_used);
    free(l->parents);
    free(l);
}

/* flags bit 0: rules-only mode (see struct orc_lpm) */
orc_lpm *orc_lpm_create2(uint32_t max_rules, uint32_t number_tbl8s, uint32_t flags)
{
    if (max_rules == 0) return NULL;
    orc_lpm *l = (orc_lpm *)calloc(1, sizeof(*l));
    if (!l) return NULL;
    l->max_rules = max_rules;
    l->number_tbl8s = number_tbl8s;
    l->rules_only = (flags & 1u) != 0;
    l->rcap = 16;
    while (l->rcap < 2ull * max_rules + 2) l->rcap <<= 1;
    l->rkey = (uint64_t *)malloc(l->rcap * sizeof(uint64_t));
    l->rnh = (uint32_t *)malloc(l->rcap * sizeof(uint32_t));
    l->rid = (uint32_t *)malloc(l->rcap * sizeof(uint32_t));
    int ok = l->rkey && l->rnh && l->rid;
    if (l->rules_only) {
        uint64_t want = number_tbl8s < max_rules ? number_tbl8s : max_rules;
        l->pcap = 16;
        while (l->pcap < 2 * want + 2) l->pcap <<= 1;
        l->parents = (uint64_t *)malloc(l->pcap * sizeof(uint64_t));
        ok = ok && l->parents;
        if (l->parents) memset(l->parents, 0xFF, l->pcap * sizeof(uint64_t));
    } else {
        l->tbl24 = (uint32_t *)calloc((size_t)1 << 24, sizeof(uint32_t));
        l->tbl8 = (uint32_t *)calloc((size_t)(number_tbl8s ? number_tbl8s : 1) * 256, sizeof(uint32_t));
        l->grp_used = (uint8_t *)calloc(number_tbl8s ? number_tbl8s : 1, 1);
        ok = ok && l->tbl24 && l->tbl8 && l->grp_used;
    }
    if (!ok) {
        orc_lpm_free(l);
        return NULL;
    }
    memset(l->rkey, 0xFF, l->rcap * sizeof(uint64_t));
    return l;
}

orc_lpm *orc_lpm_create(uint32_t max_rules, uint32_t number_tbl8s)
{
    return orc_lpm_create2(max_rules, number_tbl8s, 0);
}

/* rules-only: does /24 parent p hold a group; insert when asked */
static int parent_has(orc_lpm *l, uint64_t p, int insert)
{
    uint64_t i = rk_hash(p) & (l->pcap - 1);
    while (l->parents[i] != RK_EMPTY) {
        if (l->parents[i] == p) return 1;
        i = (i + 1) & (l->pcap - 1);
    }
    if (insert) l->parents[i] = p;
    return 0;
}

static int32_t tbl8_alloc(orc_lpm *l)
{
    for (uint32_t g = 0; g < l->number_tbl8s; g++) {
        if (!l->grp_used[g]) {
            l->grp_used[g] = 1;
            memset(&l->tbl8[(size_t)g * 256], 0, 256 * sizeof(uint32_t));
            return (int32_t)g;
        }
    }
    return -ENOSPC;
}

static void add_depth_small(orc_lpm *l, uint32_t ipm, uint32_t depth, uint32_t nh)
{
    uint32_t start = ipm >> 8, range = 1u << (24 - depth);
    for (uint32_t i = start; i < start + range; i++) {
        uint32_t e = l->tbl24[i];
        if (!(e & E_VALID) || (!(e & E_GROUP) && E_DEPTH(e) <= depth)) {
            l->tbl24[i] = MK(nh, depth, 0);
            continue;
        }
        if (e & E_GROUP) {
            uint32_t *g = &l->tbl8[(size_t)E_NH(e) * 256];
            for (uint32_t j = 0; j < 256; j++)
                if (!(g[j] & E_VALID) || E_DEPTH(g[j]) <= depth) g[j] = MK(nh, depth, 1);
        }
    }
}

static int add_depth_big(orc_lpm *l, uint32_t ipm, uint32_t depth, uint32_t nh)
{
    uint32_t i24 = ipm >> 8, range = 1u << (32 - depth);
    uint32_t e = l->tbl24[i24];
    if (!(e & E_VALID)) {
        int32_t g = tbl8_alloc(l);
        if (g < 0) return g;
        uint32_t *t8 = &l->tbl8[(size_t)g * 256];
        for (uint32_t i = (ipm & 0xFF); i < (ipm & 0xFF) + range; i++) t8[i] = MK(nh, depth, 0);
        l->tbl24[i24] = (uint32_t)g | E_VALID | E_GROUP;
    } else if (!(e & E_GROUP)) {
        int32_t g = tbl8_alloc(l);
        if (g < 0) return g;
        uint32_t *t8 = &l->tbl8[(size_t)g * 256];
        for (uint32_t i = 0; i < 256; i++) t8[i] = MK(E_NH(e), E_DEPTH(e), 0);
        for (uint32_t i = (ipm & 0xFF); i < (ipm & 0xFF) + range; i++) t8[i] = MK(nh, depth, 0);
        l->tbl24[i24] = (uint32_t)g | E_VALID | E_GROUP;
    } else {
        uint32_t *t8 = &l->tbl8[(size_t)E_NH(e) * 256];
        for (uint32_t i = (ipm & 0xFF); i < (ipm & 0xFF) + range; i++)
            if (!(t8[i] & E_VALID) || E_DEPTH(t8[i]) <= depth) t8[i] = MK(nh, depth, 0);
    }
    return 0;
}

int orc_lpm_add(orc_lpm *l, uint32_t ip, uint32_t depth, uint32_t next_hop)
{
    if (!l || depth < 1 || depth > 32) return -EINVAL;
    uint32_t ipm = ip & (uint32_t)(0xFFFFFFFFull << (32 - depth));
    uint32_t nh = next_hop & 0x00FFFFFFu;  /* next_hop:24 bitfield */
    uint64_t key = ((uint64_t)depth << 32) | ipm, slot;
    int existed = (int)rk_find(l, key, &slot);
    if (existed) {
        l->rnh[slot] = nh;                  /* rule_add: update next hop */
    } else {
        if (l->n_rules == l->max_rules) return -ENOSPC;
        l->rkey[slot] = key;
        l->rnh[slot] = nh;
        l->rid[slot] = l->n_rules;
        l->n_rules++;
    }
    if (l->rules_only) {
        /* tbl8 accounting only: a depth > 24 rule in a /24 without a group
         * takes the next group (groups are never freed: no deletes) */
        if (depth > 24 && !parent_has(l, ipm >> 8, 0)) {
            if (l->n_groups >= l->number_tbl8s) {
                if (!existed) {
                    rk_erase(l, slot);
                    l->n_rules--;
                }
                return -ENOSPC;
            }
            parent_has(l, ipm >> 8, 1);
            l->n_groups++;
        }
        return 0;
    }
    if (depth <= 24) {
        add_depth_small(l, ipm, depth, nh);
    } else {
        int st = add_depth_big(l, ipm, depth, nh);
        if (st < 0) {
            if (!existed) {                 /* rule_delete of the new rule */
                rk_erase(l, slot);
                l->n_rules--;
            }
            return st;
        }
    }
    return 0;
}

/* Longest match by hash probes from depth 32 down: the rule id, or -1.
 * Independent of the DIR-24-8 image (works in both modes). */
int32_t orc_lpm_match_rule(const orc_lpm *l, uint32_t ip, uint32_t *next_hop)
{
    for (int d = 32; d >= 1; d--) {
        uint64_t slot;
        uint32_t ipm = ip & (uint32_t)(0xFFFFFFFFull << (32 - d));
        if (rk_find(l, ((uint64_t)d << 32) | ipm, &slot)) {
            if (next_hop) *next_hop = l->rnh[slot];
            return (int32_t)l->rid[slot];
        }
    }
    if (next_hop) *next_hop = 0;
    return -1;
}

void orc_lpm_match_rules(const orc_lpm *l, const uint32_t *ips, uint64_t n, int32_t *rule)
{
    for (uint64_t i = 0; i < n; i++) rule[i] = orc_lpm_match_rule(l, ips[i], NULL);
}

int orc_lpm_lookup(const orc_lpm *l, uint32_t ip, uint32_t *next_hop)
{
    if (l->rules_only) return orc_lpm_match_rule(l, ip, next_hop) >= 0 ? 0 : -ENOENT;
    uint32_t e = l->tbl24[ip >> 8];
    if ((e & (E_VALID | E_GROUP)) == (E_VALID | E_GROUP)) e = l->tbl8[(size_t)E_NH(e) * 256 + (ip & 0xFF)];
    *next_hop = E_NH(e);
    return (e & E_VALID) ? 0 : -ENOENT;
}

void orc_lpm_lookup_batch(const orc_lpm *l, const uint32_t *ips, uint64_t n, uint32_t *nh, uint8_t *hit)
{
    for (uint64_t i = 0; i < n; i++) {
        uint32_t v;
        int r = orc_lpm_lookup(l, ips[i], &v);
        nh[i] = v;
        hit[i] = r == 0;
    }
}

uint32_t orc_lpm_n_rules(const orc_lpm *l) { return l->n_rules; }

uint32_t orc_lpm_tbl8_used(const orc_lpm *l)
{
    if (l->rules_only) return l->n_groups;
    uint32_t u = 0;
    for (uint32_t g = 0; g < l->number_tbl8s; g++) u += l->grp_used[g];
    return u;
}

int orc_lpm_rules(const orc_lpm *l, uint32_t *ip, uint8_t *depth, uint32_t *nh, uint32_t cap)
{
    /* in rule id order */
    if (cap < l->n_rules) return -ENOSPC;
    for (uint64_t i = 0; i < l->rcap; i++) {
        if (l->rkey[i] == RK_EMPTY) continue;
        uint32_t k = l->rid[i];
        ip[k] = (uint32_t)l->rkey[i];
        depth[k] = (uint8_t)(l->rkey[i] >> 32);
        nh[k] = l->rnh[i];
    }
    return (int)l->n_rules;
}

const uint32_t *orc_lpm_tbl24(const orc_lpm *l) { return l->tbl24; }
const uint32_t *orc_lpm_tbl8(const orc_lpm *l) { return l->tbl8; }

/* lpm_setup (firewall.c:215-255): add in order, return 1 at the first error
 * (later rules are never added). stop_at_error = 0 keeps going instead.
 * Returns the index of the first failed rule or -1; *first_err = errno. */
int orc_lpm_setup(orc_lpm *l, const uint32_t *ip, const uint8_t *depth, const uint32_t *nh, uint32_t n,
                  int stop_at_error, int *first_err)
{
    int first = -1;
    if (first_err) *first_err = 0;
    for (uint32_t i = 0; i < n; i++) {
        int r = orc_lpm_add(l, ip[i], depth[i], nh[i]);
        if (r < 0) {
            if (first < 0) {
                first = (int)i;
                if (first_err) *first_err = r;
            }
            if (stop_at_error) break;
        }
    }
    return first;
}

/* Independent check: exact LPM by linear scan over a rule list. */
void orc_brute_lookup(const uint32_t *rip, const uint8_t *rdepth, const uint32_t *rnh, uint32_t nr,
                      const uint32_t *ips, uint64_t n, uint32_t *nh, uint8_t *hit)
{
    for (uint64_t i = 0; i < n; i++) {
        int best = -1;
        uint32_t v = 0;
        for (uint32_t r = 0; r < nr; r++) {
            uint32_t m = (uint32_t)(0xFFFFFFFFull << (32 - rdepth[r]));
            if ((ips[i] & m) == rip[r] && (int)rdepth[r] > best) {
                best = rdepth[r];
                v = rnh[r];
            }
        }
        nh[i] = v;
        hit[i] = best >= 0;
    }
}

/* ---------------------------------------------------------------------- */
/* firewall.c:131-213 and the per-packet contract                          */
/* ---------------------------------------------------------------------- */

typedef struct orc_fw_stats {   /* struct firewall_pkt_stats, firewall.h:56-61 */
    uint64_t pkt_drop, pkt_accept, pkt_not_ipv4, pkt_total;
} orc_fw_stats;

enum { ORC_FORWARD = 0, ORC_DROP_FW = 1, ORC_DROP_PARSE = 2, ORC_DROP_NOT_IPV4 = 3, ORC_DROP_NO_PORT = 4 };

static inline int fw_pkt_is_ipv4(const uint8_t *pkt)
{
    return ((pkt[14] >> 4) & 0xF) == 4;          /* firewall.c:148-153 */
}

/* Returns FW_FORWARD (0) / FW_DROP (1), or ORC_DROP_NOT_IPV4 where the
 * reference dereferences NULL. *hit = rte_lpm_lookup() == 0. */
int orc_fw_packet_handler(const uint8_t *pkt, const orc_lpm *lpm, orc_fw_stats *st, int *hit)
{
    uint32_t rule = 0;
    int ret;
    st->pkt_total++;                              /* firewall.c:184 */
    *hit = 0;
    if (!fw_pkt_is_ipv4(pkt)) {                   /* firewall.c:186-190 */
        st->pkt_not_ipv4++;
        return ORC_DROP_NOT_IPV4;                 /* reference: NULL deref (UB) */
    }
    ret = orc_lpm_lookup(lpm, be32at(pkt + 14 + 12), &rule);  /* src_addr, firewall.c:193-194 */
    *hit = ret == 0;
    /* firewall.c:196-210: the ret < 0 branch is overwritten by switch(rule) */
    return rule == 0 ? 0 : 1;
}

#define ORC_STAGE_PARSE 1u
#define ORC_STAGE_FW 2u
#define ORC_STAGE_LPM 4u

/* One batch through the contract; results are 8-byte records
 * {verdict, flags, port, route_nh}; fwd[] lists FORWARD indices in order;
 * rule_hits[rule id] (optional) counts FW-stage hits per matching rule.
 * pkt i at base + (offsets ? offsets[i] : i*stride). Returns fwd count. */
uint32_t orc_process(const uint8_t *base, const uint32_t *offsets, uint64_t stride, uint32_t n,
                     const uint16_t *rt, uint32_t n_ports, uint32_t stages, const orc_lpm *fw,
                     const orc_lpm *route, uint8_t *results, uint32_t *fwd, uint64_t *counters,
                     uint64_t *rule_hits)
{
    orc_fw_stats st = {0, 0, 0, 0};
    uint32_t nf = 0;
    uint64_t parse = 0, noport = 0, fwdc = 0, rhit = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint8_t *p = base + (offsets ? (uint64_t)offsets[i] : (uint64_t)i * stride);
        uint32_t verdict = ORC_FORWARD, flags = 0, port = 0, rnh = 0;
        if (stages & ORC_STAGE_PARSE) {
            port = orc_get_next_hop(p, rt);
            if (port == 0xFFFF) verdict = ORC_DROP_PARSE;           /* switch.c:406-410 */
            else if (port >= n_ports) verdict = ORC_DROP_NO_PORT;   /* switch.c:316-319 */
            if (be16at(p + 12) != 0x0800) port = 0xFFFF;
        }
        int reached = verdict == ORC_FORWARD;
        if ((stages & ORC_STAGE_FW) && reached) {
            int hit;
            uint32_t before_not = (uint32_t)st.pkt_not_ipv4;
            int a = orc_fw_packet_handler(p, fw, &st, &hit);
            if (a == ORC_DROP_NOT_IPV4) {
                verdict = ORC_DROP_NOT_IPV4;
                st.pkt_drop++;
            } else {
                verdict = a ? ORC_DROP_FW : ORC_FORWARD;
                if (a) st.pkt_drop++;
                else st.pkt_accept++;
                if (hit) {
                    flags |= 2;
                    /* per-rule hit counter: the rule rte_lpm_lookup resolved */
                    if (rule_hits) rule_hits[orc_lpm_match_rule(fw, be32at(p + 26), NULL)]++;
                }
            }
            (void)before_not;
        }
        if ((stages & ORC_STAGE_LPM) && reached) {
            uint32_t v;
            if (orc_lpm_lookup(route, be32at(p + 30), &v) == 0) {
                flags |= 1;
                rhit++;
            }
            rnh = v;
        }
        uint8_t *r = results + (size_t)i * 8;
        r[0] = (uint8_t)verdict;
        r[1] = (uint8_t)flags;
        r[2] = (uint8_t)port;
        r[3] = (uint8_t)(port >> 8);
        r[4] = (uint8_t)rnh;
        r[5] = (uint8_t)(rnh >> 8);
        r[6] = (uint8_t)(rnh >> 16);
        r[7] = (uint8_t)(rnh >> 24);
        if (verdict == ORC_DROP_PARSE) parse++;
        if (verdict == ORC_DROP_NO_PORT) noport++;
        if (verdict == ORC_FORWARD) {
            fwdc++;
            if (fwd) fwd[nf] = i;
            nf++;
        }
    }
    if (counters) {  /* cop_counters order */
        counters[0] += st.pkt_drop;
        counters[1] += st.pkt_accept;
        counters[2] += st.pkt_not_ipv4;
        counters[3] += st.pkt_total;
        counters[4] += parse;
        counters[5] += noport;
        counters[6] += fwdc;
        counters[7] += rhit;
        counters[8] += n;
    }
    return nf;
}

/* ---------------------------------------------------------------------- */
/* The CPU coprocessor loop, timed (switch.c:443-474)                      */
/* ---------------------------------------------------------------------- */

#define ORC_PKT_BURST_SZ 32             /* init.h:47 */
#define ORC_RINGSIZE 16384              /* init.h:54 */
#define ORC_MBUF_STRIDE 2176            /* MBUF_DATA_SZ = 2048 + 128 headroom, init.h:38-41 */
#define ORC_HEADROOM 128                /* RTE_PKTMBUF_HEADROOM */
#define ORC_NB_MBUF (8192 * 16)         /* init.h:44 */

typedef struct orc_mbuf {               /* the rte_mbuf fields the path reads */
    void *buf_addr;
    uint64_t buf_iova;
    uint16_t data_off;
    uint16_t refcnt;
    uint32_t pad[11];                   /* one 64-byte line per descriptor */
} orc_mbuf;

typedef struct orc_ring {               /* rte_ring SPSC (init.c:74-75) */
    volatile uint32_t prod, cons;
    uint32_t mask, cap;
    void **slot;
} orc_ring;

static unsigned ring_enq_bulk(orc_ring *r, void **o, unsigned n)
{
    uint32_t h = r->prod, t = __atomic_load_n(&r->cons, __ATOMIC_ACQUIRE);
    if (n > r->cap - (h - t)) return 0;
    for (unsigned i = 0; i < n; i++) r->slot[(h + i) & r->mask] = o[i];
    __atomic_store_n(&r->prod, h + n, __ATOMIC_RELEASE);
    return n;
}

static unsigned ring_deq_burst(orc_ring *r, void **o, unsigned n)
{
    uint32_t h = r->cons, t = __atomic_load_n(&r->prod, __ATOMIC_ACQUIRE);
    if (n > t - h) n = t - h;
    for (unsigned i = 0; i < n; i++) o[i] = r->slot[(h + i) & r->mask];
    __atomic_store_n(&r->cons, h + n, __ATOMIC_RELEASE);
    return n;
}

typedef struct {
    const uint8_t *trace;
    uint64_t n_trace;
    const orc_lpm *lpm;
    double budget_s;
    uint64_t pkts;
    double secs;
    uint64_t forwarded;
    int cpu;
} bench_arg;

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void *bench_thread(void *va)
{
    bench_arg *a = (bench_arg *)va;
    if (a->cpu >= 0) {
        cpu_set_t cs;
        CPU_ZERO(&cs);
        CPU_SET(a->cpu, &cs);
        pthread_setaffinity_np(pthread_self(), sizeof(cs), &cs);
    }
    const uint32_t nmb = ORC_NB_MBUF;
    orc_mbuf *mb = (orc_mbuf *)aligned_alloc(64, (size_t)nmb * sizeof(orc_mbuf));
    uint8_t *bufs = (uint8_t *)aligned_alloc(64, (size_t)nmb * ORC_MBUF_STRIDE);
    void **freel = (void **)malloc((size_t)nmb * sizeof(void *));
    orc_ring rx = {0, 0, ORC_RINGSIZE - 1, ORC_RINGSIZE - 1, (void **)malloc(ORC_RINGSIZE * sizeof(void *))};
    orc_ring tx = {0, 0, ORC_RINGSIZE - 1, ORC_RINGSIZE - 1, (void **)malloc(ORC_RINGSIZE * sizeof(void *))};
    if (!mb || !bufs || !freel || !rx.slot || !tx.slot) {
        a->pkts = 0;
        a->secs = 0;
        goto out;
    }
    for (uint32_t i = 0; i < nmb; i++) {
        mb[i].buf_addr = bufs + (size_t)i * ORC_MBUF_STRIDE;
        mb[i].buf_iova = 0;
        mb[i].data_off = ORC_HEADROOM;
        mb[i].refcnt = 1;
        memcpy(bufs + (size_t)i * ORC_MBUF_STRIDE + ORC_HEADROOM, a->trace + (i % a->n_trace) * 64, 64);
        freel[i] = &mb[i];
    }
    uint32_t nfree = nmb;
    orc_fw_stats st = {0, 0, 0, 0};
    double secs = 0;
    uint64_t pkts = 0, fwdn = 0;
    while (secs < a->budget_s) {
        /* producer (fast path, untimed): fill rx_q in bursts of 32 */
        void *burst[ORC_PKT_BURST_SZ];
        for (;;) {
            if (nfree < ORC_PKT_BURST_SZ) break;
            for (int k = 0; k < ORC_PKT_BURST_SZ; k++) burst[k] = freel[nfree - 1 - k];
            if (!ring_enq_bulk(&rx, burst, ORC_PKT_BURST_SZ)) break;
            nfree -= ORC_PKT_BURST_SZ;
        }
        /* coprocessor(): timed until rx_q is drained */
        double t0 = now_s();
        uint64_t done = 0;
        void *txbuf[ORC_PKT_BURST_SZ];
        unsigned txc = 0;
        for (;;) {
            void *pb[ORC_PKT_BURST_SZ];
            unsigned nd = ring_deq_burst(&rx, pb, ORC_PKT_BURST_SZ);      /* switch.c:463 */
            if (!nd) break;
            for (unsigned k = 0; k < nd; k++) {
                orc_mbuf *m = (orc_mbuf *)pb[k];
                const uint8_t *pkt = (const uint8_t *)m->buf_addr + m->data_off;  /* mtod */
                int hit;
                int act = orc_fw_packet_handler(pkt, a->lpm, &st, &hit);           /* process_packet */
                if (act == 0) {                                                   /* enqueue_nf_tx */
                    txbuf[txc++] = m;
                    if (txc == ORC_PKT_BURST_SZ) {
                        if (!ring_enq_bulk(&tx, txbuf, txc))
                            for (unsigned q = 0; q < txc; q++) freel[nfree++] = txbuf[q];
                        txc = 0;
                    }
                } else {
                    freel[nfree++] = m;                                           /* rte_pktmbuf_free */
                }
            }
            done += nd;
            if (txc) {                                                            /* flush_nf_tx_queue */
                if (!ring_enq_bulk(&tx, txbuf, txc))
                    for (unsigned q = 0; q < txc; q++) freel[nfree++] = txbuf[q];
                txc = 0;
            }
        }
        secs += now_s() - t0;
        pkts += done;
        /* fast path drains tx_q (untimed) and the mbufs go back to the pool */
        for (;;) {
            void *pb[ORC_PKT_BURST_SZ];
            unsigned nd = ring_deq_burst(&tx, pb, ORC_PKT_BURST_SZ);
            if (!nd) break;
            fwdn += nd;
            for (unsigned k = 0; k < nd; k++) freel[nfree++] = pb[k];
        }
    }
    a->pkts = pkts;
    a->secs = secs;
    a->forwarded = fwdn;
out:
    free(mb);
    free(bufs);
    free(freel);
    free(rx.slot);
    free(tx.slot);
    return NULL;
}

/* Run the coprocessor loop on nthreads threads (pinned to cpus first_cpu..
 * when first_cpu >= 0), each with its own rings and mbuf pool over the same
 * 64-byte trace and the same read-only LPM. Returns aggregate Mpkt/s. */
double orc_coprocessor_bench(const uint8_t *trace, uint64_t n_trace, const orc_lpm *lpm, double budget_s,
                             int nthreads, int first_cpu, uint64_t *pkts_out, double *secs_out)
{
    if (nthreads < 1) nthreads = 1;
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    bench_arg *ar = (bench_arg *)calloc((size_t)nthreads, sizeof(bench_arg));
    double rate = 0, maxs = 0;
    uint64_t tot = 0;
    for (int i = 0; i < nthreads; i++) {
        ar[i].trace = trace;
        ar[i].n_trace = n_trace;
        ar[i].lpm = lpm;
        ar[i].budget_s = budget_s;
        ar[i].cpu = first_cpu >= 0 ? first_cpu + i : -1;
        pthread_create(&th[i], NULL, bench_thread, &ar[i]);
    }
    for (int i = 0; i < nthreads; i++) {
        pthread_join(th[i], NULL);
        if (ar[i].secs > 0) rate += ar[i].pkts / ar[i].secs / 1e6;
        tot += ar[i].pkts;
        if (ar[i].secs > maxs) maxs = ar[i].secs;
    }
    if (pkts_out) *pkts_out = tot;
    if (secs_out) *secs_out = maxs;
    free(th);
    free(ar);
    return rate;
}
