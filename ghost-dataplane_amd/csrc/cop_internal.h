/*
 * cop_internal.h — host-side structures shared between the C setup code
 * (LPM builder, rules loader) and the HIP runtime. Not part of the ABI.
 */
#ifndef COP_INTERNAL_H
#define COP_INTERNAL_H

#include <stdint.h>
#include "cop_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Internal interval value: bits 0-23 next hop, bit 24 hit, bits 26-31 depth
 * of the matching rule (0 on a miss). Lookups only observe bits 0-24. */
#define COP_IV_HIT      0x01000000u
#define COP_IV_NHHIT    0x01FFFFFFu
#define COP_IV_DEPTH_SH 26

/* DIR-24-8 entry bits (DPDK v1604 rte_lpm_tbl_entry, little-endian). */
#define COP_DIR_VALID     0x01000000u
#define COP_DIR_EXT       0x02000000u
#define COP_DIR_VALID_EXT 0x03000000u

struct cop_lpm_table {
    /* accepted rule set (masked prefix, depth, final next hop) */
    uint32_t  n_rules;
    uint32_t *rule_ip;
    uint8_t  *rule_depth;
    uint32_t *rule_nh;
    /* flattened function over [0, 2^32): starts ascending, starts[0] = 0 */
    uint32_t  n_iv;
    uint32_t *iv_start;
    uint32_t *iv_val;      /* internal value incl. depth */
    uint32_t  tbl8_used;   /* DPDK-semantics tbl8 groups (acceptance) */
    uint32_t  n_ext;       /* /24 blocks that need a tbl8 group in our image */
    /* the same function keyed by matching rule id (index into rule_*;
     * COP_NO_RULE on a miss): the firewall's device image form */
    uint32_t  n_rv;
    uint32_t *rv_start;
    uint32_t *rv_rule;
    uint32_t  n_ext_rule;
    cop_lpm_report report;
};

#define COP_NO_RULE 0xFFFFFFFFu

/* Device image forms. NH: entry = next_hop | VALID (the route stage).
 * RULE: entry = rule_id | VALID | DROP (bit 26: the rule's next hop, i.e.
 * its firewall action, is non-zero) — the firewall stage, which needs the
 * verdict and the matching rule (per-rule hit counters), not the action. */
enum { COP_FORM_NH = 0, COP_FORM_RULE = 1 };
#define COP_RV_DROP 0x04000000u

/* Merged (start, device entry) intervals of a form; arrays are malloc-ed. */
uint32_t cop_lpm_form_intervals(const cop_lpm_table *t, int form, uint32_t **starts, uint32_t **entries);
/* /24 blocks with an interior boundary in a form's image (tbl8 groups). */
uint32_t cop_lpm_form_n_ext(const cop_lpm_table *t, int form);
/* Paint a form's DIR-24-8 image (tbl24: 1<<24, tbl8: n_ext(form) * 256). */
void cop_lpm_form_fill_dir24(const cop_lpm_table *t, int form, uint32_t *tbl24, uint32_t *tbl8);

/* Flatten (hit,nh) only: merged interval arrays for the LDS search form.
 * Returns the count; the starts and vals arrays are malloc-ed. */
uint32_t cop_lpm_merged_intervals(const cop_lpm_table *t, uint32_t **starts, uint32_t **vals);
/* Build the DIR-24-8 image into caller buffers (tbl24: 1<<24 entries,
 * tbl8: t->n_ext * 256 entries). */
void cop_lpm_fill_dir24(const cop_lpm_table *t, uint32_t *tbl24, uint32_t *tbl8);

/* Multibit-trie device form (lpm_trie.c): a 12-bit top level (LDS), then
 * popcount-compressed 6-bit nodes of COP_TRIE_NODE_WORDS u32 and a leaf
 * array (L2-resident). Level-0 entries with COP_TRIE_NODE set are nodes. */
#define COP_TRIE_L0 4096u
#define COP_TRIE_NODE 0x80000000u
#define COP_TRIE_NODE_WORDS 6u
typedef struct {
    uint32_t l0[COP_TRIE_L0];
    uint32_t n_nodes, n_leaves;
    uint32_t *nodes;    /* n_nodes * COP_TRIE_NODE_WORDS */
    uint32_t *leaves;
} cop_lpm_trie;
int cop_lpm_trie_build(const uint32_t *starts, const uint32_t *vals, uint32_t m, cop_lpm_trie *out);
void cop_lpm_trie_free(cop_lpm_trie *t);
uint32_t cop_lpm_trie_lookup(const cop_lpm_trie *t, uint32_t ip);
/* tests: the trie of a table's form; per ip the trie walk (out) and the
 * interval search (ref); node and leaf counts */
int cop_lpm_trie_probe(const cop_lpm_table *tab, int form, const uint32_t *ips, uint32_t n, uint32_t *out,
                       uint32_t *ref, uint32_t *n_nodes, uint32_t *n_leaves);

/* Bucketed interval device form (lpm_bkt.c, COP_CFG_LPM_BKT): idx = 2^ib + 1
 * first-candidate positions, pairs = (start, value) x (m + COP_BKT_PADS) */
#define COP_BKT_MIN_BITS 12u
#define COP_BKT_MAX_BITS 22u
#define COP_BKT_PADS 8u
#define COP_BKT_XBITS 1u   /* default: 2 buckets per interval */
typedef struct {
    uint32_t m, ib, lv, widest;
    uint32_t *idx;
    uint32_t *pairs;
} cop_lpm_bkt;
int cop_lpm_bkt_build(const uint32_t *starts, const uint32_t *vals, uint32_t m, uint32_t xbits, cop_lpm_bkt *out);
void cop_lpm_bkt_free(cop_lpm_bkt *t);
uint32_t cop_lpm_bkt_lookup(const cop_lpm_bkt *t, uint32_t ip, uint32_t *rounds);
/* tests: the bucketed form of a table's form; per ip its lookup (out) and
 * the binary search over all intervals (ref); info = {m, ib, lv, widest,
 * lookups that needed a wide-bucket round, the wide-bucket rounds} */
int cop_lpm_bkt_probe(const cop_lpm_table *tab, int form, uint32_t xbits, const uint32_t *ips, uint32_t n,
                      uint32_t *out, uint32_t *ref, uint32_t *info);

/* tests: the route stage's table form a launch would use (COPK_TBL_*: 1 LDS
 * intervals, 2 DIR-24-8, 3 trie, 4 bucketed) */
int cop_debug_route_form(cop_ctx *c);

/* Host paths with an explicit stage mask instead of the context's: the
 * drop-in coprocessor API (dropin.c) runs the coprocessor thread's NF chain,
 * COP_DROPIN_STAGES (process_packet, coprocessor.c:50-65). */
int cop_process_host_stages(cop_ctx *c, uint32_t stages, const void *const *pkt_data, uint32_t n,
                            cop_result *results, uint32_t *fwd_idx, uint32_t *fwd_count);
/* cop_config.max_batch of a context (0 for NULL). */
uint32_t cop_ctx_max_batch(const cop_ctx *c);
int cop_host_batch_submit_stages(cop_ctx *c, uint32_t stages, uint32_t slot, const void *const *pkt_data,
                                 uint32_t n);

/* cop_pmd_start_rings with an explicit stage mask (the drop-in's NF chain) */
typedef struct cop_pmd cop_pmd;
int cop_pmd_start_rings_stages(cop_ctx *c, const cop_batch_ring *rings, uint32_t n_rings, uint32_t flags,
                               uint32_t stages, cop_pmd **out);

/* Diagnostics ($COP_HOST_PROF=1): host ns per op of the host batch paths of
 * a context: [0] gather, [1] launch, [2] wait, [3] copy-out, [4] batches,
 * [5] packets; and of the calling thread's drop-in ring loop:
 * [0] drain, [1] batch call, [2] async wait, [3] forward/free, [4] calls,
 * [5] calls with packets, [6] packets. Return the word count. */
int cop_debug_host_prof(cop_ctx *c, uint64_t *out, uint32_t n, int reset);
int cop_debug_dropin_prof(uint64_t *out, uint32_t n, int reset);

#ifdef __cplusplus
}
#endif
#endif
