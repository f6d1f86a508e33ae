"""The multibit-trie device form of the LPM tables (csrc/lpm_trie.c), walked
on the host: every lookup equals the binary search over the table's
flattened intervals, the form the LDS and DIR-24-8 lookups are pinned to
(rte_lpm_lookup semantics, firewall.c:194). Addresses: random, every
interval start and the address before it, and the ends of the space."""
import numpy as np
import pytest

import copgpu as cg

FORM_NH, FORM_RULE = 0, 1


def probe_ips(tab, rng, n_random):
    s, _ = tab.intervals()
    edges = np.concatenate([s, s - 1, s + 1, [0, 1, 0xFFFFFFFE, 0xFFFFFFFF]]).astype(np.uint32)
    return np.concatenate([edges, rng.integers(0, 1 << 32, n_random, dtype=np.uint64).astype(np.uint32)])


@pytest.mark.parametrize("n,kind,form", [
    (100000, cg.GEN_ROUTES, FORM_NH),     # the FW + LPM route table (BASELINE configs[2], [3])
    (1000, cg.GEN_FW, FORM_RULE),         # fw1k keyed by rule id
    (20000, cg.GEN_FW, FORM_NH),
    (1000000, cg.GEN_ROUTES, FORM_NH),    # config 5's route table
    (1000000, cg.GEN_FW, FORM_RULE),      # config 5's firewall, keyed by rule id
])
def test_trie_equals_interval_search(n, kind, form):
    rules = cg.gen_rules(0x5EED7000 + n, n, kind, 0 if kind == cg.GEN_ROUTES else 20)
    tab = cg.LpmTable(rules, n, 1 << 20, False)
    rng = np.random.default_rng(n)
    ips = probe_ips(tab, rng, 200000)
    got, ref, nodes, leaves = tab.trie_probe(ips, form)
    bad = np.nonzero(got != ref)[0]
    assert bad.size == 0, (bad[:5], ips[bad[:5]], got[bad[:5]], ref[bad[:5]])
    if n == 100000:
        # small enough to stay in one XCD's 4 MiB L2 (24-byte nodes, 4-byte leaves)
        assert nodes * 24 + leaves * 4 < 4 << 20, (nodes, leaves)


def test_trie_edge_tables():
    """Empty table, one default route, a /32 at each end of the space, and
    nested prefixes down to /32 inside one /24 (the deepest node level)."""
    def table(rows):   # (ip, depth, next_hop)
        out = np.zeros(len(rows), dtype=cg.PREFIX_DT)
        for i, (ip, d, nh) in enumerate(rows):
            out[i]["ip"], out[i]["depth"], out[i]["next_hop"] = ip, d, nh
        return out

    cases = [
        table([]),
        table([(0, 0, 7)]),
        table([(0, 32, 1), (0xFFFFFFFF, 32, 2), (0x80000000, 1, 3)]),
        table([(0x0A000000, 8, 1), (0x0A010100, 24, 2), (0x0A010180, 25, 3), (0x0A0101C0, 30, 4),
               (0x0A0101C1, 32, 5), (0x0A0101C3, 32, 6)]),
    ]
    for rules in cases:
        tab = cg.LpmTable(rules, 64, 64, False)
        ips = probe_ips(tab, np.random.default_rng(1), 20000)
        for form in (FORM_NH, FORM_RULE):
            got, ref, _, _ = tab.trie_probe(ips, form)
            assert np.array_equal(got, ref), rules
