"""The bucketed interval device form of the route tables (csrc/lpm_bkt.c,
COP_CFG_LPM_BKT), looked up on the host exactly as the kernel's two rounds
and lifting do (cop_device.h bkt_issue / bkt_step): every lookup equals the
binary search over the table's flattened intervals, the form the LDS and
DIR-24-8 lookups are pinned to (rte_lpm_lookup semantics, firewall.c:194).
Addresses: random, every interval start, the address either side of it, and
the ends of the space."""
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
    (20000, cg.GEN_FW, FORM_NH),
    (1000000, cg.GEN_ROUTES, FORM_NH),    # config 5's route table
    (1000000, cg.GEN_FW, FORM_RULE),      # config 5's firewall, keyed by rule id
])
def test_bkt_equals_interval_search(n, kind, form):
    rules = cg.gen_rules(0x5EED7000 + n, n, kind, 0 if kind == cg.GEN_ROUTES else 20)
    tab = cg.LpmTable(rules, n, 1 << 20, False)
    rng = np.random.default_rng(n)
    ips = probe_ips(tab, rng, 200000)
    got, ref, info = tab.bkt_probe(ips, form)
    bad = np.nonzero(got != ref)[0]
    assert bad.size == 0, (bad[:5], ips[bad[:5]], got[bad[:5]], ref[bad[:5]])
    assert (1 << info["ib"]) >= min(info["m"], 1 << 22)
    if n == 100000 and kind == cg.GEN_ROUTES:
        # index + pairs (default: two buckets per interval) about one XCD's
        # 4 MiB L2; a random address rarely needs a wide-bucket round (two
        # pairs a round), and the widest bucket takes at most four
        assert ((1 << info["ib"]) + 1) * 4 + (info["m"] + 4) * 8 < 4 << 20, info
        rnd = ips[-200000:]
        _, _, ri = tab.bkt_probe(rnd, form)
        assert ri["lifted"] < 0.10 * len(rnd), ri
        assert ri["widest"] // 2 <= 4, ri


@pytest.mark.parametrize("xbits", [0, 1, 2, 3, 8])
def test_bkt_extra_bits(xbits):
    """Any bucket count ($COP_BKT_XBITS) gives the same lookups."""
    rules = cg.gen_rules(0x5EED7100, 50000, cg.GEN_ROUTES, 0)
    tab = cg.LpmTable(rules, 50000, 1 << 20, False)
    ips = probe_ips(tab, np.random.default_rng(xbits), 50000)
    got, ref, info = tab.bkt_probe(ips, FORM_NH, xbits)
    assert np.array_equal(got, ref), info
    assert 12 <= info["ib"] <= 22


def test_bkt_edge_tables():
    """Empty table, one default route, a /32 at each end of the space,
    nested prefixes down to /32 inside one /24 (a bucket with many
    intervals: the lifting path), and a table whose intervals all start in
    one bucket."""
    def table(rows):   # (ip, depth, next_hop)
        out = np.zeros(len(rows), dtype=cg.PREFIX_DT)
        for i, (ip, d, nh) in enumerate(rows):
            out[i]["ip"], out[i]["depth"], out[i]["next_hop"] = ip, d, nh
        return out

    dense = [(0x0A0B0C00 + 2 * i, 32, 100 + i) for i in range(100)]
    cases = [
        table([]),
        table([(0, 0, 7)]),
        table([(0, 32, 1), (0xFFFFFFFF, 32, 2), (0x80000000, 1, 3)]),
        table([(0x0A000000, 8, 1), (0x0A010100, 24, 2), (0x0A010180, 25, 3), (0x0A0101C0, 30, 4),
               (0x0A0101C1, 32, 5), (0x0A0101C3, 32, 6)]),
        table(dense + [(0xFFFFFF00, 24, 9), (0xFFFFFFFE, 32, 8)]),
    ]
    for rules in cases:
        tab = cg.LpmTable(rules, 256, 256, False)
        ips = probe_ips(tab, np.random.default_rng(1), 20000)
        for form in (FORM_NH, FORM_RULE):
            got, ref, info = tab.bkt_probe(ips, form)
            assert np.array_equal(got, ref), (rules, info)
    # the dense /24 needs lifting inside one bucket
    tab = cg.LpmTable(table(dense), 256, 256, False)
    ips = np.arange(0x0A0B0C00, 0x0A0B0D00, dtype=np.uint32)
    got, ref, info = tab.bkt_probe(ips, FORM_NH)
    assert np.array_equal(got, ref)
    assert info["lifted"] > 0 and info["rounds"] >= 20 * info["lifted"] // 32, info
