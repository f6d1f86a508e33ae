"""Host-side LPM builder (product setup path, cop_lpm_build) against the
oracle's incremental restatement of DPDK rte_lpm and the brute-force LPM:
acceptance (rte_lpm_add return codes), the accepted rule set, and the
lookup function of both device images (interval form and the
DIR-24-8 image)."""
import numpy as np
import pytest

import copgpu as cg
import oracle as orc


def lookup_intervals(t: cg.LpmTable, ips):
    s, v = t.intervals()
    k = np.searchsorted(s, ips, side="right") - 1
    return v[k] & 0xFFFFFF, (v[k] >> 24) & 1


def lookup_dir24(t: cg.LpmTable, ips):
    t24, t8 = t.dir24()
    e = t24[ips >> 8]
    ext = (e & 0x03000000) == 0x03000000
    e = e.copy()
    e[ext] = t8[((e[ext] & 0xFFFFFF).astype(np.int64) << 8) | (ips[ext] & 0xFF)]
    return e & 0xFFFFFF, (e >> 24) & 1


def probes_for(rules, rng, n=30000):
    ip = rules["ip"].astype(np.uint32)
    d = rules["depth"].astype(np.int64)
    m = np.array([(0xFFFFFFFF << (32 - int(x))) & 0xFFFFFFFF if 1 <= x <= 32 else 0 for x in d], dtype=np.uint32)
    lo = ip & m
    hi = lo | ~m
    base = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    return np.concatenate([base, lo, hi, lo - 1, hi + 1, np.array([0, 0xFFFFFFFF], np.uint32)]).astype(np.uint32)


def compare(rules, max_rules, ntbl8, stop, rng):
    t = cg.LpmTable(rules, max_rules, ntbl8, stop)
    o = orc.OracleLpm(max_rules, ntbl8)
    first, err = o.setup(rules["ip"], rules["depth"], rules["next_hop"], stop_at_error=stop)
    rep = t.report
    if first < 0:
        assert rep.n_failed == 0
    else:
        assert rep.first_error_idx == first and rep.first_error == err
    assert rep.n_distinct == o.n_rules
    assert rep.tbl8_used == o.tbl8_used
    rip, rd, rnh = o.rules()
    pr = t.rules()
    order = np.lexsort((pr["depth"], pr["ip"]))
    assert np.array_equal(pr["ip"][order], rip)
    assert np.array_equal(pr["depth"][order], rd)
    assert np.array_equal(pr["next_hop"][order], rnh)
    ips = probes_for(rules, rng)
    onh, ohit = o.lookup(ips)
    for fn in (lookup_intervals, lookup_dir24):
        nh, hit = fn(t, ips)
        assert np.array_equal(nh, onh), fn.__name__
        assert np.array_equal(hit, ohit), fn.__name__
    return t


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_fw_1k_rules(seed):
    rules = cg.gen_rules(seed, 1000, cg.GEN_FW, 20)
    compare(rules, 1024, 24, True, np.random.default_rng(seed))


def test_routes_100k():
    rules = cg.gen_rules(0x5EED2003, 100000, cg.GEN_ROUTES, 0)
    compare(rules, 1 << 20, 1 << 16, False, np.random.default_rng(5))


def test_capacity_errors_stop_and_skip():
    rng = np.random.default_rng(7)
    rules = cg.gen_rules(99, 3000, cg.GEN_FW, 60)      # > 1024 rules, > 24 tbl8 parents
    t = compare(rules, 1024, 24, True, rng)
    assert t.report.n_failed == 1 and t.report.n_skipped > 0
    t = compare(rules, 1024, 24, False, rng)
    assert t.report.n_failed > 1 and t.report.n_skipped == 0


def test_edge_prefixes():
    rng = np.random.default_rng(3)
    rules = cg.prefixes(
        [0, 0x80000000, 0xFFFFFFFF, 0xFFFFFF00, 0x0A000001, 0x0A000001, 0x0A000000, 0x0A0000FF, 1, 5, 7],
        [1, 1, 32, 24, 32, 32, 31, 25, 0, 33, 255],
        [1, 2, 3, 4, 5, 6, 0, 0x1234567, 9, 9, 9])
    t = compare(rules, 1024, 24, False, rng)
    assert t.report.n_failed == 3            # depths 0, 33, 255 -> -EINVAL
    assert t.report.n_updated == 1           # 10.0.0.1/32 twice: last write wins
    nh, hit = lookup_intervals(t, np.array([0x0A000001, 0xFFFFFFFF, 0x7FFFFFFF, 0x0A0000FF], np.uint32))
    assert list(nh) == [6, 3, 1, 0x234567] and list(hit) == [1, 1, 1, 1]


def test_empty_table_all_miss():
    t = cg.LpmTable(np.zeros(0, dtype=cg.PREFIX_DT), 1024, 24)
    nh, hit = lookup_dir24(t, np.array([0, 12345, 0xFFFFFFFF], np.uint32))
    assert not nh.any() and not hit.any()
    s, v = t.intervals()
    assert list(s) == [0] and list(v) == [0]
