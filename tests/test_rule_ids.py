"""Rule ids and per-rule hit accounting on the host (no GPU).

The firewall device image is keyed by the matching rule id;
the id is the rule's position in first-acceptance order of the distinct
(prefix, depth) pairs — cop_lpm_export_rules order. These tests pin that
definition between the product builder and the oracle's incremental
rte_lpm restatement (oracle/cop_oracle.c, rule hash + rid), and check the
oracle's image-free "rules only" mode (used for 1M-rule tables) against its
DIR-24-8 mode.
"""
import numpy as np
import pytest

import copgpu as cg
import oracle as orc


def _rand_ips(seed, n, rules):
    rng = np.random.default_rng(seed)
    ips = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    # half the addresses inside a random rule prefix
    k = n // 2
    pick = rng.integers(0, len(rules), k)
    depth = rules["depth"][pick].astype(np.uint64)
    host = (np.uint64(1) << (np.uint64(32) - depth)) - np.uint64(1)
    ips[:k] = ((rules["ip"][pick].astype(np.uint64) & ~host & np.uint64(0xFFFFFFFF))
               | (ips[:k].astype(np.uint64) & host)).astype(np.uint32)
    return ips


def _with_duplicates(rules, seed):
    rng = np.random.default_rng(seed)
    dup = rules[rng.integers(0, len(rules), len(rules) // 10)].copy()
    dup["next_hop"] = rng.integers(0, 256, len(dup))
    out = np.concatenate([rules, dup])
    return out[rng.permutation(len(out))]


CASES = [
    ("fw1k", lambda: cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20), (1024, 24, True)),
    ("fw1k_dups", lambda: _with_duplicates(cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20), 7), (1024, 24, True)),
    ("tbl8_exhaust_skip", lambda: cg.gen_rules(0xABC, 3000, cg.GEN_FW, 200), (4096, 24, False)),
    ("routes20k", lambda: cg.gen_rules(0x5EED2003, 20000, cg.GEN_ROUTES, 0), (1 << 20, 1 << 16, False)),
]


@pytest.mark.parametrize("name,make,cfg", CASES, ids=[c[0] for c in CASES])
def test_rule_id_order_matches_oracle(name, make, cfg):
    rules = make()
    t = cg.LpmTable(rules, *cfg)
    o = orc.OracleLpm(cfg[0], cfg[1])
    o.setup(rules["ip"], rules["depth"], rules["next_hop"], stop_at_error=cfg[2])
    ip, d, nh = o.rules_by_id()
    pr = t.rules()
    assert len(pr) == len(ip)
    assert np.array_equal(pr["ip"], ip) and np.array_equal(pr["depth"], d) and np.array_equal(pr["next_hop"], nh)


@pytest.mark.parametrize("name,make,cfg", CASES, ids=[c[0] for c in CASES])
def test_rule_lookup_matches_oracle(name, make, cfg):
    rules = make()
    t = cg.LpmTable(rules, *cfg)
    o = orc.OracleLpm(cfg[0], cfg[1])
    o.setup(rules["ip"], rules["depth"], rules["next_hop"], stop_at_error=cfg[2])
    ips = _rand_ips(11, 50000, rules)
    ips = np.concatenate([ips, np.array([0, 1, 0xFFFFFFFF, 0x7FFFFFFF, 0x80000000], np.uint32)])
    rid = t.lookup_rules(ips)
    assert np.array_equal(rid, o.match_rules(ips))
    # the id's rule really is the DIR-24-8 image's answer (next hop, hit)
    nh, hit = o.lookup(ips)
    assert np.array_equal(hit.astype(bool), rid >= 0)
    _, _, rnh = o.rules_by_id()
    assert np.array_equal(np.where(rid >= 0, rnh[np.maximum(rid, 0)], 0), nh)


@pytest.mark.parametrize("name,make,cfg", CASES, ids=[c[0] for c in CASES])
def test_rules_only_mode_equals_image_mode(name, make, cfg):
    rules = make()
    a = orc.OracleLpm(cfg[0], cfg[1])
    b = orc.OracleLpm(cfg[0], cfg[1], rules_only=True)
    ra = a.setup(rules["ip"], rules["depth"], rules["next_hop"], stop_at_error=cfg[2])
    rb = b.setup(rules["ip"], rules["depth"], rules["next_hop"], stop_at_error=cfg[2])
    assert ra == rb
    assert a.n_rules == b.n_rules and a.tbl8_used == b.tbl8_used
    for x, y in zip(a.rules_by_id(), b.rules_by_id()):
        assert np.array_equal(x, y)
    ips = _rand_ips(5, 20000, rules)
    na, ha = a.lookup(ips)
    nb, hb = b.lookup(ips)
    assert np.array_equal(na, nb) and np.array_equal(ha, hb)


def test_oracle_rule_hits_sum_to_fw_hits():
    rules = cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)
    o = orc.OracleLpm(1024, 24)
    o.setup(rules["ip"], rules["depth"], rules["next_hop"])
    n = 20000
    pk = cg.gen_trace(0x5EED0002, n, rules)
    hits = np.zeros(o.n_rules, np.uint64)
    res, _, cnt = orc.process(pk, n, stages=cg.STAGE_PARSE | cg.STAGE_FW, fw=o, rule_hits=hits)
    fw_hit = (res["flags"] & 2) != 0
    assert int(hits.sum()) == int(fw_hit.sum()) > 0
    # per rule: the packets whose source maps to that rule id
    src = pk.reshape(n, 64)[:, 26:30].copy().view(">u4").ravel().astype(np.uint32)
    ids = o.match_rules(src[fw_hit])
    assert np.array_equal(np.bincount(ids, minlength=o.n_rules).astype(np.uint64), hits)


def test_large_rules_only_build():
    """200k FW rules: product rule ids and host lookups equal the oracle's
    rules-only restatement (the 1M config's mode, at a CPU-test size)."""
    rules = cg.gen_rules(0x5EED1005, 200000, cg.GEN_FW, 0)
    t = cg.LpmTable(rules, 200000, 1 << 20, False)
    o = orc.OracleLpm(200000, 1 << 20, rules_only=True)
    o.setup(rules["ip"], rules["depth"], rules["next_hop"], stop_at_error=False)
    assert t.report.n_distinct == o.n_rules
    assert np.array_equal(t.rules()["ip"], o.rules_by_id()[0])
    ips = _rand_ips(3, 100000, rules)
    assert np.array_equal(t.lookup_rules(ips), o.match_rules(ips))
