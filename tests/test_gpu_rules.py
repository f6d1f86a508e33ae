"""GPU: per-rule firewall hit counters and the config-5 scale (BASELINE
configs[4]: 1M ACL rules + 1M LPM prefixes, 256k batches).

Per packet the pipeline must still be bit-exact (verdict, flags, port,
route next hop, forward list); the per-rule u64 counters must equal the
oracle's per-rule hit counts exactly, whether they are binned (each tile
sorts its hits' rule ids by bucket, cop_hit_count adds them up; the
default) or added by one atomic per hit ($COP_HIT_BINS=0). At 1M rules the oracle runs in its
rules-only mode (hash probes, no DIR-24-8 image; tests/test_rule_ids.py
checks that mode against the image mode).
"""
import numpy as np
import pytest

import copgpu as cg
import oracle as orc
from helpers import assert_parity, gpu_run

pytestmark = pytest.mark.gpu

S, F, L = cg.STAGE_PARSE, cg.STAGE_FW, cg.STAGE_LPM


def fw1k():
    return cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)


@pytest.mark.parametrize("bins", ["1", "0"], ids=["bins", "atomics"])
@pytest.mark.parametrize("flags", [0, cg.CFG_FW_FORCE_DIR24], ids=["ivt", "dir24"])
def test_rule_counters_fw1k(gpu_ctx_factory, flags, bins, monkeypatch):
    monkeypatch.setenv("COP_HIT_BINS", bins)
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=flags | cg.CFG_RULE_COUNTERS)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    o = orc.OracleLpm(1024, 24)
    o.setup(rules["ip"], rules["depth"], rules["next_hop"])
    n = 100000
    pk = cg.gen_trace(0x5EED0002, n, rules)
    hits = np.zeros(o.n_rules, np.uint64)
    ro, fo, _ = orc.process(pk, n, stages=S | F, fw=o, rule_hits=hits)
    rg, fg, _ = gpu_run(ctx, pk, n, batches=3)
    assert_parity(rg, fg, ro, fo)
    got = ctx.rule_counters()
    assert len(got) == o.n_rules
    assert np.array_equal(got, hits), np.nonzero(got != hits)[0][:10]
    assert hits.sum() > 0


def test_rule_counters_hot_rule_and_many_buckets(gpu_ctx_factory):
    """Skewed hits (70 % of the sources inside one rule's prefix) over a
    100k-rule table (7 buckets of 16384 rule ids), ragged batches: binned
    counts equal the oracle's."""
    rules = cg.gen_rules(0x5EED1044, 100000, cg.GEN_FW, 0)
    t = cg.LpmTable(rules, 100000, 1 << 16, False)
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_RULE_COUNTERS)
    ctx.set_fw_table(t)
    o = orc.OracleLpm(100000, 1 << 16, rules_only=True)
    o.setup(rules["ip"], rules["depth"], rules["next_hop"], stop_at_error=False)
    n = 3 * 65536 + 4099
    pk = cg.gen_trace(0x5EED0044, n, rules)
    hot = rules[rules["depth"] == 24][0]
    rng = np.random.default_rng(5)
    sel = rng.random(n) < 0.7
    src = (int(hot["ip"]) & 0xFFFFFF00) | rng.integers(0, 256, int(sel.sum()))
    pk.reshape(n, 64)[sel, 26:30] = src.astype(">u4").view(np.uint8).reshape(-1, 4)
    hits = np.zeros(o.n_rules, np.uint64)
    ro, fo, _ = orc.process(pk, n, stages=S | F, fw=o, rule_hits=hits)
    rg, fg, _ = gpu_run(ctx, pk, n, batches=4)
    assert_parity(rg, fg, ro, fo)
    got = ctx.rule_counters()
    assert np.array_equal(got, hits), np.nonzero(got != hits)[0][:10]
    assert hits.max() > n // 2   # the hot rule
    assert np.count_nonzero(hits) > 1000


def test_rule_counters_accumulate_and_reset(gpu_ctx_factory):
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_RULE_COUNTERS)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    o = orc.OracleLpm(1024, 24)
    o.setup(rules["ip"], rules["depth"], rules["next_hop"])
    n = 65536
    pk = cg.gen_trace(0x5EED0007, n, rules)
    hits = np.zeros(o.n_rules, np.uint64)
    orc.process(pk, n, stages=S | F, fw=o, rule_hits=hits)
    for _ in range(3):
        gpu_run(ctx, pk, n)
    assert np.array_equal(ctx.rule_counters(reset=True), 3 * hits)
    assert not ctx.rule_counters().any()
    # a new table zeroes the counters and resizes them
    t500 = cg.LpmTable(rules[:500], 1024, 24, True)
    ctx.set_fw_table(t500)
    got = ctx.rule_counters()
    assert len(got) == t500.report.n_distinct and not got.any()


def test_rule_counters_off_by_default(gpu_ctx_factory):
    ctx = gpu_ctx_factory(stages=S | F)
    ctx.set_fw_table(cg.LpmTable(fw1k(), 1024, 24, True))
    with pytest.raises(cg.CopError):
        ctx.rule_counters()


C5_FORMS = {"dir": 0, "trie": cg.CFG_LPM_TRIE, "bkt": cg.CFG_LPM_BKT,
            # the 1M-rule firewall in the bucketed form too (COP_CFG_FW_BKT),
            # beside a bucketed or a DIR-24-8 route table
            "fwbkt": cg.CFG_FW_BKT | cg.CFG_LPM_BKT, "fwbkt_rtdir": cg.CFG_FW_BKT}


@pytest.mark.parametrize("form", list(C5_FORMS))
def test_config5_scale_1m_rules_1m_prefixes(gpu_ctx_factory, form):
    """BASELINE configs[4] tables at full size, one 256k batch, full parity;
    the 1M-prefix route table as DIR-24-8, the multibit trie or the bucketed
    intervals, and the 1M-rule firewall as DIR-24-8 or bucketed intervals
    keyed by rule id (rule ids, verdicts and per-rule counters identical)."""
    cid = 5
    fw_rules = cg.gen_rules(0x5EED1000 + cid, 1000000, cg.GEN_FW, 0)
    routes = cg.gen_rules(0x5EED2000 + cid, 1000000, cg.GEN_ROUTES, 0)
    fwt = cg.LpmTable(fw_rules, 1000000, 1 << 20, False)
    rtt = cg.LpmTable(routes, 1000000, 1 << 20, False)
    ctx = gpu_ctx_factory(stages=S | F | L, max_batch=262144,
                          flags=cg.CFG_RULE_COUNTERS | C5_FORMS[form])
    ctx.set_fw_table(fwt)
    ctx.set_route_lpm(rtt)
    ofw = orc.OracleLpm(1000000, 1 << 20, rules_only=True)
    ofw.setup(fw_rules["ip"], fw_rules["depth"], fw_rules["next_hop"], stop_at_error=False)
    ort = orc.OracleLpm(1000000, 1 << 20, rules_only=True)
    ort.setup(routes["ip"], routes["depth"], routes["next_hop"], stop_at_error=False)
    assert ofw.n_rules == fwt.report.n_distinct and ort.n_rules == rtt.report.n_distinct
    n = 262144
    pk = cg.gen_trace(0x5EED0000 + cid, n, fw_rules, routes)
    hits = np.zeros(ofw.n_rules, np.uint64)
    ro, fo, co = orc.process(pk, n, stages=S | F | L, fw=ofw, route=ort, rule_hits=hits)
    ctx.counters(reset=True)
    rg, fg, _ = gpu_run(ctx, pk, n)
    assert_parity(rg, fg, ro, fo)
    cgc = ctx.counters()
    for k in co:
        assert cgc[k] == co[k], (k, cgc[k], co[k])
    assert np.array_equal(ctx.rule_counters(), hits)
    assert (ro["flags"] & 1).mean() > 0.2 and (ro["flags"] & 2).mean() > 0.2   # both tables hit


def test_rccl_single_rank_reduce(gpu_ctx_factory):
    """The RCCL reduction path with one rank: the all-reduce result equals the
    local counters; reset zeroes them. (Multi-rank runs need one GPU per
    rank: bench.py --workload fw_lpm_1m on the 8-GPU node.)"""
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_RULE_COUNTERS)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    n = 65536
    pk = cg.gen_trace(0x5EED0009, n, rules)
    ctx.counters(reset=True)
    gpu_run(ctx, pk, n)
    local = ctx.counters()
    local_hits = ctx.rule_counters()
    ctx.coll_init(cg.coll_unique_id(), 0, 1)
    tot, hits = ctx.coll_reduce_counters(reset=True)
    assert tot == local
    assert np.array_equal(hits, local_hits)
    assert ctx.counters()["rx"] == 0 and not ctx.rule_counters().any()
