"""The engines behind bench.py's line, at the line's own sizes (VERDICT r5,
next 1): every secondary workload is timed on the poll-mode kernel
(bench.py --engine auto at the driver's 20 steps), so each is checked here
through that kernel with bench.py's tables, seeds, batch size, context flags
and slot declaration, bit for bit against the oracle (records, segmented
forward lists, verdict counters and, for config 5, every per-rule hit
counter). Each test names the kernel instantiation it ran
(cop_pmd_info_t.kernel, as rocprofv3 names it in the bench's profiles).

Oracle functions: firewall.c:170-213 (fw_packet_handler), firewall.c:194
(rte_lpm_lookup), firewall.h:56-61 (the counters), switch.c:443-474 (the
ordered forward list)."""
import numpy as np
import pytest

import copgpu as cg
import copdist
import oracle as orc
from test_gpu_seg import nseg, seg_to_dense

pytestmark = pytest.mark.gpu

S, F, L = cg.STAGE_PARSE, cg.STAGE_FW, cg.STAGE_LPM


def bench_workload(name):
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import WORKLOADS
    return WORKLOADS[name]


def check_slot(res, fwd, cnt, s, B, ro, fo, what):
    assert np.array_equal(res[s * B:(s + 1) * B].view(np.uint8), ro.view(np.uint8)), f"{what}: slot {s} records"
    ns = nseg(B)
    got = seg_to_dense(fwd[s * B:(s + 1) * B], cnt[s * ns:(s + 1) * ns], B)
    assert np.array_equal(got, fo), f"{what}: slot {s} forward list"


def test_config5_poll_mode_ext_kernel_at_bench_size(gpu_ctx_factory):
    """BASELINE configs[4] exactly as bench.py times it: 1M firewall rules
    and 1M route prefixes (seeds 0x5EED1005 / 0x5EED2005), both DIR-24-8,
    262,144-packet batches, per-rule hit counters (CFG_RULE_COUNTERS: the
    EXT kernel cop_pmd<2, 2, 2, 4, true>), segmented lists, slots declared
    static; 12 batches through the 4-slot ring (bench.py's run_steps: posts of
    a quarter ring, so it wraps three times while batches are in flight). Every slot's
    records and lists, the verdict counters and all per-rule hit counters
    (each slot's batch counted as often as it ran) equal the oracle's."""
    W = bench_workload("fw_lpm_1m")
    B, cid = W["batch"], W["cid"]
    assert B == 262144 and W["fw"] == 1000000 and W["routes"] == 1000000 and W["rule_counters"]
    fw_rules = cg.gen_rules(0x5EED1000 + cid, W["fw"], cg.GEN_FW, 0)
    routes = cg.gen_rules(0x5EED2000 + cid, W["routes"], cg.GEN_ROUTES, 0)
    fwt = cg.LpmTable(fw_rules, W["fw"], 1 << 20, False)
    rtt = cg.LpmTable(routes, W["routes"], 1 << 20, False)
    ctx = gpu_ctx_factory(stages=W["stages"], max_batch=B, max_batches=32,
                          flags=cg.CFG_RULE_COUNTERS | cg.CFG_SEG_LISTS)
    ctx.set_fw_table(fwt)
    ctx.set_route_lpm(rtt)
    assert ctx.route_form() == "dir"
    ofw = orc.OracleLpm(1000000, 1 << 20, rules_only=True)
    ofw.setup(fw_rules["ip"], fw_rules["depth"], fw_rules["next_hop"], stop_at_error=False)
    ort = orc.OracleLpm(1000000, 1 << 20, rules_only=True)
    ort.setup(routes["ip"], routes["depth"], routes["next_hop"], stop_at_error=False)
    P = 4
    pk = cg.gen_trace(copdist.shard_seed(0x5EED0000 + cid, 0, 0), P * B, fw_rules, routes)
    dp = ctx.alloc(P * B * 64)
    dp.upload(pk)
    dr = ctx.alloc(P * B * 8)
    df = ctx.alloc(P * B * 4)
    dc = ctx.alloc(P * nseg(B) * 4 + 16)
    dr.fill(0xAB)
    ring = cg.make_ring(dp, P, B, dr, B * 64, stride=64, fwd_idx=df, fwd_count=dc)
    ctx.counters(reset=True)
    ctx.rule_counters(reset=True)
    total = 12
    with ctx.pmd_start(ring, cg.PMD_STATIC_SLOTS) as m:
        info = m.info()
        assert info["kernel_name"] == "cop_pmd<2, 2, 2, 4, true>", info
        m.run(total)          # as bench.py's run_steps: posts of a quarter ring, then the wait
        assert m.info()["completed"] == total
    runs = [len(range(s, total, P)) for s in range(P)]     # batch b ran in slot b % P
    res = dr.download(cg.RESULT_DT, P * B)
    fwd = df.download(np.uint32, P * B)
    cnt = dc.download(np.uint32, P * nseg(B))
    hits = np.zeros(ofw.n_rules, np.uint64)
    want = None
    for s in range(P):
        h = np.zeros(ofw.n_rules, np.uint64)
        ro, fo, co = orc.process(pk[s * B * 64:(s + 1) * B * 64], B, stages=W["stages"], fw=ofw, route=ort,
                                 rule_hits=h)
        check_slot(res, fwd, cnt, s, B, ro, fo, "config 5")
        hits += h * np.uint64(runs[s])
        want = {k: v * runs[s] for k, v in co.items()} if want is None else \
            {k: want[k] + co[k] * runs[s] for k in co}
        if s == 0:
            assert (ro["flags"] & 1).mean() > 0.2 and (ro["flags"] & 2).mean() > 0.2   # both tables hit
    got = ctx.counters()
    for k in want:
        assert got[k] == want[k], (k, got[k], want[k])
    assert np.array_equal(ctx.rule_counters(), hits)
    assert int(hits.sum()) > 0


def test_imix_poll_mode_at_bench_size(gpu_ctx_factory):
    """BASELINE configs[2] exactly as bench.py times it: FW 1k rules + route
    LPM 100k prefixes (seeds 0x5EED1003 / 0x5EED2003; the route table leaves
    LDS for DIR-24-8), IMIX 64/594/1518 B at 7:4:1 in a slab with u32
    offsets, 65,536-packet batches, segmented lists, slots declared static,
    the IMIX kernel cop_pmd<1, 2, 1, 4, false>; the driver's 20 steps
    through an 8-slot ring (bench.py's run_steps) wrap it twice. Every
    slot's records and lists, and the counters, equal the oracle's."""
    W = bench_workload("fw_lpm_imix")
    B, cid = W["batch"], W["cid"]
    assert B == 65536 and W["imix"] and W["routes"] == 100000
    fw_rules = cg.gen_rules(0x5EED1000 + cid, W["fw"], cg.GEN_FW, 20)
    routes = cg.gen_rules(0x5EED2000 + cid, W["routes"], cg.GEN_ROUTES, 0)
    ctx = gpu_ctx_factory(stages=W["stages"], max_batch=B, max_batches=32, flags=cg.CFG_SEG_LISTS)
    ctx.set_fw_table(cg.LpmTable(fw_rules, 1024, 24, True))
    ctx.set_route_lpm(cg.LpmTable(routes, W["routes"], 1 << 20, False))
    assert ctx.route_form() == "dir"
    slab, offs = cg.gen_imix(copdist.shard_seed(0x5EED0000 + cid, 0), B, fw_rules, routes)
    per_batch = slab.nbytes + offs.nbytes
    P = 8
    dp = ctx.alloc(P * per_batch)
    for s in range(P):
        dp.upload(slab, s * per_batch)
        dp.upload(offs, s * per_batch + slab.nbytes)
    dr = ctx.alloc(P * B * 8)
    df = ctx.alloc(P * B * 4)
    dc = ctx.alloc(P * nseg(B) * 4 + 16)
    dr.fill(0xAB)
    ring = cg.make_ring(dp, P, B, dr, per_batch, offsets=dp.addr + slab.nbytes,
                        offsets_slot_words=per_batch // 4, fwd_idx=df, fwd_count=dc)
    ctx.counters(reset=True)
    with ctx.pmd_start(ring, cg.PMD_STATIC_SLOTS) as m:
        assert m.info()["kernel_name"] == "cop_pmd<1, 2, 1, 4, false>", m.info()
        m.run(20)
    ofw = orc.OracleLpm(1024, 24)
    ofw.setup(fw_rules["ip"], fw_rules["depth"], fw_rules["next_hop"])
    ort = orc.OracleLpm(W["routes"], 1 << 20)
    ort.setup(routes["ip"], routes["depth"], routes["next_hop"], stop_at_error=False)
    ro, fo, co = orc.process(slab, B, offsets=offs, stages=W["stages"], fw=ofw, route=ort)
    assert (ro["flags"] & 1).mean() > 0.2                  # the route stage hits
    res = dr.download(cg.RESULT_DT, P * B)
    fwd = df.download(np.uint32, P * B)
    cnt = dc.download(np.uint32, P * nseg(B))
    for s in range(P):
        check_slot(res, fwd, cnt, s, B, ro, fo, "IMIX")
    got = ctx.counters()
    for k in co:
        assert got[k] == co[k] * 20, (k, got[k], co[k] * 20)
