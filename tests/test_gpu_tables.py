"""GPU: large tables against the oracle.

Tables above 8192 intervals leave LDS for the DIR-24-8 image in HBM (the
firewall's with rule-id payload, the route stage's with next hops). Records
must stay bit-identical with thousands of tbl8 groups, a /16 holding 6000
host routes, /1 prefixes and the two ends of the address space — with the
default mode selection, with FORCE_DIR24 set explicitly, with the
tbl8 groups in their packed run-block form ($COP_TBL8=packed), and with the
route stage in its multibit-trie form (CFG_LPM_TRIE) and in its bucketed
interval form (CFG_LPM_BKT).
"""
import numpy as np
import pytest

import copgpu as cg
import oracle as orc
from helpers import assert_parity, gpu_run

pytestmark = pytest.mark.gpu

S, F, L = cg.STAGE_PARSE, cg.STAGE_FW, cg.STAGE_LPM
DIR = cg.CFG_FW_FORCE_DIR24 | cg.CFG_LPM_FORCE_DIR24
# trie: the route stage in its multibit-trie form (LDS top level + L2 nodes);
# bkt: in its bucketed interval form (index + (start, value) pairs in L2)
MODES = {"auto": (0, "plain"), "forced": (DIR, "plain"), "packed": (DIR, "packed"),
         "trie": (cg.CFG_LPM_TRIE, "plain"), "bkt": (cg.CFG_LPM_BKT, "plain"),
         # the firewall's table in the bucketed form too (COP_CFG_FW_BKT)
         "fwbkt": (cg.CFG_LPM_BKT | cg.CFG_FW_BKT, "plain")}
ROUTE_FORM = {"trie": "trie", "bkt": "bkt", "fwbkt": "bkt"}


def dense_routes():
    """A route set with one /16 holding 6000 host routes (6000 tbl8
    groups' worth of structure in one /16), full-width prefixes and the two
    ends of the address space."""
    rng = np.random.default_rng(42)
    base = cg.gen_rules(0x5EED2099, 30000, cg.GEN_ROUTES, 0)
    hosts = np.zeros(6000, dtype=cg.PREFIX_DT)
    hosts["ip"] = 0x0A140000 | rng.choice(65536, 6000, replace=False).astype(np.uint32)
    hosts["depth"] = 32
    hosts["next_hop"] = rng.integers(1, 1 << 24, 6000)
    edge = np.zeros(6, dtype=cg.PREFIX_DT)
    edge["ip"] = [0, 0x80000000, 0xFFFFFFFF, 0, 0x0A140000, 0xFFFF0000]
    edge["depth"] = [1, 1, 32, 32, 16, 16]
    edge["next_hop"] = [11, 12, 13, 14, 15, 16]
    return np.concatenate([base, hosts, edge])


@pytest.mark.parametrize("mode", list(MODES))
def test_large_fw_and_routes(gpu_ctx_factory, mode, monkeypatch):
    monkeypatch.setenv("COP_TBL8", MODES[mode][1])
    fw_rules = cg.gen_rules(0x5EED1077, 20000, cg.GEN_FW, 0)
    routes = dense_routes()
    fwt = cg.LpmTable(fw_rules, 20000, 1 << 16, False)
    rtt = cg.LpmTable(routes, 1 << 20, 1 << 16, False)
    assert len(fwt.intervals()[0]) > 8192       # leaves LDS
    ctx = gpu_ctx_factory(stages=S | F | L, flags=MODES[mode][0] | cg.CFG_RULE_COUNTERS)
    ctx.set_fw_table(fwt)
    ctx.set_route_lpm(rtt)
    assert ctx.route_form() == ROUTE_FORM.get(mode, "dir")
    ofw = orc.OracleLpm(20000, 1 << 16)
    ofw.setup(fw_rules["ip"], fw_rules["depth"], fw_rules["next_hop"], stop_at_error=False)
    ort = orc.OracleLpm(1 << 20, 1 << 16)
    ort.setup(routes["ip"], routes["depth"], routes["next_hop"], stop_at_error=False)
    n = 262144
    pk = cg.gen_trace(0x5EED0077, n, fw_rules, routes)
    # steer 1/8 of the destinations into the dense /16 and onto the edges
    pk2 = pk.reshape(n, 64)
    rng = np.random.default_rng(3)
    sel = rng.choice(n, n // 8, replace=False)
    d = (0x0A140000 | rng.integers(0, 65536, len(sel))).astype(np.uint32)
    d[:4] = [0, 0xFFFFFFFF, 0x0A140000, 0x0A14FFFF]
    pk2[sel, 30:34] = d.astype(">u4").view(np.uint8).reshape(-1, 4)
    hits = np.zeros(ofw.n_rules, np.uint64)
    ro, fo, co = orc.process(pk, n, stages=S | F | L, fw=ofw, route=ort, rule_hits=hits)
    ctx.counters(reset=True)
    rg, fg, _ = gpu_run(ctx, pk, n, batches=4)
    assert_parity(rg, fg, ro, fo)
    cgc = ctx.counters()
    for k in co:
        assert cgc[k] == co[k], (k, cgc[k], co[k])
    assert np.array_equal(ctx.rule_counters(), hits)
    # the dense /16 was actually exercised
    dense = ((ro["flags"] & 1) == 1)[sel]
    assert dense.mean() > 0.05


@pytest.mark.parametrize("mode", list(MODES))
def test_large_table_all_addresses_of_a_dense_chunk(gpu_ctx_factory, mode, monkeypatch):
    """Every address of the dense /16 (65536 lookups) against the oracle."""
    monkeypatch.setenv("COP_TBL8", MODES[mode][1])
    routes = dense_routes()
    rtt = cg.LpmTable(routes, 1 << 20, 1 << 16, False)
    ctx = gpu_ctx_factory(stages=S | L, flags=MODES[mode][0])
    ctx.set_route_lpm(rtt)
    assert ctx.route_form() == ROUTE_FORM.get(mode, "dir")
    ort = orc.OracleLpm(1 << 20, 1 << 16)
    ort.setup(routes["ip"], routes["depth"], routes["next_hop"], stop_at_error=False)
    n = 65536
    pk = cg.gen_trace(0x5EED0078, n, None, routes, opts=cg.trace_opts(pct_non_ipv4=0))
    pk2 = pk.reshape(n, 64)
    d = (0x0A140000 + np.arange(n)).astype(np.uint32)
    pk2[:, 30:34] = d.astype(">u4").view(np.uint8).reshape(-1, 4)
    ro, fo, _ = orc.process(pk, n, stages=S | L, route=ort)
    rg, fg, _ = gpu_run(ctx, pk, n)
    assert_parity(rg, fg, ro, fo)


def test_bkt_wide_bucket_on_device(gpu_ctx_factory):
    """The bucketed form's wide-bucket scan (bkt_step's ballot rounds for a
    bucket with more than 7 boundaries) run by the GPU kernels, not only by
    the host mirror: 100 host routes inside one /24 among 30k
    random routes (so the table leaves LDS for CFG_LPM_BKT); every address of
    that /24 and of its neighbours, through a one-shot launch and through the
    poll-mode kernel, against the oracle."""
    dense = np.zeros(100, dtype=cg.PREFIX_DT)
    dense["ip"] = 0x0A0B0C00 + 2 * np.arange(100, dtype=np.uint32)
    dense["depth"] = 32
    dense["next_hop"] = 100 + np.arange(100)
    routes = np.concatenate([cg.gen_rules(0x5EED2098, 30000, cg.GEN_ROUTES, 0), dense])
    rtt = cg.LpmTable(routes, 1 << 20, 1 << 16, False)
    assert len(rtt.intervals()[0]) > 8192
    ips = np.arange(0x0A0B0B00, 0x0A0B0E00, dtype=np.uint32)          # the /24 and both neighbours
    _, _, info = rtt.bkt_probe(ips, 0)
    assert info["lifted"] > 0, info                                    # the wide-bucket scan is reached
    ort = orc.OracleLpm(1 << 20, 1 << 16)
    ort.setup(routes["ip"], routes["depth"], routes["next_hop"], stop_at_error=False)
    n = 65536
    pk = cg.gen_trace(0x5EED0079, n, None, routes, opts=cg.trace_opts(pct_non_ipv4=0))
    pk2 = pk.reshape(n, 64)
    d = ips[np.arange(n) % len(ips)]
    pk2[:, 30:34] = d.astype(">u4").view(np.uint8).reshape(-1, 4)
    ro, fo, _ = orc.process(pk, n, stages=S | L, route=ort)
    assert ((ro["flags"] & 1) == 1).mean() > 0.3
    ctx = gpu_ctx_factory(stages=S | L, flags=cg.CFG_LPM_BKT | cg.CFG_SEG_LISTS)
    ctx.set_route_lpm(rtt)
    assert ctx.route_form() == "bkt"
    rg, _, _ = gpu_run(ctx, pk, n, compact=False)
    for f in ("verdict", "flags", "port", "route_nh"):
        assert np.array_equal(rg[f], ro[f]), f"one-shot {f}"
    # the poll-mode kernel (its own instantiation of the bkt lookup)
    dp = ctx.alloc(pk.nbytes)
    dp.upload(pk)
    dr = ctx.alloc(n * 8)
    dr.fill(0xEE)
    ring = cg.make_ring(dp, 1, n, dr, n * 64)
    with ctx.pmd_start(ring) as m:
        m.run(3)
    res = dr.download(cg.RESULT_DT, n)
    for f in ("verdict", "flags", "port", "route_nh"):
        assert np.array_equal(res[f], ro[f]), f"poll mode {f}"


def test_fw_bkt_poll_mode_with_rule_counters(gpu_ctx_factory):
    """The bucketed firewall (COP_CFG_FW_BKT) in the poll-mode kernel: a 20k
    rule table (out of LDS) with per-rule counters, FW + bucketed route
    stage, batches posted past the ring's slots: records, lists, counters and
    per-rule hits equal the oracle's."""
    fw_rules = cg.gen_rules(0x5EED1078, 20000, cg.GEN_FW, 0)
    routes = dense_routes()
    fwt = cg.LpmTable(fw_rules, 20000, 1 << 16, False)
    rtt = cg.LpmTable(routes, 1 << 20, 1 << 16, False)
    ctx = gpu_ctx_factory(stages=S | F | L, flags=cg.CFG_FW_BKT | cg.CFG_LPM_BKT | cg.CFG_RULE_COUNTERS)
    ctx.set_fw_table(fwt)
    ctx.set_route_lpm(rtt)
    ofw = orc.OracleLpm(20000, 1 << 16)
    ofw.setup(fw_rules["ip"], fw_rules["depth"], fw_rules["next_hop"], stop_at_error=False)
    ort = orc.OracleLpm(1 << 20, 1 << 16)
    ort.setup(routes["ip"], routes["depth"], routes["next_hop"], stop_at_error=False)
    B, P, N = 65536, 3, 7
    pk = cg.gen_trace(0x5EED0080, B * P, fw_rules, routes)
    dp = ctx.alloc(pk.nbytes)
    dp.upload(pk)
    dr = ctx.alloc(B * P * 8)
    df = ctx.alloc(B * P * 4)
    dc = ctx.alloc(P * 4 + 16)
    ring = cg.make_ring(dp, P, B, dr, B * 64, fwd_idx=df, fwd_count=dc)
    ctx.counters(reset=True)
    with ctx.pmd_start(ring) as m:
        m.run(N)
    res = dr.download(cg.RESULT_DT, B * P)
    fwd = df.download(np.uint32, B * P)
    cnt = dc.download(np.uint32, P)
    hits = np.zeros(ofw.n_rules, np.uint64)
    for s in range(P):
        h = np.zeros(ofw.n_rules, np.uint64)
        ro, fo, _ = orc.process(pk[s * B * 64:(s + 1) * B * 64], B, stages=S | F | L, fw=ofw, route=ort, rule_hits=h)
        assert_parity(res[s * B:(s + 1) * B], fwd[s * B:s * B + int(cnt[s])], ro, fo)
        hits += h * np.uint64(len(range(s, N, P)))   # slot s served batches s, s + P, ...
    assert ctx.counters()["rx"] == N * B
    assert np.array_equal(ctx.rule_counters(), hits)


@pytest.mark.parametrize("route", ["lds", "trie", "empty"])
def test_fw_bkt_beside_small_or_trie_routes(gpu_ctx_factory, route):
    """the bucketed firewall's kernel parts are built for the
    large route forms only (DIR-24-8, bucketed). A route table small enough
    for LDS (1k routes) or in the trie form (CFG_LPM_TRIE) is looked up in
    its DIR-24-8 image beside it, with the oracle's results, in one-shot
    launches and in the poll-mode kernel; with no route table at all the
    launch fails with -EINVAL and a message, not an opaque -EIO."""
    fw_rules = cg.gen_rules(0x5EED1079, 20000, cg.GEN_FW, 0)
    fwt = cg.LpmTable(fw_rules, 20000, 1 << 16, False)
    assert len(fwt.intervals()[0]) > 8192
    routes = cg.gen_rules(0x5EED2097, 1000 if route == "lds" else 30000, cg.GEN_ROUTES, 0)
    flags = cg.CFG_FW_BKT | (cg.CFG_LPM_TRIE if route == "trie" else 0)
    ctx = gpu_ctx_factory(stages=S | F | L, flags=flags)
    ctx.set_fw_table(fwt)
    n = 65536
    pk = cg.gen_trace(0x5EED0081, n, fw_rules, routes)
    if route == "empty":
        with pytest.raises(cg.CopError) as ei:
            gpu_run(ctx, pk, n)
        assert ei.value.code == -22
        return
    rtt = cg.LpmTable(routes, 1 << 20, 1 << 16, False)
    ctx.set_route_lpm(rtt)
    assert ctx.route_form() == ("trie" if route == "trie" else "lds")   # the launch maps it to DIR-24-8
    ofw = orc.OracleLpm(20000, 1 << 16)
    ofw.setup(fw_rules["ip"], fw_rules["depth"], fw_rules["next_hop"], stop_at_error=False)
    ort = orc.OracleLpm(1 << 20, 1 << 16)
    ort.setup(routes["ip"], routes["depth"], routes["next_hop"], stop_at_error=False)
    ro, fo, _ = orc.process(pk, n, stages=S | F | L, fw=ofw, route=ort)
    assert ((ro["flags"] & 1) == 1).mean() > 0.3      # the route stage hits
    rg, fg, _ = gpu_run(ctx, pk, n, batches=2)
    assert_parity(rg, fg, ro, fo)
    dp = ctx.alloc(pk.nbytes)
    dp.upload(pk)
    dr = ctx.alloc(n * 8)
    dr.fill(0xEE)
    ring = cg.make_ring(dp, 1, n, dr, n * 64)
    with ctx.pmd_start(ring) as m:
        m.run(2)
    res = dr.download(cg.RESULT_DT, n)
    assert np.array_equal(res.view(np.uint8), ro.view(np.uint8))


@pytest.mark.parametrize("layout", ["slots", "imix"])
def test_bkt_route_on_the_step_path(gpu_ctx_factory, layout):
    """The bucketed route form (CFG_LPM_BKT) on the poll-mode step path
    (segmented lists: its index and pair rounds pipelined across steps,
    bkt_pairs_issue / bkt_pairs_finish, with the wide-bucket rounds inside
    the finish): 100 host routes in one /24 among 30k random routes, a
    quarter of the destinations steered into that /24 and its neighbours;
    64-byte slots and IMIX; records, segment lists and counters against the
    oracle over posts that wrap the ring."""
    from test_gpu_seg import nseg, seg_to_dense
    fw_rules = cg.gen_rules(0x5EED1081, 1000, cg.GEN_FW, 20)
    dense = np.zeros(100, dtype=cg.PREFIX_DT)
    dense["ip"] = 0x0A0B0C00 + 2 * np.arange(100, dtype=np.uint32)
    dense["depth"] = 32
    dense["next_hop"] = 100 + np.arange(100)
    routes = np.concatenate([cg.gen_rules(0x5EED2096, 30000, cg.GEN_ROUTES, 0), dense])
    rtt = cg.LpmTable(routes, 1 << 20, 1 << 16, False)
    ctx = gpu_ctx_factory(stages=S | F | L, flags=cg.CFG_LPM_BKT | cg.CFG_SEG_LISTS)
    ctx.set_fw_table(cg.LpmTable(fw_rules, 1024, 24, True))
    ctx.set_route_lpm(rtt)
    assert ctx.route_form() == "bkt"
    ofw = orc.OracleLpm(1024, 24)
    ofw.setup(fw_rules["ip"], fw_rules["depth"], fw_rules["next_hop"])
    ort = orc.OracleLpm(1 << 20, 1 << 16)
    ort.setup(routes["ip"], routes["depth"], routes["next_hop"], stop_at_error=False)
    B, P = 65536, 3
    rng = np.random.default_rng(9)
    ips = np.arange(0x0A0B0B00, 0x0A0B0E00, dtype=np.uint32)
    if layout == "imix":
        slab, offs = cg.gen_imix(0x5EED0083, B, fw_rules, routes)
        sel = rng.choice(B, B // 4, replace=False)
        for i, d in zip(sel, ips[rng.integers(0, len(ips), len(sel))]):
            slab[offs[i] + 30:offs[i] + 34] = np.array([d], dtype=">u4").view(np.uint8)
        per = slab.nbytes + offs.nbytes
        dp = ctx.alloc(per * P)
        for s_ in range(P):
            dp.upload(slab, s_ * per)
            dp.upload(offs, s_ * per + slab.nbytes)
        ro, fo, co = orc.process(slab, B, offsets=offs, stages=S | F | L, fw=ofw, route=ort)
        kname, ros, fos = "cop_pmd<1, 4, 1, 4, false>", [ro] * P, [fo] * P
    else:
        pk = cg.gen_trace(0x5EED0083, B * P, fw_rules, routes)
        pk2 = pk.reshape(B * P, 64)
        sel = rng.choice(B * P, B * P // 4, replace=False)
        pk2[sel, 30:34] = ips[rng.integers(0, len(ips), len(sel))].astype(">u4").view(np.uint8).reshape(-1, 4)
        per = B * 64
        dp = ctx.alloc(per * P)
        dp.upload(pk)
        outs = [orc.process(pk[s_ * per:(s_ + 1) * per], B, stages=S | F | L, fw=ofw, route=ort) for s_ in range(P)]
        kname, ros, fos = "cop_pmd<1, 4, 2, 4, false>", [o[0] for o in outs], [o[1] for o in outs]
    assert ((ros[0]["flags"] & 1) == 1).mean() > 0.3
    dr = ctx.alloc(B * P * 8)
    df = ctx.alloc(B * P * 4)
    dc = ctx.alloc(P * nseg(B) * 4)
    if layout == "imix":
        ring = cg.make_ring(dp, P, B, dr, per, offsets=dp.addr + slab.nbytes, offsets_slot_words=per // 4,
                            fwd_idx=df, fwd_count=dc)
    else:
        ring = cg.make_ring(dp, P, B, dr, per, stride=64, fwd_idx=df, fwd_count=dc)
    with ctx.pmd_start(ring) as m:
        assert m.info()["kernel_name"] == kname, m.info()
        m.run(7)
    res = dr.download(cg.RESULT_DT, B * P)
    fwd = df.download(np.uint32, B * P)
    cnt = dc.download(np.uint32, P * nseg(B))
    for s_ in range(P):
        assert np.array_equal(res[s_ * B:(s_ + 1) * B].view(np.uint8), ros[s_].view(np.uint8)), f"slot {s_}"
        got = seg_to_dense(fwd[s_ * B:(s_ + 1) * B], cnt[s_ * nseg(B):(s_ + 1) * nseg(B)], B)
        assert np.array_equal(got, fos[s_]), f"slot {s_} list"
