"""Segmented forward lists (COP_CFG_SEG_LISTS) and the poll-mode kernel's
round-3 machinery: per-tile completion words, live counters beside the
running kernel, binned per-rule hits, and an idle exit racing a post.

Segment k of a batch holds the indices of its forwarded packets among
packets k*256 .. k*256+255, in arrival order, at fwd_idx[k*256 ..], and
their number at fwd_count[k]. Walking the segments in order must give
exactly the oracle's dense forward list (the order coprocessor() enqueues
to tx_q, switch.c:464-470); records must equal the oracle's bit for bit."""
import time

import numpy as np
import pytest

import copgpu as cg
import oracle as orc
from helpers import oracle_tables

pytestmark = pytest.mark.gpu

S, F, L = cg.STAGE_PARSE, cg.STAGE_FW, cg.STAGE_LPM
SEG = cg.SEG_PKTS


def nseg(n):
    return (n + SEG - 1) // SEG


def seg_to_dense(fwd, cnt, n):
    """The dense list a tx side walking the segments in order sees."""
    parts = [fwd[k * SEG:k * SEG + int(cnt[k])] for k in range(nseg(n))]
    for k, p in enumerate(parts):
        assert len(p) <= SEG and (len(p) == 0 or (p[0] >= k * SEG and p[-1] < (k + 1) * SEG)), f"segment {k}"
    return np.concatenate(parts) if parts else np.zeros(0, np.uint32)


def fw1k(seed=0x5EED1002):
    return cg.gen_rules(seed, 1000, cg.GEN_FW, 20)


def oracle_batch(pk, n, stages, fw, rt=None):
    r, f, _ = orc.process(pk, n, stages=stages, fw=fw, route=rt)
    return r, f


@pytest.mark.parametrize("sizes", [(65536,), (1, 255, 256, 257, 4099, 0, 70001), (262144,)])
def test_seg_submit_matches_oracle(gpu_ctx_factory, sizes):
    """cop_submit with several batches of ragged sizes (an empty one, sizes
    around the segment edge) and one large batch: per-segment counts and
    lists."""
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_SEG_LISTS, max_batch=262144)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    fw, _ = oracle_tables(rules)
    total = sum(sizes)
    pk = cg.gen_trace(0x5EED5E00 + len(sizes), max(total, 1), rules)
    dp = ctx.alloc(max(pk.nbytes, 64))
    dp.upload(pk)
    dr = ctx.alloc(max(total, 1) * 8)
    # segment-aligned output regions per batch
    offs, o = [], 0
    for n in sizes:
        offs.append(o)
        o += nseg(n) * SEG
    df = ctx.alloc(max(o, 4) * 4)
    dc = ctx.alloc(max(o // SEG, 1) * 4)
    dc.fill(0xFF)
    bl, lo = [], 0
    for n, fo in zip(sizes, offs):
        bl.append(cg.make_batch(dp, n, dr, pkts_offset=lo * 64, results_offset=lo * 8, fwd_idx=df.addr + fo * 4,
                                fwd_count=dc.addr + (fo // SEG) * 4))
        lo += n
    ctx.submit(bl)
    ctx.sync()
    res = dr.download(cg.RESULT_DT, max(total, 1))
    fwd = df.download(np.uint32, max(o, 4))
    cnt = dc.download(np.uint32, max(o // SEG, 1))
    lo = 0
    for n, fo in zip(sizes, offs):
        if n == 0:
            continue
        r, f = oracle_batch(pk[lo * 64:(lo + n) * 64], n, S | F, fw)
        assert np.array_equal(res[lo:lo + n].view(np.uint8), r.view(np.uint8))
        c = cnt[fo // SEG:fo // SEG + nseg(n)]
        assert np.array_equal(seg_to_dense(fwd[fo:fo + nseg(n) * SEG], c, n), f)
        lo += n
    assert ctx.counters()["rx"] == total


@pytest.mark.parametrize("n", [65533, 258, 1])
def test_seg_lists_write_exactly_n_entries(gpu_ctx_factory, n):
    """fwd_idx holds n entries, no more: the last segment's list
    chunk that would reach past entry n-1 is stored word by word. One batch
    of n (not a multiple of 4) packets with guard words right after its n
    list entries: one-shot submit, ring launch and poll-mode kernel."""
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_SEG_LISTS)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    fw, _ = oracle_tables(rules)
    pk = cg.gen_trace(0x5EED5E07, n, rules)
    _, f = oracle_batch(pk, n, S | F, fw)
    dp = ctx.alloc(pk.nbytes)
    dp.upload(pk)
    dr = ctx.alloc(n * 8)
    dc = ctx.alloc(nseg(n) * 4)
    guard = 64
    df = ctx.alloc((n + guard) * 4)
    df.fill(0xAB)
    ctx.submit([cg.make_batch(dp, n, dr, fwd_idx=df, fwd_count=dc)])
    ctx.sync()
    words = df.download(np.uint32, n + guard)
    assert np.all(words[n:] == 0xABABABAB), "list stores past entry n-1"
    assert np.array_equal(seg_to_dense(words[:n], dc.download(np.uint32, nseg(n)), n), f)
    # ring slots of n packets whose lists sit fwd_slot = n rounded up to 4
    # words apart: the words between n and fwd_slot stay untouched
    P, slot = 3, (n + 3) // 4 * 4 + 4
    pkr = np.tile(pk, P)
    dpr = ctx.alloc(pkr.nbytes)
    dpr.upload(pkr)
    drr = ctx.alloc(P * n * 8)
    dfr = ctx.alloc(P * slot * 4)
    dcr = ctx.alloc(P * nseg(n) * 4)
    ring = cg.make_ring(dpr, P, n, drr, n * 64, fwd_idx=dfr, fwd_slot=slot, fwd_count=dcr)
    for engine in ("launch", "pmd"):
        dfr.fill(0xAB)
        if engine == "launch":
            ctx.submit_ring(ring, 0, P)
            ctx.sync()
        else:
            with ctx.pmd_start(ring) as m:
                m.post(P)
                m.wait()
        w = dfr.download(np.uint32, P * slot)
        c = dcr.download(np.uint32, P * nseg(n))
        for s_ in range(P):
            assert np.all(w[s_ * slot + n:(s_ + 1) * slot] == 0xABABABAB), f"{engine}: slot {s_} past n"
            got = seg_to_dense(w[s_ * slot:s_ * slot + n], c[s_ * nseg(n):(s_ + 1) * nseg(n)], n)
            assert np.array_equal(got, f), f"{engine}: slot {s_}"


def test_seg_ring_fw_lpm(gpu_ctx_factory):
    """Ring launches (the bench's form) with the route stage: FW + LPM 100k,
    both DIR-24-8 route probes and LDS firewall intervals."""
    rules = fw1k()
    rts = cg.gen_rules(0x5EED2004, 100000, cg.GEN_ROUTES, 0)
    ctx = gpu_ctx_factory(stages=S | F | L, flags=cg.CFG_SEG_LISTS)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    ctx.set_route_lpm(cg.LpmTable(rts, 1 << 20, 1 << 16, False))
    fw, rt = oracle_tables(rules, rts)
    B, P = 65536, 6
    pk = cg.gen_trace(0x5EED5E10, B * P, rules, rts)
    dp = ctx.alloc(pk.nbytes)
    dp.upload(pk)
    dr = ctx.alloc(B * P * 8)
    df = ctx.alloc(B * P * 4)
    dc = ctx.alloc(P * nseg(B) * 4)
    ring = cg.make_ring(dp, P, B, dr, B * 64, fwd_idx=df, fwd_slot=B, fwd_count=dc)
    ctx.submit_ring(ring, 2, P)   # wraps: slots 2..5, 0, 1
    ctx.sync()
    res = dr.download(cg.RESULT_DT, B * P)
    fwd = df.download(np.uint32, B * P)
    cnt = dc.download(np.uint32, P * nseg(B))
    for s in range(P):
        r, f = oracle_batch(pk[s * B * 64:(s + 1) * B * 64], B, S | F | L, fw, rt)
        assert np.array_equal(res[s * B:(s + 1) * B].view(np.uint8), r.view(np.uint8)), f"slot {s}"
        assert np.array_equal(seg_to_dense(fwd[s * B:(s + 1) * B], cnt[s * nseg(B):(s + 1) * nseg(B)], B), f)


def test_seg_rejects_misaligned_and_demux(gpu_ctx_factory):
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_SEG_LISTS | cg.CFG_DEMUX_PORTS)
    ctx.set_fw_table(cg.LpmTable(fw1k(), 1024, 24, True))
    dp = ctx.alloc(64 * 1024)
    dr = ctx.alloc(1024 * 8)
    df = ctx.alloc(1024 * 4 * 5)
    dc = ctx.alloc(64)
    with pytest.raises(cg.CopError):
        ctx.submit([cg.make_batch(dp, 1024, dr, fwd_idx=df, fwd_count=dc)])
    ctx2 = gpu_ctx_factory(stages=S | F, flags=cg.CFG_SEG_LISTS)
    ctx2.set_fw_table(cg.LpmTable(fw1k(), 1024, 24, True))
    dp2 = ctx2.alloc(64 * 1024)
    dr2 = ctx2.alloc(1024 * 8)
    df2 = ctx2.alloc(1024 * 4 + 16)
    dc2 = ctx2.alloc(64)
    with pytest.raises(cg.CopError):
        ctx2.submit([cg.make_batch(dp2, 1024, dr2, fwd_idx=df2.addr + 4, fwd_count=dc2)])


class SegRing:
    def __init__(self, ctx, pk, B, P):
        self.B, self.P = B, P
        self.dp = ctx.alloc(B * P * 64)
        self.dp.upload(pk)
        self.dr = ctx.alloc(B * P * 8)
        self.df = ctx.alloc(B * P * 4)
        self.dc = ctx.alloc(P * nseg(B) * 4)
        self.ring = cg.make_ring(self.dp, P, B, self.dr, B * 64, fwd_idx=self.df, fwd_slot=B, fwd_count=self.dc)

    def check(self, pk, stages, fw, rt=None, slots=None):
        B = self.B
        res = self.dr.download(cg.RESULT_DT, B * self.P)
        fwd = self.df.download(np.uint32, B * self.P)
        cnt = self.dc.download(np.uint32, self.P * nseg(B))
        for s in (range(self.P) if slots is None else slots):
            r, f = oracle_batch(pk[s * B * 64:(s + 1) * B * 64], B, stages, fw, rt)
            assert np.array_equal(res[s * B:(s + 1) * B].view(np.uint8), r.view(np.uint8)), f"slot {s} records"
            assert np.array_equal(seg_to_dense(fwd[s * B:(s + 1) * B], cnt[s * nseg(B):(s + 1) * nseg(B)], B),
                                  f), f"slot {s} list"
        return res


@pytest.mark.parametrize("flags", [0, cg.PMD_DYNAMIC_TILES])
def test_pmd_seg_posts_wrap(gpu_ctx_factory, flags):
    """The bench's engine and shape: a 20-batch post (one tile per worker),
    then posts that wrap the ring; counters read beside the running kernel
    see every completed batch. In the static tile order and with dynamic
    tiles (COP_PMD_DYNAMIC_TILES: claimed from tickets, the next tile's
    loads issued early)."""
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_SEG_LISTS)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    fw, _ = oracle_tables(rules)
    B, P = 65536, 24
    pk = cg.gen_trace(0x5EED5E20, B * P, rules)
    rg = SegRing(ctx, pk, B, P)
    with ctx.pmd_start(rg.ring, flags) as m:
        m.post(20)
        m.wait()
        assert ctx.counters()["rx"] == 20 * B      # read while the kernel runs
        rg.check(pk, S | F, fw, slots=range(20))
        total = 20
        for k in (4, 1, 24, 7):
            m.post(k)
            total += k
        m.wait()
        rg.check(pk, S | F, fw)
        c = ctx.counters()
        assert c["rx"] == total * B
    assert ctx.counters()["rx"] == total * B


@pytest.mark.parametrize("flags", [0, cg.PMD_DYNAMIC_TILES])
def test_pmd_seg_prefetch_deep_posts(gpu_ctx_factory, flags):
    """Posts deeper than one tile per worker: every worker holds several
    tiles of one post (with dynamic tiles each prefetches its next tile's
    first steps while it finishes the current one); posts of the whole
    ring, then odd sizes that wrap it, with the outputs cleared in between."""
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_SEG_LISTS)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    fw, _ = oracle_tables(rules)
    B, P = 65536, 64
    pk = cg.gen_trace(0x5EED5E64, B * P, rules)
    rg = SegRing(ctx, pk, B, P)
    with ctx.pmd_start(rg.ring, flags) as m:
        assert m.info()["workers"] * 3 < P * m.info()["tiles_per_batch"]
        m.post(P)
        m.wait()
        rg.check(pk, S | F, fw)
        rg.dr.fill(0xAB)
        rg.dc.fill(0xFF)
        total = P
        for k in (33, 64, 31, 5):
            m.post(k)
            total += k
        m.wait()
        rg.check(pk, S | F, fw)
        assert ctx.counters()["rx"] == total * B


def test_pmd_live_snapshots_sum_exactly(gpu_ctx_factory):
    """print_stats' read-and-zero (switch.c:33-90) beside the running kernel:
    batches are posted continuously, snapshots (reset) and per-rule reads
    (reset) are taken between posts while batches are in flight; their sums
    plus the final read equal the posted packets and the oracle's per-rule
    hits exactly (binned per-rule counting, 100k firewall rules: several
    buckets)."""
    rules = cg.gen_rules(0x5EED1077, 100000, cg.GEN_FW, 0)
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_SEG_LISTS | cg.CFG_RULE_COUNTERS, max_batch=65536)
    tab = cg.LpmTable(rules, 100000, 1 << 16, False)
    ctx.set_fw_table(tab)
    o = orc.OracleLpm(100000, 1 << 16, rules_only=True)
    o.setup(rules["ip"], rules["depth"], rules["next_hop"], stop_at_error=False)
    B, P = 65536, 8
    pk = cg.gen_trace(0x5EED5E30, B * P, rules)
    rg = SegRing(ctx, pk, B, P)
    per_slot_hits = []
    for s in range(P):
        h = np.zeros(o.n_rules, np.uint64)
        orc.process(pk[s * B * 64:(s + 1) * B * 64], B, stages=S | F, fw=o, rule_hits=h)
        per_slot_hits.append(h)
    rx_sum, hits_sum, posted = 0, np.zeros(o.n_rules, np.uint64), 0
    with ctx.pmd_start(rg.ring) as m:
        for i in range(12):
            k = 1 + (i * 5) % 7
            m.post(k)
            posted += k
            snap, _ = ctx.snapshot(reset=True)
            rx_sum += snap["rx"]
            if i % 3 == 2:
                hits_sum += ctx.rule_counters(reset=True)
        m.wait()
        rx_sum += ctx.snapshot(reset=True)[0]["rx"]
        hits_sum += ctx.rule_counters(reset=True)
    assert rx_sum == posted * B
    want = np.zeros(o.n_rules, np.uint64)
    for b in range(posted):
        want += per_slot_hits[b % P]
    assert np.array_equal(hits_sum, want)


@pytest.mark.parametrize("flags,pflags", [(0, 0), (cg.CFG_SEG_LISTS, 0), (cg.CFG_SEG_LISTS, cg.PMD_DYNAMIC_TILES)])
def test_pmd_idle_exit_races_posts(gpu_ctx_factory, monkeypatch, flags, pflags):
    """A post racing the idle exit: with a 2 ms idle limit the
    host posts at intervals around it, so some posts land while leaders are
    leaving. Every batch must still complete with the oracle's outputs
    (dense lists: no look-back granule of a half-done batch survives the
    relaunch; segmented: no chain at all; dynamic tiles: every ticket below
    the closed gate is served, the relaunch restarts the tickets)."""
    monkeypatch.setenv("COP_PMD_IDLE_MS", "2")
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=flags)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    fw, _ = oracle_tables(rules)
    B, P = 65536, 4
    pk = cg.gen_trace(0x5EED5E40, B * P, rules)
    if flags:
        rg = SegRing(ctx, pk, B, P)
    else:
        from test_gpu_pmd import Ring, check, oracle_slots
        rg = Ring(ctx, pk, B, P)
        ro, fos = oracle_slots(pk, B, P, S | F, fw)
    m = ctx.pmd_start(rg.ring, pflags)
    posted = 0
    for i in range(40):
        time.sleep((1.0 + 0.05 * (i % 41)) * 1e-3 + (0.002 if i % 5 == 4 else 0.0))
        m.post(1 + i % P)
        posted += 1 + i % P
        if i % 8 == 7:
            m.wait()
            if flags:
                rg.check(pk, S | F, fw)
            else:
                check(*rg.read(), ro, fos, B, P)
    launches = m.info()["launches"]
    m.stop()
    assert ctx.counters()["rx"] == posted * B
    assert launches >= 2   # the idle exits did happen


def test_pmd_idle_exit_counts_every_batch_once(gpu_ctx_factory, monkeypatch):
    """a batch a racing idle exit left half done was redone whole
    by the relaunch, and its finished tiles' counter and per-rule adds were
    counted twice. The gate (cop_pmd.hip) now makes an idle exit finish every
    batch any worker started. Posts race a 2 ms idle limit; per-rule hits by
    one atomic per hit (COP_HIT_BINS=0: no count kernel, each tile adds its
    own) and the verdict counters must equal the oracle's exactly."""
    monkeypatch.setenv("COP_PMD_IDLE_MS", "2")
    monkeypatch.setenv("COP_HIT_BINS", "0")
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_SEG_LISTS | cg.CFG_RULE_COUNTERS)
    tab = cg.LpmTable(rules, 1024, 24, True)
    ctx.set_fw_table(tab)
    o = orc.OracleLpm(1024, 24, rules_only=True)
    o.setup(rules["ip"], rules["depth"], rules["next_hop"])
    B, P = 65536, 4
    pk = cg.gen_trace(0x5EED5E41, B * P, rules)
    per_slot = []
    for s_ in range(P):
        h = np.zeros(o.n_rules, np.uint64)
        orc.process(pk[s_ * B * 64:(s_ + 1) * B * 64], B, stages=S | F, fw=o, rule_hits=h)
        per_slot.append(h)
    rg = SegRing(ctx, pk, B, P)
    m = ctx.pmd_start(rg.ring)
    posted = 0
    for i in range(48):
        time.sleep((1.0 + 0.04 * (i % 51)) * 1e-3 + (0.002 if i % 6 == 5 else 0.0))
        k = 1 + i % P
        m.post(k)
        posted += k
    m.wait()
    launches = m.info()["launches"]
    m.stop()
    assert launches >= 2
    assert ctx.counters()["rx"] == posted * B
    want = np.zeros(o.n_rules, np.uint64)
    for b in range(posted):
        want += per_slot[b % P]
    assert np.array_equal(ctx.rule_counters(), want)


@pytest.mark.parametrize("fw_dir,tbl8", [(False, "plain"), (False, "packed"), (True, "plain")])
def test_pmd_seg_fw_lpm_dir_probes(gpu_ctx_factory, monkeypatch, fw_dir, tbl8):
    """The poll-mode kernel with segmented lists and DIR-24-8 stages: FW +
    LPM 100k with the route stage in HBM runs step by step, the route's
    tbl24 and tbl8 probes pipelined across steps (cop_tile.h tile_steps_v;
    DESIGN.md §15.9), with the tbl8 groups plain or as packed run blocks
    (a second dependent load); with the firewall forced to DIR-24-8 too it
    runs in tile_body. A post of every slot, then posts of 1, 5 and 12
    batches that wrap the 6-slot ring (so later tiles take the coherent
    load form)."""
    monkeypatch.setenv("COP_TBL8", tbl8)
    rules = fw1k()
    rts = cg.gen_rules(0x5EED2004, 100000, cg.GEN_ROUTES, 0)
    ctx = gpu_ctx_factory(stages=S | F | L,
                          flags=cg.CFG_SEG_LISTS | (cg.CFG_FW_FORCE_DIR24 if fw_dir else 0))
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    ctx.set_route_lpm(cg.LpmTable(rts, 1 << 20, 1 << 16, False))
    fw, rt = oracle_tables(rules, rts)
    B, P = 65536, 6
    pk = cg.gen_trace(0x5EED5E20 + fw_dir, B * P, rules, rts)
    rg = SegRing(ctx, pk, B, P)
    with ctx.pmd_start(rg.ring) as m:
        for k in (P, 1, 5, 12):
            while k:
                m.post(min(k, P))
                k -= min(k, P)
            m.wait()
            rg.check(pk, S | F | L, fw, rt)
        assert m.info()["launches"] == 1
