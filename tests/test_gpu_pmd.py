"""The poll-mode (persistent) kernel, cop_pmd_* (csrc/cop_pmd.hip): one
long-lived launch serving a batch ring, batches posted through a host
doorbell. Every record, forward list and count must equal the oracle's, as
for the one-shot launches (test_gpu_ring.py), across: posts of one batch
and of many, ring wrap-around with slot reuse, every packet layout
(coalesced 64 B slots, mbuf stride with headroom, 16-byte header records,
IMIX), the DIR-24-8 stages, per-rule counters, demux and port statistics,
an idle exit followed by a relaunch, and stop/restart on one context."""
import time

import numpy as np
import pytest

import copgpu as cg
import oracle as orc
from helpers import oracle_tables

pytestmark = pytest.mark.gpu

S, F, L = cg.STAGE_PARSE, cg.STAGE_FW, cg.STAGE_LPM


def fw1k(seed=0x5EED1002):
    return cg.gen_rules(seed, 1000, cg.GEN_FW, 20)


def routes(n=100000, seed=0x5EED2004):
    return cg.gen_rules(seed, n, cg.GEN_ROUTES, 0)


class Ring:
    """P slots of B packets in HBM (64 B slots unless stride/data_off say
    otherwise), with records, forward lists (x lists) and counts."""

    def __init__(self, ctx, pk, B, P, stride=64, data_off=0, lists=1):
        self.B, self.P, self.lists = B, P, lists
        self.slot_bytes = ((B * stride + data_off + 4095) // 4096) * 4096
        self.dp = ctx.alloc(self.slot_bytes * P)
        for s in range(P):
            if stride == 64 and data_off == 0:
                self.dp.upload(pk[s * B * 64:(s + 1) * B * 64], s * self.slot_bytes)
            else:
                buf = np.zeros(self.slot_bytes, np.uint8)
                v = buf[data_off:data_off + B * stride].reshape(B, stride)
                v[:, :min(64, stride)] = pk[s * B * 64:(s + 1) * B * 64].reshape(B, 64)[:, :min(64, stride)]
                self.dp.upload(buf, s * self.slot_bytes)
        self.dr = ctx.alloc(B * P * 8)
        self.df = ctx.alloc(B * P * 4 * lists)
        self.dc = ctx.alloc(P * 4 * lists)
        self.dr.fill(0xAB)
        self.dc.fill(0xFF)
        self.ring = cg.make_ring(self.dp, P, B, self.dr, self.slot_bytes, stride=stride, data_off=data_off,
                                 fwd_idx=self.df, fwd_slot=B * lists, fwd_count=self.dc)

    def read(self):
        return (self.dr.download(cg.RESULT_DT, self.B * self.P), self.df.download(np.uint32, self.B * self.P * self.lists),
                self.dc.download(np.uint32, self.P * self.lists))


def oracle_slots(pk, B, P, stages, fw, rt=None):
    recs, fos = [], []
    for s in range(P):
        r, f, _ = orc.process(pk[s * B * 64:(s + 1) * B * 64], B, stages=stages, fw=fw, route=rt)
        recs.append(r)
        fos.append(f)
    return np.concatenate(recs), fos


def check(res, fwd, cnt, ro, fos, B, P):
    for s in range(P):
        assert np.array_equal(res[s * B:(s + 1) * B].view(np.uint8), ro[s * B:(s + 1) * B].view(np.uint8)), \
            f"slot {s} records"
        c = int(cnt[s])
        assert c == len(fos[s]), f"slot {s} count"
        assert np.array_equal(fwd[s * B:s * B + c], fos[s]), f"slot {s} forward list"


def test_pmd_fw1k_posts_and_wraparound(gpu_ctx_factory):
    """The bench's shape (64k-packet slots): one post of every slot, then
    posts of 1, 7 and 24 that wrap the ring and reuse slots (each slot's
    outputs are rewritten identically); counters sum every posted batch."""
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    B, P = 65536, 24
    pk = cg.gen_trace(0x5EED0B00, B * P, rules)
    fw, _ = oracle_tables(rules)
    ro, fos = oracle_slots(pk, B, P, S | F, fw)
    rg = Ring(ctx, pk, B, P)
    with ctx.pmd_start(rg.ring) as m:
        info = m.info()
        assert info["tiles_per_batch"] * info["packets_per_tile"] >= B and info["workers"] >= 256
        assert info["state"] == 0 and info["launches"] == 1
        m.post(P)
        m.wait()
        check(*rg.read(), ro, fos, B, P)
        rg.dr.fill(0xAB)
        rg.dc.fill(0xFF)
        total = P
        for k in (1, 7, 24, 24, 3):
            m.post(k)
            total += k
        m.wait()
        assert m.posted == total
        check(*rg.read(), ro, fos, B, P)
    c = ctx.counters()
    assert c["rx"] == total * B
    assert c["forward"] == sum(len(fos[b % P]) for b in range(total))   # batch b ran in slot b % P


def test_pmd_one_batch_at_a_time(gpu_ctx_factory):
    """Post, wait, post, wait: the doorbell path with nothing queued (the
    workers idle between posts, the relay wakes them)."""
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    B, P = 65536, 5
    pk = cg.gen_trace(0x5EED0B10, B * P, rules)
    fw, _ = oracle_tables(rules)
    ro, fos = oracle_slots(pk, B, P, S | F, fw)
    rg = Ring(ctx, pk, B, P)
    m = ctx.pmd_start(rg.ring)
    for i in range(40):
        m.post(1)
        m.wait(i + 1)
        if i == P - 1:
            check(*rg.read(), ro, fos, B, P)
    m.stop()
    check(*rg.read(), ro, fos, B, P)
    assert ctx.counters()["rx"] == 40 * B


@pytest.mark.parametrize("layout", ["mbuf", "hdr16", "small"])
def test_pmd_layouts(gpu_ctx_factory, layout):
    """Packets at mbuf stride (2176 B, 128 B headroom), as 16-byte header
    records, and small batches (a few tiles of 256 or 1024 packets)."""
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    B, P = (30000 + 5, 4) if layout != "small" else (5000 + 3, 9)
    pk = cg.gen_trace(0x5EED0B20, B * P, rules)
    fw, _ = oracle_tables(rules)
    ro, fos = oracle_slots(pk, B, P, S | F, fw)
    if layout == "hdr16":
        rec = np.zeros((B * P, 16), np.uint8)
        fr = pk.reshape(B * P, 64)
        rec[:, 0:4] = fr[:, 12:16]
        rec[:, 4:16] = fr[:, 24:36]
        hp = np.zeros(B * P * 64, np.uint8)
        hp.reshape(B * P, 64)[:, :16] = rec
        rg = Ring(ctx, hp, B, P, stride=16)
    elif layout == "mbuf":
        rg = Ring(ctx, pk, B, P, stride=2176, data_off=128)
    else:
        rg = Ring(ctx, pk, B, P)
    with ctx.pmd_start(rg.ring) as m:
        m.post(P)
        m.post(P)
        m.wait()
    check(*rg.read(), ro, fos, B, P)


@pytest.mark.parametrize("form", ["dir", "trie", "bkt"])
def test_pmd_imix(gpu_ctx_factory, form):
    """IMIX slab + u32 offsets per slot; the 20k-route table (beyond LDS) as
    DIR-24-8 or in the multibit-trie form."""
    rules = fw1k()
    rts = routes(20000)
    ctx = gpu_ctx_factory(stages=S | F | L, flags={"dir": 0, "trie": cg.CFG_LPM_TRIE, "bkt": cg.CFG_LPM_BKT}[form])
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    ctx.set_route_lpm(cg.LpmTable(rts, 1 << 20, 1 << 16, False))
    B, P = 20000, 3
    slab, offs = cg.gen_imix(0x5EED0B30, B, rules, rts)
    per = ((slab.nbytes + offs.nbytes + 4095) // 4096) * 4096
    dp = ctx.alloc(per * P)
    for s in range(P):
        dp.upload(slab, s * per)
        dp.upload(offs, s * per + slab.nbytes)
    dr = ctx.alloc(B * P * 8)
    df = ctx.alloc(B * P * 4)
    dc = ctx.alloc(P * 4)
    ring = cg.make_ring(dp, P, B, dr, per, offsets=dp.addr + slab.nbytes, offsets_slot_words=per // 4,
                        fwd_idx=df, fwd_slot=B, fwd_count=dc)
    with ctx.pmd_start(ring) as m:
        m.post(P)
        m.wait()
    fw, rt = oracle_tables(rules, rts)
    r1, f1, _ = orc.process(slab, B, offsets=offs, stages=S | F | L, fw=fw, route=rt)
    res = dr.download(cg.RESULT_DT, B * P)
    fwd = df.download(np.uint32, B * P)
    cnt = dc.download(np.uint32, P)
    for s in range(P):
        assert np.array_equal(res[s * B:(s + 1) * B].view(np.uint8), r1.view(np.uint8))
        assert int(cnt[s]) == len(f1) and np.array_equal(fwd[s * B:s * B + len(f1)], f1)


@pytest.mark.parametrize("form", ["dir", "trie", "bkt"])
def test_pmd_dir24_rule_counters(gpu_ctx_factory, form):
    """FW stage DIR-24-8 in HBM, the route stage DIR-24-8 or trie, per-rule
    hit counters (the EXT kernel): counters equal the oracle's hits over
    every posted batch."""
    rules = fw1k()
    rts = routes()
    ctx = gpu_ctx_factory(stages=S | F | L, flags=cg.CFG_FW_FORCE_DIR24 | cg.CFG_RULE_COUNTERS
                          | {"dir": 0, "trie": cg.CFG_LPM_TRIE, "bkt": cg.CFG_LPM_BKT}[form])
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    ctx.set_route_lpm(cg.LpmTable(rts, 1 << 20, 1 << 16, False))
    B, P = 65536, 6
    pk = cg.gen_trace(0x5EED0B40, B * P, rules, rts)
    fw, rt = oracle_tables(rules, rts)
    ro, fos = oracle_slots(pk, B, P, S | F | L, fw, rt)
    rg = Ring(ctx, pk, B, P)
    with ctx.pmd_start(rg.ring) as m:
        m.post(P)
        m.post(2)
        m.wait()
    check(*rg.read(), ro, fos, B, P)
    hits = ctx.rule_counters()
    per_slot = [int(np.sum((ro["flags"][s * B:(s + 1) * B] & cg.FLAG_FW_HIT) != 0)) for s in range(P)]
    assert int(hits.sum()) == sum(per_slot) + per_slot[0] + per_slot[1]


def test_pmd_demux_port_stats(gpu_ctx_factory):
    """One ordered forward list per vport and per-port counters."""
    rules = fw1k()
    K = 5
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_DEMUX_PORTS | cg.CFG_PORT_STATS)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    B, P = 65536, 4
    pk = cg.gen_trace(0x5EED0B50, B * P, rules)
    fw, _ = oracle_tables(rules)
    ro, fos = oracle_slots(pk, B, P, S | F, fw)
    rg = Ring(ctx, pk, B, P, lists=K)
    with ctx.pmd_start(rg.ring) as m:
        m.post(P)
        m.wait()
    res, fwd, cnt = rg.read()
    assert np.array_equal(res.view(np.uint8), ro.view(np.uint8))
    for s in range(P):
        port = ro["port"][s * B:(s + 1) * B]
        for q in range(K):
            want = fos[s][port[fos[s]] == q]
            c = int(cnt[s * K + q])
            assert np.array_equal(fwd[s * B * K + q * B: s * B * K + q * B + c], want), f"slot {s} port {q}"
    ps = ctx.port_stats()
    for q in range(K):
        assert ps[q]["rx_packets"] == int(np.sum(ro["port"] == q))


def test_pmd_idle_exit_relaunch_and_restart(gpu_ctx_factory, monkeypatch):
    """The kernel leaves after an idle spell ($COP_PMD_IDLE_MS) and the next
    post relaunches it; tables cannot change under it (-EBUSY); after stop,
    one-shot launches and a second poll-mode kernel work on the context."""
    monkeypatch.setenv("COP_PMD_IDLE_MS", "50")
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F)
    tab = cg.LpmTable(rules, 1024, 24, True)
    ctx.set_fw_table(tab)
    B, P = 65536, 4
    pk = cg.gen_trace(0x5EED0B60, B * P, rules)
    fw, _ = oracle_tables(rules)
    ro, fos = oracle_slots(pk, B, P, S | F, fw)
    rg = Ring(ctx, pk, B, P)
    m = ctx.pmd_start(rg.ring)
    with pytest.raises(cg.CopError):
        ctx.set_fw_table(tab)
    m.post(2)
    m.wait()
    time.sleep(0.5)
    assert m.info()["state"] == 2            # left idle
    m.post(P)
    m.wait()
    assert m.info()["launches"] == 2
    check(*rg.read(), ro, fos, B, P)
    m.stop()
    ctx.set_fw_table(tab)                    # allowed again
    rg.dr.fill(0xAB)
    ctx.submit_ring(rg.ring, 0, P)
    ctx.sync()
    check(*rg.read(), ro, fos, B, P)
    rg.dr.fill(0xAB)
    with ctx.pmd_start(rg.ring) as m2:
        m2.post(P)
        m2.wait()
    check(*rg.read(), ro, fos, B, P)


def test_pmd_counter_reduce_while_serving(gpu_ctx_factory, monkeypatch):
    """The config-5 stall: with a poll-mode kernel live (a long
    idle spell, so it never leaves on its own) and 100k-rule per-rule
    counters, every RCCL counter reduce and every rule-counter read returns
    in well under 50 ms with exact sums. Side work pauses the kernel
    (cop_runtime.cpp pmd_pause / pmd_resume) instead of waiting for it to go
    idle — a side kernel is not guaranteed to run beside it."""
    monkeypatch.setenv("COP_PMD_IDLE_MS", "20000")
    fw_rules = cg.gen_rules(0x5EED1077, 100000, cg.GEN_FW, 0)
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_RULE_COUNTERS)
    ctx.set_fw_table(cg.LpmTable(fw_rules, 100000, 1 << 20, False))
    ctx.coll_init(cg.coll_unique_id(), 0, 1)
    ofw = orc.OracleLpm(100000, 1 << 20, rules_only=True)
    ofw.setup(fw_rules["ip"], fw_rules["depth"], fw_rules["next_hop"], stop_at_error=False)
    B, P = 65536, 4
    pk = cg.gen_trace(0x5EED0B70, B * P, fw_rules)
    hits = np.zeros(ofw.n_rules, np.uint64)
    ro, _, co = orc.process(pk, B * P, stages=S | F, fw=ofw, rule_hits=hits)
    assert hits.sum() > B
    rg = Ring(ctx, pk, B, P)
    ctx.counters(reset=True)
    times = []
    with ctx.pmd_start(rg.ring) as m:
        for rnd in range(5):
            m.post(P)
            m.wait()
            t0 = time.perf_counter()
            got = ctx.rule_counters()
            t1 = time.perf_counter()
            tot, red = ctx.coll_reduce_counters(reset=True)
            t2 = time.perf_counter()
            times.append((round((t1 - t0) * 1e3, 3), round((t2 - t1) * 1e3, 3)))
            assert np.array_equal(got, hits), f"round {rnd}: rule counters"
            assert np.array_equal(red, hits), f"round {rnd}: reduced rule counters"
            for k in co:
                assert tot[k] == co[k], (rnd, k, tot[k], co[k])
        res, _, _ = rg.read()
        assert np.array_equal(res.view(np.uint8), ro.view(np.uint8))
        assert m.info()["launches"] >= 1
    assert all(a < 50 and b < 50 for a, b in times), times


def test_pmd_look_back_give_up_completes_nothing(gpu_ctx_factory, monkeypatch):
    """a dense-list tile whose look-back gives up must not
    write its list or count, nor be counted for its slot. Tile 1 of batch 0
    never runs ($COP_PMD_TEST_SKIP_TILE, tests only), so tiles 2.. of that
    batch wait on a predecessor that never publishes: they time out, give up
    and the kernel aborts. The batch never completes (the wait reports the
    abort), its forward count is never written, and past tile 0's own
    entries the list is untouched."""
    monkeypatch.setenv("COP_PMD_TEST_SKIP_TILE", "1")
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    B, P = 65536, 2
    pk = cg.gen_trace(0x5EED0B80, B * P, rules)
    rg = Ring(ctx, pk, B, P)
    rg.df.fill(0xFF)
    m = ctx.pmd_start(rg.ring)
    tpb = m.info()["tiles_per_batch"]
    try:
        m.post(1)
        with pytest.raises(cg.CopError):
            m.wait()
        assert m.info()["state"] == 3          # aborted
    finally:
        try:
            m.stop()
        except cg.CopError:
            pass
    _, fwd, cnt = rg.read()
    assert int(cnt[0]) == 0xFFFFFFFF          # the last tile gave up: no count
    _, fos = oracle_slots(pk[:B * 64], B, 1, S | F, oracle_tables(rules)[0])
    c0 = int(np.sum(fos[0] < B // tpb))       # tile 0's forwarded packets
    assert np.array_equal(fwd[:c0], fos[0][:c0])
    assert (fwd[c0:B] == 0xFFFFFFFF).all()


@pytest.mark.parametrize("flags", [0, cg.PMD_SYS_ACQUIRE, cg.PMD_STATIC_SLOTS])
def test_pmd_imix_steps_ragged_and_rewritten(gpu_ctx_factory, flags):
    """IMIX on the poll-mode step path (segmented lists: offsets, headers,
    tbl24 and tbl8 of successive steps pipelined, cop_tile.h tile_steps_v):
    a ragged batch (20,003 packets: a last tile of 547 packets, a last step
    of 35), slots rewritten between generations (a new slab and new offsets
    each time, except with COP_PMD_STATIC_SLOTS), read with the plain,
    coherent-once-wrapped and coherent-every-tile loads; every generation's
    records and segment lists against the oracle."""
    from test_gpu_seg import nseg, seg_to_dense
    rules = fw1k()
    rts = routes(20000)
    ctx = gpu_ctx_factory(stages=S | F | L, flags=cg.CFG_SEG_LISTS)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    ctx.set_route_lpm(cg.LpmTable(rts, 1 << 20, 1 << 16, False))
    fw, rt = oracle_tables(rules, rts)
    B, P = 20003, 2
    gens = [cg.gen_imix(0x5EED0B60 + g, B, rules, rts) for g in range(6)]
    per = max(((sl.nbytes + of.nbytes + 4095) // 4096) * 4096 for sl, of in gens)
    dp = ctx.alloc(per * P)

    def put(g, s_):
        sl, of = gens[g]
        dp.upload(sl, s_ * per)
        dp.upload(of, s_ * per + per - of.nbytes)   # offsets at the slot's end (16-byte aligned)
    for s_ in range(P):
        put(s_, s_)
    FS = ((B + 3) // 4) * 4
    dr = ctx.alloc(B * P * 8)
    df = ctx.alloc(FS * P * 4)
    dc = ctx.alloc(P * nseg(B) * 4)
    offs_at = dp.addr + per - gens[0][1].nbytes
    assert all(of.nbytes == gens[0][1].nbytes for _, of in gens)
    ring = cg.make_ring(dp, P, B, dr, per, offsets=offs_at, offsets_slot_words=per // 4,
                        fwd_idx=df, fwd_slot=FS, fwd_count=dc)
    n_gen = 6 if flags != cg.PMD_STATIC_SLOTS else P
    with ctx.pmd_start(ring, flags) as m:
        assert m.info()["kernel_name"] == "cop_pmd<1, 2, 1, 4, false>"
        for g in range(n_gen):
            s_ = g % P
            if g >= P:
                put(g, s_)
            m.post(1)
            m.wait()
            sl, of = gens[g]
            ro, fo, _ = orc.process(sl, B, offsets=of, stages=S | F | L, fw=fw, route=rt)
            res = dr.download(cg.RESULT_DT, B * P)[s_ * B:(s_ + 1) * B]
            fwd = df.download(np.uint32, FS * P)[s_ * FS:s_ * FS + B]
            cnt = dc.download(np.uint32, P * nseg(B))[s_ * nseg(B):(s_ + 1) * nseg(B)]
            assert np.array_equal(res.view(np.uint8), ro.view(np.uint8)), f"generation {g} records"
            assert np.array_equal(seg_to_dense(fwd, cnt, B), fo), f"generation {g} list"
        assert m.info()["launches"] == 1


@pytest.mark.parametrize("stages", [S | F | L, F | L, S | L, L])
@pytest.mark.parametrize("form", ["dir", "bkt"])
def test_pmd_imix_steps_stage_masks(gpu_ctx_factory, stages, form):
    """The IMIX step path (segmented lists) with every stage mask that keeps
    the route stage, and both route forms it pipelines (DIR-24-8's tbl24 /
    tbl8, the bucketed index / pairs): the stage-P drop, the firewall's
    verdict and the route's next hop of every packet, and the segment lists,
    against the oracle."""
    from test_gpu_seg import nseg, seg_to_dense
    rules = fw1k()
    rts = routes(30000)
    ctx = gpu_ctx_factory(stages=stages, flags=cg.CFG_SEG_LISTS | (cg.CFG_LPM_BKT if form == "bkt" else 0))
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    ctx.set_route_lpm(cg.LpmTable(rts, 1 << 20, 1 << 16, False))
    assert ctx.route_form() == form
    B, P = 30001, 2
    opts = cg.trace_opts(pct_bad_version=5, pct_non_ipv4=5, pct_unknown_dst=5)
    slab, offs = cg.gen_imix(0x5EED0B70 + stages, B, rules, rts, opts=opts)
    per = ((slab.nbytes + offs.nbytes + 4095) // 4096) * 4096
    dp = ctx.alloc(per * P)
    for s_ in range(P):
        dp.upload(slab, s_ * per)
        dp.upload(offs, s_ * per + slab.nbytes)
    FS = ((B + 3) // 4) * 4
    dr = ctx.alloc(B * P * 8)
    df = ctx.alloc(FS * P * 4)
    dc = ctx.alloc(P * nseg(B) * 4)
    ring = cg.make_ring(dp, P, B, dr, per, offsets=dp.addr + slab.nbytes, offsets_slot_words=per // 4,
                        fwd_idx=df, fwd_slot=FS, fwd_count=dc)
    with ctx.pmd_start(ring) as m:
        fw_part = 1 if stages & F else 0
        lpm_part = 4 if form == "bkt" else 2
        assert m.info()["kernel_name"] == f"cop_pmd<{fw_part}, {lpm_part}, 1, 4, false>", m.info()
        m.run(5)
    fw, rt = oracle_tables(rules, rts)
    ro, fo, _ = orc.process(slab, B, offsets=offs, stages=stages, fw=fw, route=rt)
    res = dr.download(cg.RESULT_DT, B * P)
    fwd = df.download(np.uint32, FS * P)
    cnt = dc.download(np.uint32, P * nseg(B))
    for s_ in range(P):
        assert np.array_equal(res[s_ * B:(s_ + 1) * B].view(np.uint8), ro.view(np.uint8)), f"slot {s_}"
        assert np.array_equal(seg_to_dense(fwd[s_ * FS:s_ * FS + B], cnt[s_ * nseg(B):(s_ + 1) * nseg(B)], B), fo)
