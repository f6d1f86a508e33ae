"""One poll-mode kernel serving several rx rings (cop_pmd_start_rings): the
GPU form of the reference's five coprocessor lcores, each polling its own
rx ring (KNI_KTHREAD = 5, main.c:92-94; coprocessor(), switch.c:443-474).
Each ring is posted and waited by its own host thread; every ring's records
and ordered forward lists must equal the oracle's bit for bit, in that
ring's own batch order."""
import threading
import time

import numpy as np
import pytest

import copgpu as cg
import oracle as orc
from helpers import oracle_tables
from test_gpu_seg import SegRing, fw1k, nseg, oracle_batch, seg_to_dense

pytestmark = pytest.mark.gpu

S, F, L = cg.STAGE_PARSE, cg.STAGE_FW, cg.STAGE_LPM


def run_threads(fns):
    errs = []

    def wrap(f):
        try:
            f()
        except BaseException as e:  # noqa: BLE001 (re-raised in the test thread)
            errs.append(e)

    th = [threading.Thread(target=wrap, args=(f,)) for f in fns]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not any(t.is_alive() for t in th), "a ring thread hung"
    if errs:
        raise errs[0]


@pytest.mark.parametrize("flags", [cg.CFG_SEG_LISTS, 0])
def test_five_rings_five_threads(gpu_ctx_factory, flags):
    """Five rings (distinct traces), five threads each posting its ring in
    posts of 1..4 batches that wrap it, one kernel: per-ring bit-exact
    records and lists (segmented, and dense with its per-(ring, slot)
    look-back chains); the counters sum every ring's packets."""
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=flags)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    fw, _ = oracle_tables(rules)
    B, P, R = 65536, 4, 5
    pks = [cg.gen_trace(0x5EED7000 + r, B * P, rules) for r in range(R)]
    if flags:
        rgs = [SegRing(ctx, pk, B, P) for pk in pks]
    else:
        from test_gpu_pmd import Ring
        rgs = [Ring(ctx, pk, B, P) for pk in pks]
    posted = [0] * R
    with ctx.pmd_start([g.ring for g in rgs]) as m:
        assert m.info()["workers"] >= R

        def feeder(r):
            def f():
                for i in range(9):
                    k = 1 + (i + r) % 4
                    m.post_ring(r, k)
                    posted[r] += k
                    if i % 3 == 2:
                        m.wait_ring(r)
                m.wait_ring(r)
                assert m.completed_ring(r) == posted[r]
            return f

        run_threads([feeder(r) for r in range(R)])
        for r in range(R):
            if flags:
                rgs[r].check(pks[r], S | F, fw)
            else:
                from test_gpu_pmd import check, oracle_slots
                ro, fos = oracle_slots(pks[r], B, P, S | F, fw)
                check(*rgs[r].read(), ro, fos, B, P)
        assert m.info()["posted"] == sum(posted)
    assert ctx.counters()["rx"] == sum(posted) * B


def test_variable_size_batches(gpu_ctx_factory):
    """COP_PMD_VARIABLE_N: each post carries its batch's packet count (the
    drop-in loop's drains are not a fixed size); records and segment lists
    of the first n packets equal the oracle's on those n packets, and
    nothing past n is written."""
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_SEG_LISTS)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    fw, _ = oracle_tables(rules)
    B, P = 16384, 4
    pk = cg.gen_trace(0x5EED7100, B * P, rules)
    rg = SegRing(ctx, pk, B, P)
    sizes = [1, 255, 256, 4099, 16384, 1024, 7, 16383]
    total = 0
    with ctx.pmd_start(rg.ring, cg.PMD_VARIABLE_N) as m:
        for i, n in enumerate(sizes):
            s = i % P
            rg.dr.fill(0xEE) if s == 0 else None
            m.post_batch(0, n)
            m.wait_ring(0)
            total += n
            res = rg.dr.download(cg.RESULT_DT, B * P)[s * B:(s + 1) * B]
            fwd = rg.df.download(np.uint32, B * P)[s * B:(s + 1) * B]
            cnt = rg.dc.download(np.uint32, P * nseg(B))[s * nseg(B):(s + 1) * nseg(B)]
            r, f = oracle_batch(pk[s * B * 64:s * B * 64 + n * 64], n, S | F, fw)
            assert np.array_equal(res[:n].view(np.uint8), r.view(np.uint8)), f"batch {i} (n={n}) records"
            assert np.array_equal(seg_to_dense(fwd, cnt, n), f), f"batch {i} (n={n}) list"
            if s == 0 and n < B:
                assert np.all(res[n:].view(np.uint8) == 0xEE), f"batch {i}: records past n"
        with pytest.raises(cg.CopError):
            m.post_batch(0, B + 1)
    assert ctx.counters()["rx"] == total


def test_rings_idle_exit_races_posts(gpu_ctx_factory, monkeypatch):
    """Three rings posted by three threads at intervals around a 2 ms idle
    limit: the kernel leaves and is relaunched (by whichever thread sees it
    first) while other rings post; every batch of every ring completes with
    the oracle's outputs and the counters count each batch once."""
    monkeypatch.setenv("COP_PMD_IDLE_MS", "2")
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_SEG_LISTS)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    fw, _ = oracle_tables(rules)
    B, P, R = 65536, 4, 3
    pks = [cg.gen_trace(0x5EED7200 + r, B * P, rules) for r in range(R)]
    rgs = [SegRing(ctx, pk, B, P) for pk in pks]
    posted = [0] * R
    m = ctx.pmd_start([g.ring for g in rgs])

    def feeder(r):
        def f():
            for i in range(16):
                time.sleep((1.0 + 0.13 * ((i * 7 + r * 3) % 23)) * 1e-3)
                m.post_ring(r, 1)
                posted[r] += 1
            m.wait_ring(r)
        return f

    run_threads([feeder(r) for r in range(R)])
    launches = m.info()["launches"]
    m.stop()
    for r in range(R):
        rgs[r].check(pks[r], S | F, fw)
    assert ctx.counters()["rx"] == sum(posted) * B
    assert launches >= 2


def test_rings_reject_mismatched_geometry(gpu_ctx_factory):
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_SEG_LISTS)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    B = 65536
    pk = cg.gen_trace(0x5EED7300, B * 4, rules)
    a = SegRing(ctx, pk, B, 4)
    b = SegRing(ctx, pk[:B * 2 * 64], B, 2)   # two slots, not four
    with pytest.raises(cg.CopError):
        ctx.pmd_start([a.ring, b.ring])
    with pytest.raises(cg.CopError):
        ctx.pmd_start([a.ring] * 9)


@pytest.mark.parametrize("stages", [F, S | F])
def test_hdr16_rings_variable_n(gpu_ctx_factory, stages):
    """The drop-in's kernel shape through the batch-ring API: two rings of
    packed 16-byte header records (COP_HDR16_STRIDE), variable-size batches,
    no forward lists, the firewall alone (the drop-in's NF chain) or P + FW:
    records equal the oracle's for the first n packets of every batch."""
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=stages)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    fw, _ = oracle_tables(rules)
    B, P, R = 4096, 4, 2
    pks = [cg.gen_trace(0x5EED7400 + r, B * P, rules) for r in range(R)]
    bufs, rings = [], []
    for r in range(R):
        hdr = cg.pack_headers_np(pks[r], B * P)
        dp = ctx.alloc(hdr.nbytes)
        dp.upload(hdr)
        dr = ctx.alloc(B * P * 8)
        dr.fill(0xEE)
        bufs.append((dp, dr))
        rings.append(cg.make_ring(dp, P, B, dr, B * cg.HDR16_STRIDE, stride=cg.HDR16_STRIDE))
    sizes = [4096, 1, 2500, 1024, 1025, 77, 4095, 3000]
    with ctx.pmd_start(rings, cg.PMD_VARIABLE_N) as m:
        for i, n in enumerate(sizes):
            for r in range(R):
                m.post_batch(r, n)
            for r in range(R):
                m.wait_ring(r)
                s_ = i % P
                res = bufs[r][1].download(cg.RESULT_DT, B * P)[s_ * B:s_ * B + n]
                ro, _, _ = orc.process(pks[r][s_ * B * 64:(s_ * B + n) * 64], n, stages=stages, fw=fw)
                assert np.array_equal(res.view(np.uint8), ro.view(np.uint8)), f"ring {r} batch {i} (n={n})"


def test_slots_rewritten_between_batches(gpu_ctx_factory):
    """A producer that rewrites ring slots between batches (here the host,
    by copies into HBM; on a real deployment a NIC): with COP_PMD_SYS_ACQUIRE
    each tile acquires before its loads, so a slot's new packets are read,
    never the previous batch's that a CU or L2 may still hold. Eight
    generations through a two-slot ring, records and lists per batch."""
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_SEG_LISTS)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    fw, _ = oracle_tables(rules)
    B, P = 65536, 2
    gens = [cg.gen_trace(0x5EED7500 + g, B, rules) for g in range(8)]
    rg = SegRing(ctx, np.concatenate([gens[0], gens[1]]), B, P)
    with ctx.pmd_start(rg.ring, cg.PMD_SYS_ACQUIRE) as m:
        for g in range(8):
            s_ = g % P
            if g >= P:
                rg.dp.upload(gens[g], s_ * B * 64)
            m.post(1)
            m.wait()
            res = rg.dr.download(cg.RESULT_DT, B * P)[s_ * B:(s_ + 1) * B]
            fwd = rg.df.download(np.uint32, B * P)[s_ * B:(s_ + 1) * B]
            cnt = rg.dc.download(np.uint32, P * nseg(B))[s_ * nseg(B):(s_ + 1) * nseg(B)]
            ro, fo = oracle_batch(gens[g], B, S | F, fw)
            assert np.array_equal(res.view(np.uint8), ro.view(np.uint8)), f"generation {g}"
            assert np.array_equal(seg_to_dense(fwd, cnt, B), fo), f"generation {g} list"
        assert m.info()["launches"] == 1   # served by one launch: no relaunch invalidated the caches
