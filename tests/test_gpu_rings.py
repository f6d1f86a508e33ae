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


def test_rings_over_2gib_need_static_slots(gpu_ctx_factory):
    """coherent slot loads take 31-bit offsets from the slot's
    base, so a ring whose batch spans 2 GiB or more (1M packets 2176 bytes
    apart, an mbuf pool's stride) is refused unless its slots are declared
    static (plain 64-bit addressing). Nothing is launched: the geometry is
    checked before the kernel starts."""
    rules = fw1k()
    n = 1 << 20
    ctx = gpu_ctx_factory(stages=S | F, max_batch=n)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    dp = ctx.alloc(1 << 20)   # the descriptor is only validated
    dr = ctx.alloc(n * 8)
    ring = cg.make_ring(dp, 1, n, dr, n * 2176, stride=2176)
    with pytest.raises(cg.CopError) as ei:
        ctx.pmd_start(ring)
    assert ei.value.code == -22
    with pytest.raises(cg.CopError):
        ctx.pmd_start(ring, cg.PMD_SYS_ACQUIRE)


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


@pytest.mark.parametrize("flags", [cg.PMD_SYS_ACQUIRE, 0])
def test_slots_rewritten_between_batches(gpu_ctx_factory, flags):
    """A producer that rewrites ring slots between batches (here the host,
    by cop_memcpy_h2d copies into HBM; on a real deployment a NIC, as the
    reference's fast path refills its rings, switch.c:463-470): each tile
    reads its slot with system-coherent (sc0 sc1) loads once the ring has
    wrapped (the default: flags 0 goes through the single-ring
    cop_pmd_start) or on every tile (COP_PMD_SYS_ACQUIRE), so a slot's new
    packets are read, never the previous batch's that a CU or L2 may still
    hold. Eight generations through a two-slot ring, records and lists per
    batch."""
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_SEG_LISTS)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    fw, _ = oracle_tables(rules)
    B, P = 65536, 2
    gens = [cg.gen_trace(0x5EED7500 + g, B, rules) for g in range(8)]
    rg = SegRing(ctx, np.concatenate([gens[0], gens[1]]), B, P)
    with ctx.pmd_start(rg.ring, flags) as m:
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
        assert m.info()["slot_loads"] == (3 if flags else 4)


def test_unaligned_slots_rewritten_between_batches(gpu_ctx_factory):
    """slots that do not start on 128-byte lines (4097 packets 64
    bytes apart: a slot's last packet shares its line with the next slot's
    first). Reading slot s's last packet caches the first line of slot s+1
    before the producer rewrites it, so a first-lap plain load of slot s+1
    could see stale bytes; such a ring takes coherent loads on every tile
    (slot_loads 3). Nine generations through three slots, every slot
    rewritten before its first post, records and lists per batch."""
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_SEG_LISTS)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    fw, _ = oracle_tables(rules)
    B, P = 4097, 3
    assert (B * 64) % 128 != 0
    gens = [cg.gen_trace(0x5EED7A00 + g, B, rules) for g in range(9)]
    # the slots hold an older generation when the kernel starts; lists of a
    # slot start 16-byte aligned (fwd_slot 4100)
    rg = SegRing(ctx, np.concatenate([cg.gen_trace(0x5EED7AF0, B, rules)] * P), B, P)
    FS = 4100
    rg.df = ctx.alloc(FS * P * 4)
    rg.ring = cg.make_ring(rg.dp, P, B, rg.dr, B * 64, fwd_idx=rg.df, fwd_slot=FS, fwd_count=rg.dc)
    with ctx.pmd_start(rg.ring) as m:
        assert m.info()["slot_loads"] == 3
        for g in range(9):
            s_ = g % P
            rg.dp.upload(gens[g], s_ * B * 64)
            m.post(1)
            m.wait()
            res = rg.dr.download(cg.RESULT_DT, B * P)[s_ * B:(s_ + 1) * B]
            fwd = rg.df.download(np.uint32, FS * P)[s_ * FS:s_ * FS + B]
            cnt = rg.dc.download(np.uint32, P * nseg(B))[s_ * nseg(B):(s_ + 1) * nseg(B)]
            ro, fo = oracle_batch(gens[g], B, S | F, fw)
            assert np.array_equal(res.view(np.uint8), ro.view(np.uint8)), f"generation {g}"
            assert np.array_equal(seg_to_dense(fwd, cnt, B), fo), f"generation {g} list"
        assert m.info()["launches"] == 1


@pytest.mark.parametrize("flags", [0, cg.PMD_DYNAMIC_TILES])
def test_host_slots_rewritten_in_place(gpu_ctx_factory, flags):
    """Slots in pinned host memory (cop_host_alloc_pinned: not coherent, so
    a GPU L2 may keep a copy of a line it read) rewritten in place by the
    CPU between batches, as the reference's fast path refills its rx ring
    (switch.c:463-470). Every step of every 1024-packet tile must read the
    new packets: the first step's loads and the later steps' refills alike
    (a one-step load window refills three of four). Eight generations
    through two 64k-packet slots, static and dynamic tiles."""
    import ctypes
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_SEG_LISTS)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    fw, _ = oracle_tables(rules)
    B, P = 65536, 2
    L_ = cg.lib()
    hp = ctypes.c_void_p()
    assert L_.cop_host_alloc_pinned(ctx.handle, B * P * 64, ctypes.byref(hp)) == 0
    try:
        gens = [np.ascontiguousarray(cg.gen_trace(0x5EED7600 + g, B, rules)) for g in range(8)]
        for s_ in range(P):
            ctypes.memmove(hp.value + s_ * B * 64, gens[s_].ctypes.data, B * 64)
        dr = ctx.alloc(B * P * 8)
        df = ctx.alloc(B * P * 4)
        dc = ctx.alloc(P * nseg(B) * 4)
        ring = cg.make_ring(hp.value, P, B, dr, B * 64, fwd_idx=df, fwd_slot=B, fwd_count=dc)
        with ctx.pmd_start(ring, flags) as m:
            for g in range(8):
                s_ = g % P
                if g >= P:
                    ctypes.memmove(hp.value + s_ * B * 64, gens[g].ctypes.data, B * 64)
                m.post(1)
                m.wait()
                res = dr.download(cg.RESULT_DT, B * P)[s_ * B:(s_ + 1) * B]
                fwd = df.download(np.uint32, B * P)[s_ * B:(s_ + 1) * B]
                cnt = dc.download(np.uint32, P * nseg(B))[s_ * nseg(B):(s_ + 1) * nseg(B)]
                ro, fo = oracle_batch(gens[g], B, S | F, fw)
                assert np.array_equal(res.view(np.uint8), ro.view(np.uint8)), f"generation {g}"
                assert np.array_equal(seg_to_dense(fwd, cnt, B), fo), f"generation {g} list"
            assert m.info()["launches"] == 1
    finally:
        L_.cop_host_free_pinned(ctx.handle, hp)


def test_static_slots_contradicts_acquire(gpu_ctx_factory):
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_SEG_LISTS)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    rg = SegRing(ctx, cg.gen_trace(0x5EED7510, 2 * 65536, rules), 65536, 2)
    with pytest.raises(cg.CopError):
        ctx.pmd_start(rg.ring, cg.PMD_SYS_ACQUIRE | cg.PMD_STATIC_SLOTS)
    with ctx.pmd_start(rg.ring, cg.PMD_STATIC_SLOTS) as m:   # the bench's declaration
        m.run(4)
        assert m.info()["slot_loads"] == 0
    assert ctx.counters()["rx"] == 4 * 65536


def fw_hits_per_slot(pk, B, P, fw):
    """FW hits (records with the FW-hit flag) of each slot's batch."""
    out = []
    for s_ in range(P):
        r, _ = oracle_batch(pk[s_ * B * 64:(s_ + 1) * B * 64], B, S | F, fw)
        out.append(int(((r["flags"] & 2) != 0).sum()))
    return out


@pytest.mark.parametrize("rule_counters", [False, True])
def test_pause_while_rings_post_from_threads(gpu_ctx_factory, rule_counters):
    """every counter read pauses the poll-mode kernel (it finishes
    the batches below its gates, leaves, and is relaunched from each ring's
    first incomplete batch). Four rings posted and waited by four threads
    while a fifth thread reads the counters (and, with per-rule counters,
    reads and zeroes them) in a loop, so pauses land while other threads have
    batches in flight and while they post: every ring's records and lists
    stay bit-exact, the packet count and the per-rule hit totals are exact
    (each batch counted once), and the kernel was relaunched."""
    rules = fw1k()
    flags = cg.CFG_SEG_LISTS | (cg.CFG_RULE_COUNTERS if rule_counters else 0)
    ctx = gpu_ctx_factory(stages=S | F, flags=flags)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    fw, _ = oracle_tables(rules)
    B, P, R = 65536, 4, 4
    pks = [cg.gen_trace(0x5EED7600 + r, B * P, rules) for r in range(R)]
    rgs = [SegRing(ctx, pk, B, P) for pk in pks]
    posted = [0] * R
    stop = threading.Event()
    reads = [0]
    hits_read = [0]
    seen_rx = []
    m = ctx.pmd_start([g.ring for g in rgs])

    def reader():
        while not stop.is_set():
            seen_rx.append(ctx.counters()["rx"])
            if rule_counters:
                hits_read[0] += int(ctx.rule_counters(reset=True).sum())
            reads[0] += 1

    def feeder(r):
        def f():
            for i in range(24):
                k = 1 + (i + r) % 3
                m.post_ring(r, k)
                posted[r] += k
                if i % 4 == 3:
                    m.wait_ring(r)
            m.wait_ring(r)
        return f

    rd = threading.Thread(target=reader)
    rd.start()
    try:
        run_threads([feeder(r) for r in range(R)])
    finally:
        stop.set()
        rd.join(120)
    assert not rd.is_alive(), "the counter reader hung"
    launches = m.info()["launches"]
    m.stop()
    for r in range(R):
        rgs[r].check(pks[r], S | F, fw)
    assert ctx.counters()["rx"] == sum(posted) * B
    assert seen_rx == sorted(seen_rx)                       # counts never go back
    assert reads[0] >= 2 and launches >= 2, (reads[0], launches)
    if rule_counters:
        per_slot = [fw_hits_per_slot(pks[r], B, P, fw) for r in range(R)]
        want = sum(per_slot[r][b % P] for r in range(R) for b in range(posted[r]))
        assert hits_read[0] + int(ctx.rule_counters().sum()) == want


def test_completed_count_never_moves_back(gpu_ctx_factory):
    """a ring's completed count is read and raised by threads
    other than the ring's own (cop_pmd_completed_ring, and the binned-hit
    flush of cop_rule_counters_read for ring 0). One thread posts a 4-slot
    ring one batch at a time far past its slots while another calls both in
    a loop: the count it sees never falls, the poster never stalls on a
    count moved back below a reposted slot, and the hits are exact."""
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_SEG_LISTS | cg.CFG_RULE_COUNTERS)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    fw, _ = oracle_tables(rules)
    B, P, N = 65536, 4, 96
    pk = cg.gen_trace(0x5EED7700, B * P, rules)
    rg = SegRing(ctx, pk, B, P)
    stop = threading.Event()
    seen = []
    m = ctx.pmd_start(rg.ring)

    def watcher():
        while not stop.is_set():
            seen.append(m.completed_ring(0))
            ctx.rule_counters()
            time.sleep(0)

    def poster():
        for i in range(N):
            m.post(1)
            if i % 8 == 7:
                m.wait()
        m.wait()

    w = threading.Thread(target=watcher)
    w.start()
    try:
        t0 = time.time()
        run_threads([poster])
        assert time.time() - t0 < 60
    finally:
        stop.set()
        w.join(120)
    assert not w.is_alive()
    assert seen == sorted(seen) and seen[-1] <= N
    m.stop()
    rg.check(pk, S | F, fw)
    per_slot = fw_hits_per_slot(pk, B, P, fw)
    assert int(ctx.rule_counters().sum()) == sum(per_slot[b % P] for b in range(N))
