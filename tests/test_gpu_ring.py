"""GPU parity at bench-scale launch shapes (csrc/cop_kernels.hip: coalesced
loads, batches interleaved over workgroups, LDS-staged forward lists):
batch rings of 64k-packet slots (the bench's layout), DIR-24-8 stages, demux
and port statistics, rule counters, non-uniform descriptor batches, and the
runtime's state hand-offs between launches on one lane (ticket buffers,
look-back growth, counter resets). Bit-exact against the oracle on every
record and every forward list.
"""
import numpy as np
import pytest

import copgpu as cg
import oracle as orc
from helpers import oracle_tables

pytestmark = pytest.mark.gpu

S = cg.STAGE_PARSE
F = cg.STAGE_FW
L = cg.STAGE_LPM


def fw1k(seed=0x5EED1002):
    return cg.gen_rules(seed, 1000, cg.GEN_FW, 20)


def routes(n=100000, seed=0x5EED2004):
    return cg.gen_rules(seed, n, cg.GEN_ROUTES, 0)


def run_ring(ctx, pk, B, P, first, count, stride=64, data_off=0, fwd_lists=1):
    """Upload P slots of B packets (slot layout stride/data_off), run one ring
    launch of `count` slots from `first`, return per-slot records, forward
    lists (per port with demux) and counts."""
    slot_bytes = ((B * stride + data_off + 4095) // 4096) * 4096
    dp = ctx.alloc(slot_bytes * P)
    if stride == 64 and data_off == 0:
        for s in range(P):
            dp.upload(pk[s * B * 64:(s + 1) * B * 64], s * slot_bytes)
    else:
        for s in range(P):
            buf = np.zeros(slot_bytes, np.uint8)
            v = buf[data_off:data_off + B * stride].reshape(B, stride)
            v[:, :64] = pk[s * B * 64:(s + 1) * B * 64].reshape(B, 64)
            dp.upload(buf, s * slot_bytes)
    dr = ctx.alloc(B * P * 8)
    df = ctx.alloc(B * P * 4 * fwd_lists)
    dc = ctx.alloc(P * 4 * fwd_lists)
    dr.fill(0xAB)
    dc.fill(0xFF)
    ring = cg.make_ring(dp, P, B, dr, slot_bytes, stride=stride, data_off=data_off, fwd_idx=df,
                        fwd_slot=B * fwd_lists, fwd_count=dc)
    ctx.submit_ring(ring, first, count)
    ctx.sync()
    res = dr.download(cg.RESULT_DT, B * P)
    fwd = df.download(np.uint32, B * P * fwd_lists)
    cnt = dc.download(np.uint32, P * fwd_lists)
    for x in (dp, dr, df, dc):
        x.free()
    return res, fwd, cnt


def check_slots(res, fwd, cnt, ro, fo_slot, B, slots):
    for s in slots:
        got = res[s * B:(s + 1) * B]
        want = ro[s * B:(s + 1) * B]
        assert np.array_equal(got.view(np.uint8), want.view(np.uint8)), f"slot {s} records differ"
        c = int(cnt[s])
        assert np.array_equal(fwd[s * B: s * B + c], fo_slot[s]), f"slot {s} forward list differs"


def oracle_slots(pk, B, P, stages, fw, rt=None):
    recs, fos = [], []
    for s in range(P):
        r, f, _ = orc.process(pk[s * B * 64:(s + 1) * B * 64], B, stages=stages, fw=fw, route=rt)
        recs.append(r)
        fos.append(f)
    return np.concatenate(recs), fos


def test_auto_ring_fw1k_bench_shape(gpu_ctx_factory):
    """The bench's layout: 64k-packet slots, 40 slots in one ring launch
    (2.6M packets), wrapping; the kernel the library picks by itself."""
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    B, P = 65536, 40
    pk = cg.gen_trace(0x5EED0A00, B * P, rules)
    fw, _ = oracle_tables(rules)
    ro, fos = oracle_slots(pk, B, P, S | F, fw)
    res, fwd, cnt = run_ring(ctx, pk, B, P, 7, P)
    check_slots(res, fwd, cnt, ro, fos, B, range(P))
    c = ctx.counters()
    assert c["rx"] == B * P and c["forward"] == sum(len(f) for f in fos)


@pytest.mark.parametrize("fw_dir", [False, True])
def test_ring_fw_lpm_dir24(gpu_ctx_factory, fw_dir):
    """FW + route LPM 100k (DIR-24-8 in HBM: the late-prefetch variant),
    firewall either in LDS or forced to DIR-24-8 too."""
    rules = fw1k()
    rts = routes()
    flags = cg.CFG_FW_FORCE_DIR24 if fw_dir else 0
    ctx = gpu_ctx_factory(stages=S | F | L, flags=flags)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    ctx.set_route_lpm(cg.LpmTable(rts, 1 << 20, 1 << 16, False))
    B, P = 65536, 36
    pk = cg.gen_trace(0x5EED0A10, B * P, rules, rts)
    fw, rt = oracle_tables(rules, rts)
    ro, fos = oracle_slots(pk, B, P, S | F | L, fw, rt)
    res, fwd, cnt = run_ring(ctx, pk, B, P, 0, P)
    check_slots(res, fwd, cnt, ro, fos, B, range(P))


def test_ring_mbuf_layout(gpu_ctx_factory):
    """Slots at mbuf stride (2176 B) with 128 B headroom."""
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    B, P = 30000 + 5, 5
    pk = cg.gen_trace(0x5EED0A20, B * P, rules)
    fw, _ = oracle_tables(rules)
    ro, fos = oracle_slots(pk, B, P, S | F, fw)
    res, fwd, cnt = run_ring(ctx, pk, B, P, 2, P, stride=2176, data_off=128)
    check_slots(res, fwd, cnt, ro, fos, B, range(P))


def test_descriptor_ragged_batches(gpu_ctx_factory):
    """Descriptor submit with non-uniform batches (0, 1, 255, 1025, 70000,
    and large ones): the tile -> batch scan."""
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    sizes = [0, 1, 255, 1025, 70000, 262144, 3, 200000, 0, 131072]
    n = sum(sizes)
    pk = cg.gen_trace(0x5EED0A30, n, rules)
    dp = ctx.alloc(pk.nbytes)
    dp.upload(pk)
    dr = ctx.alloc(n * 8)
    df = ctx.alloc(n * 4)
    dc = ctx.alloc(len(sizes) * 4)
    dc.fill(0xFF)
    bl, lo = [], 0
    for i, m in enumerate(sizes):
        bl.append(cg.make_batch(dp.addr + lo * 64, m, dr.addr + lo * 8, fwd_idx=df.addr + lo * 4,
                                fwd_count=dc.addr + i * 4))
        lo += m
    ctx.submit(bl)
    ctx.sync()
    res = dr.download(cg.RESULT_DT, n)
    fwd = df.download(np.uint32, n)
    cnt = dc.download(np.uint32, len(sizes))
    fw, _ = oracle_tables(rules)
    lo = 0
    for i, m in enumerate(sizes):
        r, f, _ = orc.process(pk[lo * 64:(lo + m) * 64], m, stages=S | F, fw=fw)
        assert np.array_equal(res[lo:lo + m].view(np.uint8), r.view(np.uint8)), f"batch {i}"
        assert int(cnt[i]) == len(f), f"batch {i} count"
        assert np.array_equal(fwd[lo:lo + len(f)], f), f"batch {i} forward list"
        lo += m


def test_ring_demux_port_stats(gpu_ctx_factory):
    """Per-port ordered forward lists and per-port counters at bench scale."""
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_DEMUX_PORTS | cg.CFG_PORT_STATS)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    B, P, K = 65536, 36, 5
    pk = cg.gen_trace(0x5EED0A40, B * P, rules)
    fw, _ = oracle_tables(rules)
    ro, fos = oracle_slots(pk, B, P, S | F, fw)
    res, fwd, cnt = run_ring(ctx, pk, B, P, 0, P, fwd_lists=K)
    assert np.array_equal(res.view(np.uint8), ro.view(np.uint8))
    for s in range(P):
        port = ro["port"][s * B:(s + 1) * B]
        for q in range(K):
            want = fos[s][port[fos[s]] == q]
            c = int(cnt[s * K + q])
            got = fwd[s * B * K + q * B: s * B * K + q * B + c]
            assert np.array_equal(got, want), f"slot {s} port {q}"
    ps = ctx.port_stats()
    for q in range(K):
        assert ps[q]["rx_packets"] == int(np.sum(ro["port"] == q))
        assert ps[q]["tx_packets"] == int(np.sum((ro["port"] == q) & (ro["verdict"] == 0)))


@pytest.mark.parametrize("ppt", ["1", "4", "8"])
def test_lane_state_handoffs(gpu_ctx_factory, monkeypatch, ppt):
    """Launches of growing size on ONE lane: every tile size ($COP_PPT) and
    launches long enough to outgrow the lane's look-back words (the growth
    path re-zeroes them in stream order before the kernel that uses them),
    the ticket buffers' double-buffer protocol across launches, and a
    counter reset between launches (it completes before the next kernel).
    The 64-slot launch at PPT 1 (16384 tiles) once hit a look-back timeout
    when the growth used an unordered null-stream memset."""
    monkeypatch.setenv("COP_PPT", ppt)
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, n_streams=1, max_batch=65536, max_batches=4)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    B, P = 65536, 8
    pk = cg.gen_trace(0x5EED0A50, B * P, rules)
    fw, _ = oracle_tables(rules)
    ro, fos = oracle_slots(pk, B, P, S | F, fw)
    dp = ctx.alloc(B * 64 * P)
    dp.upload(pk)
    dr = ctx.alloc(B * P * 8)
    df = ctx.alloc(B * P * 4)
    dc = ctx.alloc(P * 4)
    ring = cg.make_ring(dp, P, B, dr, B * 64, stride=64, fwd_idx=df, fwd_slot=B, fwd_count=dc)
    total = 0
    for i, count in enumerate((1, 4, 20, 64, 3, 64, 128)):
        ctx.submit_ring(ring, i % P, count)
        total += count
        if i == 2:
            ctx.sync()
            assert ctx.counters(reset=True)["rx"] == total * B
            total = 0
    ctx.sync()
    res = dr.download(cg.RESULT_DT, B * P)
    fwd = df.download(np.uint32, B * P)
    cnt = dc.download(np.uint32, P)
    check_slots(res, fwd, cnt, ro, fos, B, range(P))
    assert ctx.counters()["rx"] == total * B


def test_ring_rule_counters(gpu_ctx_factory):
    """Per-rule hit counters at bench scale equal the oracle's per-rule hits
    summed over the launch."""
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_RULE_COUNTERS)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    B, P = 65536, 8
    pk = cg.gen_trace(0x5EED0A60, B * P, rules)
    res, fwd, cnt = run_ring(ctx, pk, B, P, 0, P)
    hits = ctx.rule_counters()
    fw, _ = oracle_tables(rules)
    ro, _, _ = orc.process(pk, B * P, stages=S | F, fw=fw)
    assert np.array_equal(res.view(np.uint8), ro.view(np.uint8))
    assert int(hits.sum()) == int(np.sum((ro["flags"] & cg.FLAG_FW_HIT) != 0))


def test_max_ring_launch_1024_slots_wrapping(gpu_ctx_factory):
    """The bench's launch size: 1024 batches in ONE ring launch (the ticket
    buffers' full 1024 lines, 1024 look-back chains), over a ring of 300
    slots so the launch wraps it three times (a slot's batches in one launch
    write identical outputs). Two launches back to back, so the second one
    draws from the ticket buffer the first one zeroed."""
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    B, P = 4096 + 77, 300
    pk = cg.gen_trace(0x5EED0A70, B * P, rules)
    fw, _ = oracle_tables(rules)
    ro, fos = oracle_slots(pk, B, P, S | F, fw)
    dp = ctx.alloc(B * 64 * P)
    dp.upload(pk)
    dr = ctx.alloc(B * P * 8)
    df = ctx.alloc(B * P * 4)
    dc = ctx.alloc(P * 4)
    dc.fill(0xFF)
    ring = cg.make_ring(dp, P, B, dr, B * 64, stride=64, fwd_idx=df, fwd_slot=B, fwd_count=dc)
    ctx.submit_ring(ring, 123, 1024)
    ctx.submit_ring(ring, 7, 1024)
    ctx.sync()
    res = dr.download(cg.RESULT_DT, B * P)
    fwd = df.download(np.uint32, B * P)
    cnt = dc.download(np.uint32, P)
    check_slots(res, fwd, cnt, ro, fos, B, range(P))
    c = ctx.counters()
    assert c["rx"] == 2 * 1024 * B
