"""Packed 16-byte header records (COP_HDR16_STRIDE, include/cop_gpu.h): the
end-to-end host path gathers frame bytes 12..15 and 24..35 of every packet
(the only bytes get_next_hop switch.c:93-136 and fw_packet_handler
firewall.c:170-213 read) instead of a 64-byte header line.

CPU: cop_pack_headers equals the numpy restatement on frames scattered over
an mbuf-like pool. GPU: batches and rings of packed records give the same
records and forward lists as the oracle on the frames, for every stage mix,
including ragged batch sizes and the host paths that now use them."""
import numpy as np
import pytest

import copgpu as cg
import oracle as orc
from helpers import oracle_tables

S, F, L = cg.STAGE_PARSE, cg.STAGE_FW, cg.STAGE_LPM


def scattered(pk, n, stride=2176, headroom=128):
    """Frames copied into an mbuf-like pool; returns (pool, u64 addresses)."""
    pool = np.zeros(n * stride + 64, np.uint8)
    for i in range(n):
        pool[i * stride + headroom: i * stride + headroom + 64] = pk[i * 64:(i + 1) * 64]
    ptrs = pool.ctypes.data + headroom + np.arange(n, dtype=np.uint64) * stride
    return pool, ptrs


def test_pack_headers_matches_numpy():
    rules = cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)
    n = 5000
    pk = cg.gen_trace(0x5EED0C00, n, rules)
    pool, ptrs = scattered(pk, n)
    got = cg.pack_headers(ptrs)
    want = cg.pack_headers_np(pk, n)
    assert got.nbytes == n * cg.HDR16_STRIDE
    assert np.array_equal(got, want)
    # the fields sit where the kernel expects them: EtherType in bytes 0..1,
    # version nibble in byte 2, src at 6..9 and dst at 10..13 (big-endian)
    rec = got.reshape(n, 16)
    fr = pk.reshape(n, 64)
    assert np.array_equal(rec[:, 0:2], fr[:, 12:14])
    assert np.array_equal(rec[:, 2] >> 4, fr[:, 14] >> 4)
    assert np.array_equal(rec[:, 6:10], fr[:, 26:30])
    assert np.array_equal(rec[:, 10:14], fr[:, 30:34])
    del pool


@pytest.mark.gpu
@pytest.mark.parametrize("stages", [S, S | F, S | F | L])
def test_hdr16_batches_bit_exact(gpu_ctx_factory, stages):
    rules = cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)
    rts = cg.gen_rules(0x5EED2004, 100000, cg.GEN_ROUTES, 0)
    ctx = gpu_ctx_factory(stages=stages)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    ctx.set_route_lpm(cg.LpmTable(rts, 1 << 20, 1 << 16, False))
    sizes = [0, 1, 255, 1025, 65536, 3, 200000]
    n = sum(sizes)
    pk = cg.gen_trace(0x5EED0C10, n, rules, rts)
    rec = cg.pack_headers_np(pk, n)
    dp = ctx.alloc(rec.nbytes + 16)
    dp.upload(rec)
    dr = ctx.alloc(n * 8)
    df = ctx.alloc(n * 4)
    dc = ctx.alloc(len(sizes) * 4)
    dc.fill(0xFF)
    bl, lo = [], 0
    for i, m in enumerate(sizes):
        bl.append(cg.make_batch(dp.addr + lo * 16, m, dr.addr + lo * 8, stride=cg.HDR16_STRIDE,
                                fwd_idx=df.addr + lo * 4, fwd_count=dc.addr + i * 4))
        lo += m
    ctx.submit(bl)
    ctx.sync()
    res = dr.download(cg.RESULT_DT, n)
    fwd = df.download(np.uint32, n)
    cnt = dc.download(np.uint32, len(sizes))
    fw, rt = oracle_tables(rules, rts)
    lo = 0
    for i, m in enumerate(sizes):
        r, f, _ = orc.process(pk[lo * 64:(lo + m) * 64], m, stages=stages, fw=fw, route=rt)
        assert np.array_equal(res[lo:lo + m].view(np.uint8), r.view(np.uint8)), f"batch {i}"
        assert int(cnt[i]) == len(f), f"batch {i} count"
        assert np.array_equal(fwd[lo:lo + len(f)], f), f"batch {i} forward list"
        lo += m


@pytest.mark.gpu
def test_hdr16_ring_bench_shape(gpu_ctx_factory):
    """A ring of packed-record slots (64k packets each), one launch."""
    rules = cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)
    ctx = gpu_ctx_factory(stages=S | F)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    B, P = 65536, 12
    pk = cg.gen_trace(0x5EED0C20, B * P, rules)
    rec = cg.pack_headers_np(pk, B * P)
    dp = ctx.alloc(rec.nbytes)
    dp.upload(rec)
    dr = ctx.alloc(B * P * 8)
    df = ctx.alloc(B * P * 4)
    dc = ctx.alloc(P * 4)
    ring = cg.make_ring(dp, P, B, dr, B * 16, stride=cg.HDR16_STRIDE, fwd_idx=df, fwd_slot=B, fwd_count=dc)
    ctx.submit_ring(ring, 5, P)
    ctx.sync()
    res = dr.download(cg.RESULT_DT, B * P)
    fwd = df.download(np.uint32, B * P)
    cnt = dc.download(np.uint32, P)
    fw, _ = oracle_tables(rules)
    ro, _, _ = orc.process(pk, B * P, stages=S | F, fw=fw)
    assert np.array_equal(res.view(np.uint8), ro.view(np.uint8))
    for s in range(P):
        sl = slice(s * B, (s + 1) * B)
        want = np.nonzero(ro["verdict"][sl] == cg.FORWARD)[0].astype(np.uint32)
        assert int(cnt[s]) == len(want)
        assert np.array_equal(fwd[s * B: s * B + len(want)], want)


@pytest.mark.gpu
def test_hdr16_mixed_submit_rejected(gpu_ctx_factory):
    """Packed records and frames cannot share one launch."""
    ctx = gpu_ctx_factory(stages=S | F)
    ctx.set_fw_table(cg.LpmTable(cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20), 1024, 24, True))
    dp = ctx.alloc(1 << 20)
    dr = ctx.alloc(1 << 20)
    bl = [cg.make_batch(dp.addr, 100, dr.addr, stride=cg.HDR16_STRIDE),
          cg.make_batch(dp.addr + 65536, 100, dr.addr + 4096, stride=64)]
    with pytest.raises(cg.CopError):
        ctx.submit(bl)


@pytest.mark.gpu
def test_hdr16_with_demux_port_stats_and_rule_counters(gpu_ctx_factory):
    """Packed records through the kernels built with the optional features
    (EXT): per-port ordered forward lists, per-port statistics and per-rule
    hit counters equal the oracle's on the frames."""
    rules = cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_DEMUX_PORTS | cg.CFG_PORT_STATS | cg.CFG_RULE_COUNTERS)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    B, NS, P = 65536, 3, 5
    pk = cg.gen_trace(0x5EED0C30, B * NS, rules)
    rec = cg.pack_headers_np(pk, B * NS)
    dp = ctx.alloc(rec.nbytes)
    dp.upload(rec)
    dr = ctx.alloc(B * NS * 8)
    df = ctx.alloc(B * NS * P * 4)
    dc = ctx.alloc(NS * P * 4)
    rg = cg.make_ring(dp, NS, B, dr, B * 16, stride=cg.HDR16_STRIDE, fwd_idx=df, fwd_count=dc, fwd_slot=B * P)
    ctx.submit_ring(rg, 0, NS)
    ctx.sync()
    res = dr.download(cg.RESULT_DT, B * NS)
    cnt = dc.download(np.uint32, NS * P).reshape(NS, P)
    fwd_all = df.download(np.uint32, B * NS * P)
    fw, _ = oracle_tables(rules)
    ro_all = []
    for s in range(NS):
        ro, _, _ = orc.process(pk[s * B * 64:(s + 1) * B * 64], B, stages=S | F, fw=fw)
        ro_all.append(ro)
        assert np.array_equal(res[s * B:(s + 1) * B].view(np.uint8), ro.view(np.uint8)), s
        for q in range(P):
            want = np.nonzero((ro["verdict"] == 0) & (ro["port"] == q))[0].astype(np.uint32)
            got = fwd_all[s * B * P + q * B: s * B * P + q * B + cnt[s, q]]
            assert np.array_equal(got, want), (s, q)
    ro = np.concatenate(ro_all)
    ps = ctx.port_stats()
    for q in range(P):
        assert ps[q]["rx_packets"] == int(np.sum(ro["port"] == q))
        assert ps[q]["tx_packets"] == int(np.sum((ro["port"] == q) & (ro["verdict"] == 0)))
    hits = ctx.rule_counters()
    assert int(hits.sum()) == int(np.sum((ro["flags"] & cg.FLAG_FW_HIT) != 0))


@pytest.mark.gpu
def test_host_batch_slots_submit_wait(gpu_ctx_factory):
    """cop_host_batch_submit / _wait: two slots in flight at once on mapped
    pinned memory, results bit-exact against the oracle, a busy slot refuses
    a second submit (-EBUSY), an idle slot refuses a wait (-EINVAL)."""
    import ctypes
    rules = cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)
    ctx = gpu_ctx_factory(stages=S | F)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    n = 20000
    pk = cg.gen_trace(0x5EED0C40, 2 * n, rules)
    pool, ptrs = scattered(pk, 2 * n)
    fw, _ = oracle_tables(rules)
    ro, _, _ = orc.process(pk, 2 * n, stages=S | F, fw=fw)
    L = cg.lib()
    p0 = ctypes.c_void_p(int(ptrs.ctypes.data))
    p1 = ctypes.c_void_p(int(ptrs.ctypes.data) + n * 8)
    assert L.cop_host_batch_submit(ctx.handle, 0, p0, n) == 0
    assert L.cop_host_batch_submit(ctx.handle, 1, p1, n) == 0
    assert L.cop_host_batch_submit(ctx.handle, 0, p0, n) == -16      # EBUSY
    for s in (0, 1):
        rp = ctypes.c_void_p()
        cnt = ctypes.c_uint32()
        assert L.cop_host_batch_wait(ctx.handle, s, ctypes.byref(rp), ctypes.byref(cnt)) == 0
        assert cnt.value == n
        got = np.frombuffer((ctypes.c_uint8 * (n * 8)).from_address(rp.value), dtype=cg.RESULT_DT).copy()
        assert np.array_equal(got.view(np.uint8), ro[s * n:(s + 1) * n].view(np.uint8)), s
    assert L.cop_host_batch_wait(ctx.handle, 0, None, None) == -22      # EINVAL: nothing in flight
    del pool
