"""GPU: per-port demux, per-port statistics and live telemetry (SURVEY.md
§8f rows 3 and 4).

Demux (COP_CFG_DEMUX_PORTS): one ordered forward list per vport — what each
port's coprocessor would put on its tx_q (enqueue_nf_rx, switch.c:306-327;
coprocessor(), switch.c:464-470). The oracle's expectation is derived from
its own per-packet records: for port q, the indices i with verdict FORWARD
and port q, ascending.

Port stats (COP_CFG_PORT_STATS): coprocessor_stats per vport (switch.h:33-38)
— rx = packets routed to the port, tx = packets its NF forwarded.

Live snapshot: read-and-zero while launches are in flight loses nothing.
"""
import numpy as np
import pytest

import copgpu as cg
import oracle as orc
from helpers import oracle_tables

pytestmark = pytest.mark.gpu

S, F, L = cg.STAGE_PARSE, cg.STAGE_FW, cg.STAGE_LPM


def fw1k():
    return cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)


def expected_lists(res, n_ports):
    return [np.nonzero((res["verdict"] == 0) & (res["port"] == q))[0].astype(np.uint32) for q in range(n_ports)]


def expected_port_stats(res, n_ports):
    return [(int(((res["port"] == q)).sum()), int(((res["verdict"] == 0) & (res["port"] == q)).sum()))
            for q in range(n_ports)]


@pytest.mark.parametrize("n,batches", [(1000, 1), (65536, 1), (200000, 3), (262144, 7)])
def test_demux_descriptor_batches(gpu_ctx_factory, n, batches):
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_DEMUX_PORTS | cg.CFG_PORT_STATS)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    P = 5
    pk = cg.gen_trace(0x5EED0D00 + n, n, rules)
    fwo, _ = oracle_tables(rules)
    ro, fo, _ = orc.process(pk, n, stages=S | F, fw=fwo)
    dp = ctx.alloc(pk.nbytes)
    dp.upload(pk)
    dr = ctx.alloc(n * 8)
    bounds = np.linspace(0, n, batches + 1).astype(np.int64)
    sizes = np.diff(bounds)
    df = ctx.alloc(int(P * n * 4))
    dc = ctx.alloc(batches * P * 4)
    dc.fill(0xFF)
    bl = []
    for b in range(batches):
        lo = int(bounds[b])
        bl.append(cg.make_batch(dp.addr + lo * 64, int(sizes[b]), dr.addr + lo * 8,
                                fwd_idx=df.addr + lo * P * 4, fwd_count=dc.addr + b * P * 4))
    ctx.port_stats(reset=True)
    ctx.submit(bl)
    ctx.sync()
    res = dr.download(cg.RESULT_DT, n)
    assert np.array_equal(res.view(np.uint8), ro.view(np.uint8))
    cnt = dc.download(np.uint32, batches * P).reshape(batches, P)
    fwd_all = df.download(np.uint32, P * n)
    for b in range(batches):
        lo, m = int(bounds[b]), int(sizes[b])
        want = expected_lists(ro[lo:lo + m], P)
        for q in range(P):
            got = fwd_all[lo * P + q * m: lo * P + q * m + cnt[b, q]]
            assert cnt[b, q] == len(want[q]), (b, q)
            assert np.array_equal(got, want[q]), (b, q)
    ps = ctx.port_stats()
    for q, (rx, tx) in enumerate(expected_port_stats(ro, P)):
        assert ps[q]["rx_packets"] == rx and ps[q]["tx_packets"] == tx and ps[q]["nf_dropped"] == rx - tx
    # the per-port lists partition the plain forward list
    assert sum(int(c) for c in cnt.ravel()) == len(fo)


def test_demux_ring_wrapping(gpu_ctx_factory):
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F | L, flags=cg.CFG_DEMUX_PORTS, n_streams=2)
    routes = cg.gen_rules(0x5EED2003, 20000, cg.GEN_ROUTES, 0)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    ctx.set_route_lpm(cg.LpmTable(routes, 1 << 20, 1 << 16, False))
    B, NS, P = 65536, 6, 5
    pk = cg.gen_trace(0x5EED0D77, B * NS, rules, routes)
    fwo, rto = oracle_tables(rules, routes)
    dp = ctx.alloc(pk.nbytes)
    dp.upload(pk)
    dr = ctx.alloc(B * NS * 8)
    df = ctx.alloc(B * NS * P * 4)
    dc = ctx.alloc(NS * P * 4)
    rg = cg.make_ring(dp, NS, B, dr, B * 64, fwd_idx=df, fwd_count=dc, fwd_slot=B * P)
    ctx.submit_ring(rg, 4, 9)     # slots 4,5,0,1,...,0: wraps, later slots overwrite
    ctx.sync()
    res = dr.download(cg.RESULT_DT, B * NS)
    cnt = dc.download(np.uint32, NS * P).reshape(NS, P)
    fwd_all = df.download(np.uint32, B * NS * P)
    for s in range(NS):
        ro, _, _ = orc.process(pk[s * B * 64:(s + 1) * B * 64], B, stages=S | F | L, fw=fwo, route=rto)
        assert np.array_equal(res[s * B:(s + 1) * B].view(np.uint8), ro.view(np.uint8)), s
        want = expected_lists(ro, P)
        for q in range(P):
            got = fwd_all[s * B * P + q * B: s * B * P + q * B + cnt[s, q]]
            assert np.array_equal(got, want[q]), (s, q)


def test_demux_ring_slot_too_small(gpu_ctx_factory):
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_DEMUX_PORTS)
    d = ctx.alloc(1 << 20)
    rg = cg.make_ring(d, 2, 1024, d, 1024 * 64, fwd_idx=d, fwd_count=d, fwd_slot=1024)
    with pytest.raises(cg.CopError):
        ctx.submit_ring(rg, 0, 1)


def test_demux_needs_at_most_8_ports(gpu_ctx_factory):
    with pytest.raises(cg.CopError):
        gpu_ctx_factory(stages=S | F, flags=cg.CFG_DEMUX_PORTS, n_ports=9)


def test_live_snapshot_read_and_zero_loses_nothing(gpu_ctx_factory):
    """Snapshots with reset taken while launches run: their sum plus a final
    snapshot equals the exact totals."""
    rules = fw1k()
    ctx = gpu_ctx_factory(stages=S | F, flags=cg.CFG_PORT_STATS, n_streams=2)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    B, NS = 65536, 16
    pk = cg.gen_trace(0x5EED0E00, B * NS, rules)
    fwo, _ = oracle_tables(rules)
    ro, _, co = orc.process(pk, B * NS, stages=S | F, fw=fwo)
    dp = ctx.alloc(pk.nbytes)
    dp.upload(pk)
    dr = ctx.alloc(B * NS * 8)
    df = ctx.alloc(B * NS * 4)
    dc = ctx.alloc(NS * 4)
    rg = cg.make_ring(dp, NS, B, dr, B * 64, fwd_idx=df, fwd_count=dc)
    ctx.snapshot(reset=True, ports=5)
    reps = 40
    tot = {k: 0 for k in cg.COUNTER_NAMES}
    ptot = np.zeros((5, 2), np.int64)
    taken = 0
    for r in range(reps):
        ctx.submit_ring(rg, 0, NS)
        c, ps = ctx.snapshot(reset=True, ports=5)    # concurrent with the launches
        taken += 1
        for k in tot:
            tot[k] += c[k]
        ptot += np.array([[p["rx_packets"], p["tx_packets"]] for p in ps])
    ctx.sync()
    c, ps = ctx.snapshot(reset=True, ports=5)
    for k in tot:
        tot[k] += c[k]
    ptot += np.array([[p["rx_packets"], p["tx_packets"]] for p in ps])
    for k in co:
        assert tot[k] == reps * co[k], (k, tot[k], reps * co[k])
    want = np.array(expected_port_stats(ro, 5)) * reps
    assert np.array_equal(ptot, want)
    # and nothing is left behind
    c, _ = ctx.snapshot(reset=False)
    assert c["rx"] == 0
