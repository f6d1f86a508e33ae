"""GPU parity: the HIP pipeline (through the C ABI) against the oracle.

Bit-exact on every field of every per-packet record (verdict, flags, port,
route next hop) and on the ordered forward list, on seeded synthetic traces
(SURVEY.md §8d generator). At BASELINE sizes (64k/256k batches) the same
comparison runs in full — the oracle is C and finishes in well under a
second — plus size-independent properties of the forward list.
"""
import numpy as np
import pytest

import copgpu as cg
import oracle as orc
from helpers import assert_parity, gpu_run, oracle_tables

pytestmark = pytest.mark.gpu

S = cg.STAGE_PARSE
F = cg.STAGE_FW
L = cg.STAGE_LPM


def fw1k(seed=0x5EED1002):
    return cg.gen_rules(seed, 1000, cg.GEN_FW, 20)


def routes100k(seed=0x5EED2003, n=100000):
    return cg.gen_rules(seed, n, cg.GEN_ROUTES, 0)


def setup_ctx(factory, fw_rules=None, routes=None, stages=S | F, flags=0, fw_cfg=(1024, 24, True),
              rt_cfg=(1 << 20, 1 << 16, False), **kw):
    ctx = factory(stages=stages, flags=flags, **kw)
    if fw_rules is not None:
        ctx.set_fw_table(cg.LpmTable(fw_rules, *fw_cfg))
    if routes is not None:
        ctx.set_route_lpm(cg.LpmTable(routes, *rt_cfg))
    return ctx


@pytest.mark.parametrize("n", [1, 63, 64, 255, 256, 257, 1000, 4096, 65536])
def test_fw_ivt_sizes(gpu_ctx_factory, n):
    rules = fw1k()
    ctx = setup_ctx(gpu_ctx_factory, rules)
    pk = cg.gen_trace(0x5EED0002 + n, n, rules)
    fwo, rto = oracle_tables(rules)
    ro, fo, co = orc.process(pk, n, stages=S | F, fw=fwo)
    ctx.counters(reset=True)
    rg, fg, _ = gpu_run(ctx, pk, n)
    assert_parity(rg, fg, ro, fo)
    cgc = ctx.counters()
    for k in co:
        assert cgc[k] == co[k], (k, cgc[k], co[k])


def test_fw_dir24_forced(gpu_ctx_factory):
    rules = fw1k()
    ctx = setup_ctx(gpu_ctx_factory, rules, flags=cg.CFG_FW_FORCE_DIR24)
    n = 65536
    pk = cg.gen_trace(0x5EED0002, n, rules)
    fwo, _ = oracle_tables(rules)
    ro, fo, _ = orc.process(pk, n, stages=S | F, fw=fwo)
    rg, fg, _ = gpu_run(ctx, pk, n)
    assert_parity(rg, fg, ro, fo)


# the 100k route table: DIR-24-8, the multibit trie or the bucketed intervals
FORMS = {"dir": 0, "trie": cg.CFG_LPM_TRIE, "bkt": cg.CFG_LPM_BKT}


@pytest.mark.parametrize("form", list(FORMS))
def test_fw_lpm_100k(gpu_ctx_factory, form):
    rules = fw1k()
    routes = routes100k()
    ctx = setup_ctx(gpu_ctx_factory, rules, routes, stages=S | F | L, flags=FORMS[form])
    assert ctx.route_form() == form
    n = 65536
    pk = cg.gen_trace(0x5EED0003, n, rules, routes)
    fwo, rto = oracle_tables(rules, routes)
    ro, fo, _ = orc.process(pk, n, stages=S | F | L, fw=fwo, route=rto)
    rg, fg, _ = gpu_run(ctx, pk, n)
    assert_parity(rg, fg, ro, fo)
    assert (rg["flags"] & cg.FLAG_ROUTE_HIT).sum() > n // 10   # the route stage really hits


@pytest.mark.parametrize("form", list(FORMS))
def test_imix_fw_lpm(gpu_ctx_factory, form):
    rules = fw1k()
    routes = routes100k()
    ctx = setup_ctx(gpu_ctx_factory, rules, routes, stages=S | F | L, flags=FORMS[form])
    n = 65536
    slab, offs = cg.gen_imix(0x5EED0003, n, rules, routes)
    fwo, rto = oracle_tables(rules, routes)
    ro, fo, _ = orc.process(slab, n, offsets=offs, stages=S | F | L, fw=fwo, route=rto)
    rg, fg, _ = gpu_run(ctx, slab, n, offsets=offs)
    assert_parity(rg, fg, ro, fo)


@pytest.mark.parametrize("nb", [2, 7, 32])
def test_multi_batch_submit(gpu_ctx_factory, nb):
    rules = fw1k()
    ctx = setup_ctx(gpu_ctx_factory, rules)
    n = 65536 + 333
    pk = cg.gen_trace(0x5EED0042, n, rules)
    fwo, _ = oracle_tables(rules)
    ro, fo, _ = orc.process(pk, n, stages=S | F, fw=fwo)
    rg, fg, _ = gpu_run(ctx, pk, n, batches=nb)
    assert_parity(rg, fg, ro, fo)


def test_big_batch_256k_properties(gpu_ctx_factory):
    rules = fw1k()
    routes = routes100k()
    ctx = setup_ctx(gpu_ctx_factory, rules, routes, stages=S | F | L)
    n = 262144
    pk = cg.gen_trace(0x5EED0005, n, rules, routes)
    rg, fg, counts = gpu_run(ctx, pk, n)
    fwd_mask = rg["verdict"] == cg.FORWARD
    assert counts[0] == fwd_mask.sum()
    assert np.all(np.diff(fg.astype(np.int64)) > 0)          # strictly increasing = arrival order
    assert np.array_equal(fg, np.nonzero(fwd_mask)[0])        # exactly the FORWARD packets
    fwo, rto = oracle_tables(rules, routes)
    ro, fo, _ = orc.process(pk, n, stages=S | F | L, fw=fwo, route=rto)
    assert_parity(rg, fg, ro, fo)


def test_edge_versions_and_ports(gpu_ctx_factory):
    """version != 4 (reference UB, defined DROP_NOT_IPV4), non-IPv4
    EtherType, unknown dst, custom routing table with ports >= n_ports."""
    rules = fw1k()
    rt = cg.route_table_default(5)
    rt[0x1234] = 7           # port beyond nb_active_kni -> DROP_NO_PORT
    rt[0x2000:0x2100] = 3    # a uniform leaf block
    ctx = setup_ctx(gpu_ctx_factory, rules, routing_table=rt)
    n = 20000
    opts = cg.trace_opts(pct_bad_version=10, pct_non_ipv4=10, pct_unknown_dst=10)
    pk = cg.gen_trace(0x5EED0077, n, rules, opts=opts)
    # force some dsts onto the custom entries
    for i in range(0, n, 97):
        pk[i * 64 + 32] = 0x12
        pk[i * 64 + 33] = 0x34
    fwo, _ = oracle_tables(rules)
    ro, fo, _ = orc.process(pk, n, rt=rt, stages=S | F, fw=fwo)
    rg, fg, _ = gpu_run(ctx, pk, n)
    assert_parity(rg, fg, ro, fo)
    v = rg["verdict"]
    for verdict in (cg.FORWARD, cg.DROP_FW, cg.DROP_PARSE, cg.DROP_NOT_IPV4, cg.DROP_NO_PORT):
        assert (v == verdict).sum() > 0, verdict


def test_dense_routing_table_lds_fallback(gpu_ctx_factory):
    """A random routing table with every /8 block non-uniform (256 leaves,
    128 KiB of LDS) beside the firewall's and a route table's interval
    images: too much for LDS, so the launch looks the interval tables up in
    their DIR-24-8 images instead. Results identical."""
    rules = fw1k()
    routes = routes100k(n=3000)
    rng = np.random.default_rng(11)
    rt = rng.integers(0, 6, 65536).astype(np.uint16)
    rt[rng.random(65536) < 0.05] = 0xFFFF
    ctx = setup_ctx(gpu_ctx_factory, rules, routes, stages=S | F | L, routing_table=rt)
    n = 50000
    pk = cg.gen_trace(0x5EED0078, n, rules, routes)
    fwo, rto = oracle_tables(rules, routes)
    ro, fo, _ = orc.process(pk, n, rt=rt, stages=S | F | L, fw=fwo, route=rto)
    rg, fg, _ = gpu_run(ctx, pk, n)
    assert_parity(rg, fg, ro, fo)
    assert (rg["verdict"] == cg.DROP_NO_PORT).sum() > 0 and (rg["verdict"] == cg.DROP_PARSE).sum() > 0


@pytest.mark.parametrize("stages", [S, S | F, S | L, F, F | L, S | F | L])
def test_stage_masks(gpu_ctx_factory, stages):
    rules = fw1k()
    routes = routes100k(n=20000)
    ctx = setup_ctx(gpu_ctx_factory, rules, routes, stages=stages)
    n = 30000
    pk = cg.gen_trace(0x5EED0100 + stages, n, rules, routes)
    fwo, rto = oracle_tables(rules, routes)
    ro, fo, _ = orc.process(pk, n, stages=stages, fw=fwo, route=rto)
    rg, fg, _ = gpu_run(ctx, pk, n)
    assert_parity(rg, fg, ro, fo)


def test_reference_rules_json_all_forward(gpu_ctx_factory, tmp_path):
    """The reference's only fixture (engine/nfs/firewall/rules.json, copied
    as data under tests/golden/): both rules accept, so every IPv4 packet
    that reaches the coprocessor is forwarded."""
    import os
    path = os.path.join(os.path.dirname(__file__), "golden", "reference_rules.json")
    ctx = gpu_ctx_factory(stages=S | F)
    rep = ctx.load_fw_rules_file(path)
    assert rep.n_added == 2 and rep.n_failed == 0
    n = 50000
    pk = cg.gen_trace(0x5EED0001, n)
    rg, fg, _ = gpu_run(ctx, pk, n)
    reached = (rg["verdict"] != cg.DROP_PARSE) & (rg["verdict"] != cg.DROP_NO_PORT)
    assert np.all(rg["verdict"][reached] == cg.FORWARD)


def test_empty_batch_and_tiny(gpu_ctx_factory):
    rules = fw1k()
    ctx = setup_ctx(gpu_ctx_factory, rules)
    d = ctx.alloc(64)
    r = ctx.alloc(64)
    c = ctx.alloc(16)
    f = ctx.alloc(64)
    c.fill(0xFF)
    ctx.submit([cg.make_batch(d, 0, r, fwd_idx=f, fwd_count=c)])
    ctx.sync()
    assert c.download(np.uint32, 1)[0] == 0


def test_process_host_end_to_end(gpu_ctx_factory):
    rules = fw1k()
    routes = routes100k(n=20000)
    ctx = setup_ctx(gpu_ctx_factory, rules, routes, stages=S | F | L)
    n = 10000
    pk = cg.gen_trace(0x5EED0200, n, rules, routes)
    fwo, rto = oracle_tables(rules, routes)
    ro, fo, _ = orc.process(pk, n, stages=S | F | L, fw=fwo, route=rto)
    rg, fg = ctx.process_host(pk, n)
    assert_parity(rg, fg, ro, fo)


def test_tbl8_exhaustion_stop_at_first_error(gpu_ctx_factory):
    """lpm_setup truncates at the first failed rte_lpm_add: with 30 distinct
    /24 parents of /25+ rules and number_tbl8s=24 the 25th fails."""
    ip, depth, nh = [], [], []
    for k in range(30):
        ip.append((10 << 24) | (k << 8) | 0x80)
        depth.append(25)
        nh.append(1 + k)
    ip.append(0x0B000000)
    depth.append(8)
    nh.append(9)
    rules = cg.prefixes(ip, depth, nh)
    t = cg.LpmTable(rules, 1024, 24, True)
    assert t.report.n_failed == 1 and t.report.first_error_idx == 24 and t.report.n_skipped == 6
    ctx = setup_ctx(gpu_ctx_factory, rules)
    n = 4096
    pk = cg.gen_trace(0x5EED0300, n, rules)
    fwo, _ = oracle_tables(rules)
    ro, fo, _ = orc.process(pk, n, stages=S | F, fw=fwo)
    rg, fg, _ = gpu_run(ctx, pk, n)
    assert_parity(rg, fg, ro, fo)


def test_repeated_submits_epochs(gpu_ctx_factory):
    """Many launches on one context: ticket base and look-back epochs carry
    across launches without a reset."""
    rules = fw1k()
    ctx = setup_ctx(gpu_ctx_factory, rules)
    n = 8192
    pk = cg.gen_trace(0x5EED0400, n, rules)
    fwo, _ = oracle_tables(rules)
    ro, fo, _ = orc.process(pk, n, stages=S | F, fw=fwo)
    for _ in range(50):
        rg, fg, _ = gpu_run(ctx, pk, n, batches=3)
    assert_parity(rg, fg, ro, fo)


@pytest.mark.parametrize("lanes,threads", [(1, 1), (2, 1), (4, 1), (2, 8), (4, 3)])
def test_process_host_stream_lanes(gpu_ctx_factory, lanes, threads):
    """Streaming end-to-end host path over mbuf-like scattered buffers, with
    the header gather on 1..8 host threads."""
    rules = fw1k()
    ctx = setup_ctx(gpu_ctx_factory, rules, n_streams=lanes)
    ctx.set_host_threads(threads)
    n = 50000
    pk = cg.gen_trace(0x5EED0700, n, rules)
    stride = 2176
    pool = np.zeros(n * stride, dtype=np.uint8)
    pool.reshape(n, stride)[:, 128:192] = pk.reshape(n, 64)
    ptrs = (pool.ctypes.data + 128 + np.arange(n, dtype=np.uint64) * stride).astype(np.uint64)
    fwo, _ = oracle_tables(rules)
    ro, _, _ = orc.process(pk, n, stages=S | F, fw=fwo)
    res = ctx.process_host_stream(ptrs, 8192)
    assert np.array_equal(res.view(np.uint8), ro.view(np.uint8))


@pytest.mark.parametrize("lanes,threads,zc,rec", [(2, 16, 0, 16), (4, 5, 0, 12), (2, 16, 1, 12), (3, 1, 1, 16),
                                                   (4, 16, 2, 12), (1, 3, 2, 12), (4, 16, 2, 16), (2, 1, 2, 12)])
def test_process_host_stream_large_batches(gpu_ctx_factory, monkeypatch, lanes, threads, zc, rec):
    """The end-to-end path as bench.py's e2e leg runs it: 256k-packet
    batches, the records of each lane's previous batch copied out by the host
    threads in the same job as the next gather (GatherPool::run), a ragged
    last batch; 3 x 262144 + 77 packets, each of a 50k-packet mbuf pool
    visited many times, against the oracle. zc: staging and records in
    mapped pinned memory, read and written by the kernel over PCIe
    ($COP_STREAM_ZC 1), records only (2, the default) or neither (0); rec:
    12-byte (the default) or 16-byte header records ($COP_STREAM_REC)."""
    monkeypatch.setenv("COP_STREAM_ZC", str(zc))
    monkeypatch.setenv("COP_STREAM_REC", str(rec))
    rules = fw1k()
    ctx = setup_ctx(gpu_ctx_factory, rules, n_streams=lanes, max_batch=262144)
    ctx.set_host_threads(threads)
    nb = 50000
    pk = cg.gen_trace(0x5EED0710, nb, rules)
    stride = 2176
    pool = np.zeros(nb * stride, dtype=np.uint8)
    pool.reshape(nb, stride)[:, 128:192] = pk.reshape(nb, 64)
    n = 3 * 262144 + 77
    sel = np.random.default_rng(5).integers(0, nb, n)
    ptrs = (pool.ctypes.data + 128 + sel.astype(np.uint64) * stride).astype(np.uint64)
    fwo, _ = oracle_tables(rules)
    ro, _, _ = orc.process(pk, nb, stages=S | F, fw=fwo)
    out = np.full(n, 0xEE, np.uint64).view(cg.RESULT_DT)
    for _ in range(2):     # the second pass reuses the lanes' staging
        res = ctx.process_host_stream(ptrs, 262144, out=out)
        assert np.array_equal(res.view(np.uint8), ro[sel].view(np.uint8))


@pytest.mark.parametrize("lanes", [1, 4])
def test_concurrent_lanes_many_submits(gpu_ctx_factory, lanes):
    """Back-to-back submits spread over lanes (kernels may overlap): every
    batch still gets exactly its own results and ordered forward list."""
    rules = fw1k()
    ctx = setup_ctx(gpu_ctx_factory, rules, n_streams=lanes)
    B, P = 65536, 12
    pk = cg.gen_trace(0x5EED0800, B * P, rules)
    dp = ctx.alloc(pk.nbytes)
    dp.upload(pk)
    dr = ctx.alloc(B * P * 8)
    df = ctx.alloc(B * P * 4)
    dc = ctx.alloc(P * 4)
    for rep in range(3):
        for i in range(0, P, 3):
            ctx.submit([cg.make_batch(dp.addr + (i + j) * B * 64, B, dr.addr + (i + j) * B * 8,
                                      fwd_idx=df.addr + (i + j) * B * 4, fwd_count=dc.addr + (i + j) * 4)
                        for j in range(3)])
    ctx.sync()
    res = dr.download(cg.RESULT_DT, B * P)
    cnt = dc.download(np.uint32, P)
    fwd = df.download(np.uint32, B * P)
    fwo, _ = oracle_tables(rules)
    ro, fo, _ = orc.process(pk, B * P, stages=S | F, fw=fwo)
    assert np.array_equal(res.view(np.uint8), ro.view(np.uint8))
    got = np.concatenate([fwd[i * B: i * B + cnt[i]] + i * B for i in range(P)])
    assert np.array_equal(got, fo)


@pytest.mark.parametrize("lanes", [1, 2])
def test_ring_submit_wrapping(gpu_ctx_factory, lanes):
    """cop_submit_ring: slots at constant strides, launches that wrap the
    ring, with ragged n (not a tile multiple); per-slot parity."""
    rules = fw1k()
    routes = routes100k(n=20000)
    ctx = setup_ctx(gpu_ctx_factory, rules, routes, stages=S | F | L, n_streams=lanes)
    n, P = 20000 + 77, 9
    slot_bytes = ((n * 64 + 4095) // 4096) * 4096
    pk = cg.gen_trace(0x5EED0900, n * P, rules, routes)
    dp = ctx.alloc(slot_bytes * P)
    for s in range(P):
        dp.upload(pk[s * n * 64:(s + 1) * n * 64], s * slot_bytes)
    res_slot = n + 13
    dr = ctx.alloc(res_slot * P * 8)
    df = ctx.alloc(res_slot * P * 4)
    dc = ctx.alloc(P * 4)
    ring = cg.make_ring(dp, P, n, dr, slot_bytes, results_slot=res_slot, fwd_idx=df, fwd_slot=res_slot,
                        fwd_count=dc)
    ctx.submit_ring(ring, 5, 7)      # slots 5..8, 0..2
    ctx.submit_ring(ring, 3, 2)      # slots 3, 4
    ctx.sync()
    fwo, rto = oracle_tables(rules, routes)
    res_all = dr.download(cg.RESULT_DT, res_slot * P)
    fwd_all = df.download(np.uint32, res_slot * P)
    cnt = dc.download(np.uint32, P)
    for s in range(P):
        ro, fo, _ = orc.process(pk[s * n * 64:(s + 1) * n * 64], n, stages=S | F | L, fw=fwo, route=rto)
        rg = res_all[s * res_slot: s * res_slot + n]
        fg = fwd_all[s * res_slot: s * res_slot + cnt[s]]
        assert_parity(rg, fg, ro, fo)


def test_ring_large_launch_many_batches(gpu_ctx_factory):
    """One launch over 128 ring slots (more than the 32 kernel-argument
    descriptors): tickets and look-back of every batch stay separate."""
    rules = fw1k()
    ctx = setup_ctx(gpu_ctx_factory, rules, n_streams=1)
    n, P = 8192, 40
    pk = cg.gen_trace(0x5EED0A00, n * P, rules)
    dp = ctx.alloc(pk.nbytes)
    dp.upload(pk)
    dr = ctx.alloc(n * P * 8)
    df = ctx.alloc(n * P * 4)
    dc = ctx.alloc(P * 4)
    ring = cg.make_ring(dp, P, n, dr, n * 64, fwd_idx=df, fwd_count=dc)
    for rep in range(3):
        ctx.submit_ring(ring, (rep * 7) % P, 128)   # each slot processed 3-4 times per launch
    ctx.sync()
    fwo, _ = oracle_tables(rules)
    ro, fo, _ = orc.process(pk, n * P, stages=S | F, fw=fwo)
    res = dr.download(cg.RESULT_DT, n * P)
    assert np.array_equal(res.view(np.uint8), ro.view(np.uint8))
    cnt = dc.download(np.uint32, P)
    fwd = df.download(np.uint32, n * P)
    got = np.concatenate([fwd[s * n: s * n + cnt[s]] + s * n for s in range(P)])
    assert np.array_equal(got, fo)


@pytest.mark.parametrize("stride,data_off,n", [(2176, 128, 50000), (48, 0, 70000), (64, 16, 65536),
                                               (128, 64, 262144)])
def test_strides_and_data_off(gpu_ctx_factory, stride, data_off, n):
    """Device-resident mbuf-like layouts: packet i at pkts + i*stride +
    data_off (rte_pktmbuf_mtod), through cop_submit."""
    rules = fw1k()
    routes = routes100k(n=20000)
    ctx = setup_ctx(gpu_ctx_factory, rules, routes, stages=S | F | L)
    pk = cg.gen_trace(0x5EED0900 + stride, n, rules, routes)
    slots = np.zeros((n, stride), dtype=np.uint8)
    slots[:, data_off:data_off + min(64, stride - data_off)] = pk.reshape(n, 64)[:, :min(64, stride - data_off)]
    fwo, rto = oracle_tables(rules, routes)
    ro, fo, _ = orc.process(slots.reshape(-1)[data_off:], n, stride=stride, stages=S | F | L, fw=fwo, route=rto)
    dp = ctx.alloc(slots.nbytes)
    dp.upload(slots.reshape(-1))
    dr = ctx.alloc(n * 8)
    df = ctx.alloc(n * 4)
    dc = ctx.alloc(16)
    ctx.submit([cg.make_batch(dp, n, dr, stride=stride, data_off=data_off, fwd_idx=df, fwd_count=dc)])
    ctx.sync()
    res = dr.download(cg.RESULT_DT, n)
    cnt = int(dc.download(np.uint32, 1)[0])
    assert_parity(res, df.download(np.uint32, cnt), ro, fo)


def test_imix_with_data_off(gpu_ctx_factory):
    rules = fw1k()
    routes = routes100k(n=20000)
    ctx = setup_ctx(gpu_ctx_factory, rules, routes, stages=S | F | L)
    n = 30000
    slab, offs = cg.gen_imix(0x5EED0A00, n, rules, routes)
    # shift every packet 16 bytes further into its buffer: offsets stay, data_off = 16
    slab2 = np.zeros(slab.nbytes + 64, dtype=np.uint8)
    for i in range(0, n):
        o = int(offs[i])
        slab2[o + 16:o + 16 + 64] = slab[o:o + 64]
    fwo, rto = oracle_tables(rules, routes)
    ro, fo, _ = orc.process(slab, n, offsets=offs, stages=S | F | L, fw=fwo, route=rto)
    dp = ctx.alloc(slab2.nbytes)
    dp.upload(slab2)
    do = ctx.alloc(offs.nbytes)
    do.upload(offs)
    dr = ctx.alloc(n * 8)
    df = ctx.alloc(n * 4)
    dc = ctx.alloc(16)
    ctx.submit([cg.make_batch(dp, n, dr, offsets=do, data_off=16, fwd_idx=df, fwd_count=dc)])
    ctx.sync()
    cnt = int(dc.download(np.uint32, 1)[0])
    assert_parity(dr.download(cg.RESULT_DT, n), df.download(np.uint32, cnt), ro, fo)


def test_misaligned_batches_rejected(gpu_ctx_factory):
    ctx = gpu_ctx_factory(stages=S | F)
    d = ctx.alloc(1 << 20)
    for kw in (dict(stride=40), dict(stride=32), dict(data_off=8), dict(pkts_offset=4)):
        with pytest.raises(cg.CopError):
            ctx.submit([cg.make_batch(d, 1000, d, **kw)])
    r = ctx.alloc(1 << 16)
    with pytest.raises(cg.CopError):     # results must be 8-byte aligned
        ctx.submit([cg.make_batch(d, 10, r.addr + 4)])


@pytest.mark.parametrize("ppt", ["1", "4", "8"])
def test_every_tile_width_same_records(gpu_ctx_factory, monkeypatch, ppt):
    """The three kernel instantiations (PPT 1/4/8 packets per lane) on the
    same 3 batches give the same, oracle-exact records and lists."""
    monkeypatch.setenv("COP_PPT", ppt)
    rules = fw1k()
    routes = routes100k(n=20000)
    ctx = setup_ctx(gpu_ctx_factory, rules, routes, stages=S | F | L)
    n = 150001
    pk = cg.gen_trace(0x5EED0B00, n, rules, routes)
    fwo, rto = oracle_tables(rules, routes)
    ro, fo, _ = orc.process(pk, n, stages=S | F | L, fw=fwo, route=rto)
    rg, fg, _ = gpu_run(ctx, pk, n, batches=3)
    assert_parity(rg, fg, ro, fo)


@pytest.mark.parametrize("stages", [S | F, F, S | F | L])
def test_hdr12_records_match_frames(gpu_ctx_factory, stages):
    """12-byte header records (COP_HDR12_STRIDE: frame bytes 12..15 then
    26..33, what cop_process_host_stream sends by default) give the frames'
    exact records and forward lists: odd batch sizes in one submit, packets
    with bad versions, non-IPv4 EtherTypes and unknown destinations, the
    route stage on."""
    rules = fw1k()
    routes = routes100k(n=20000)
    ctx = setup_ctx(gpu_ctx_factory, rules, routes, stages=stages)
    n = 70001
    opts = cg.trace_opts(pct_bad_version=7, pct_non_ipv4=7, pct_unknown_dst=7)
    pk = cg.gen_trace(0x5EED0903, n, rules, routes, opts=opts)
    base = pk.ctypes.data
    rec = cg.pack_headers12((base + np.arange(n, dtype=np.uint64) * 64).astype(np.uint64))
    f = pk.reshape(n, 64)
    assert np.array_equal(rec.reshape(n, 12), np.concatenate([f[:, 12:16], f[:, 26:34]], axis=1))
    fwo, rto = oracle_tables(rules, routes)
    ro, fo, _ = orc.process(pk, n, stages=stages, fw=fwo, route=rto)
    rg, fg, _ = gpu_run(ctx, rec, n, stride=cg.HDR12_STRIDE, batches=3)
    assert_parity(rg, fg, ro, fo)
