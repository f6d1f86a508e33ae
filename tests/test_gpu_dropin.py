"""Drop-in coprocessor API on the GPU: coprocessor_setup / process_packet /
process_burst (coprocessor.c:21-65) with rte_mbuf-shaped descriptors, and
cop_coprocessor_poll, the GPU form of one coprocessor() call
(switch.c:443-474), over rte_ring-semantics rings.

The drop-in runs the coprocessor's NF chain only (COP_DROPIN_STAGES = FW:
process_packet -> fw_packet_handler, coprocessor.c:59-62); get_next_hop's
drop of UNKNOWN destinations and non-IPv4 EtherTypes is the fast path's
(switch.c:406-415). The traces hold both kinds of packet (5 % dst&0xFFFF in
0..4, 2 % EtherType 0x86DD), so the oracle they are checked against is the
FW-only chain, and the tests assert that it differs from the P+FW batch
pipeline on them."""
import ctypes
import os

import numpy as np
import pytest

import copgpu as cg
import oracle as orc
from helpers import oracle_tables

pytestmark = pytest.mark.gpu

HEADROOM = 128
STRIDE = 2176   # MBUF_DATA_SZ, init.h:38-41
DROPIN = cg.STAGE_FW   # COP_DROPIN_STAGES


class Mbufs:
    """n fake rte_mbufs: 64-byte descriptors {buf_addr @0, data_off @16} and
    2176-byte data buffers with the packet at buf_addr + 128."""

    def __init__(self, pkts64, n):
        self.data = np.zeros(n * STRIDE, dtype=np.uint8)
        self.desc = np.zeros(n * 64, dtype=np.uint8)
        base = self.data.ctypes.data
        for i in range(n):
            self.data[i * STRIDE + HEADROOM: i * STRIDE + HEADROOM + 64] = pkts64[i * 64:(i + 1) * 64]
            self.desc[i * 64: i * 64 + 8] = np.frombuffer(np.uint64(base + i * STRIDE).tobytes(), np.uint8)
            self.desc[i * 64 + 16: i * 64 + 18] = np.frombuffer(np.uint16(HEADROOM).tobytes(), np.uint8)
        self.n = n

    def ptr(self, i):
        return self.desc.ctypes.data + i * 64

    def index(self, p):
        return (p - self.desc.ctypes.data) // 64


@pytest.fixture
def rules_file(tmp_path):
    rules = cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)
    f = tmp_path / "rules.json"
    cg.rules_write_json(str(f), rules)
    return str(f), rules


def test_setup_process_packet_and_burst(rules_file):
    path, rules = rules_file
    L = cg.lib()
    L.cop_set_mbuf_layout(0, 16)
    L.cop_set_rule_file(path.encode())
    assert L.coprocessor_setup() == 0
    try:
        n = 3000
        pk = cg.gen_trace(0x5EED0500, n, rules)
        mb = Mbufs(pk, n)
        fwo, _ = oracle_tables(rules)
        ro, _, _ = orc.process(pk, n, stages=DROPIN, fw=fwo)
        want = np.where(ro["verdict"] == 0, 0, -1)
        rp, _, _ = orc.process(pk, n, stages=cg.STAGE_PARSE | cg.STAGE_FW, fw=fwo)
        # packets get_next_hop would drop but the firewall forwards
        assert np.sum((rp["verdict"] == cg.DROP_PARSE) & (ro["verdict"] == 0)) > 0
        for i in range(0, n, 97):
            assert L.process_packet(ctypes.c_void_p(mb.ptr(i))) == want[i], i
        ptrs = (ctypes.c_void_p * n)(*[mb.ptr(i) for i in range(n)])
        ret = np.zeros(n, dtype=np.int32)
        assert L.process_burst(ptrs, n, ret.ctypes.data) == 0
        assert np.array_equal(ret, want)
    finally:
        assert L.coprocessor_teardown() == 0


def test_coprocessor_poll_rings(rules_file):
    path, rules = rules_file
    L = cg.lib()
    L.cop_set_mbuf_layout(0, 16)
    L.cop_set_rule_file(path.encode())
    assert L.coprocessor_setup() == 0
    try:
        ctx = L.coprocessor_ctx()
        assert ctx
        n = 5000
        pk = cg.gen_trace(0x5EED0600, n, rules)
        mb = Mbufs(pk, n)
        fwo, _ = oracle_tables(rules)
        ro, fo, _ = orc.process(pk, n, stages=DROPIN, fw=fwo)
        rx = L.cop_ring_create(16384)
        tx = L.cop_ring_create(16384)
        freed = []
        FREE = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p)
        cb = FREE(lambda m, arg: freed.append(mb.index(m)))
        # fast path side: bulk-enqueue bursts of 32 (flush_nf_rx_queue)
        for i in range(0, n, 32):
            k = min(32, n - i)
            arr = (ctypes.c_void_p * k)(*[mb.ptr(j) for j in range(i, i + k)])
            assert L.cop_ring_enqueue_bulk(rx, arr, k, None) == k
        stats = cg.NfStats()
        done = 0
        while done < n:
            r = L.cop_coprocessor_poll(ctx, rx, tx, 2048, cb, None, ctypes.byref(stats))
            assert r > 0
            done += r
        out = []
        buf = (ctypes.c_void_p * 64)()
        while True:
            k = L.cop_ring_dequeue_burst(tx, buf, 64, None)
            if not k:
                break
            out += [mb.index(buf[i]) for i in range(k)]
        assert out == list(fo)                       # forwarded, in arrival order
        assert sorted(freed) == sorted(set(range(n)) - set(fo))
        assert stats.tx_packets == len(fo) and stats.tx_dropped == 0
        L.cop_ring_free(rx)
        L.cop_ring_free(tx)
    finally:
        L.coprocessor_teardown()


@pytest.mark.parametrize("max_pkts", [512, 2048, 16384])
def test_coprocessor_poll_async_rings(rules_file, max_pkts):
    """The pipelined ring loop (cop_coprocessor_poll_async): a fast path that
    keeps enqueueing between calls, batches in flight across calls, then
    cop_coprocessor_flush. Same tx_q content and order as the oracle's
    forward list, every drop freed exactly once."""
    path, rules = rules_file
    L = cg.lib()
    L.cop_set_mbuf_layout(0, 16)
    L.cop_set_rule_file(path.encode())
    assert L.coprocessor_setup() == 0
    try:
        ctx = L.coprocessor_ctx()
        n = 40000
        pk = cg.gen_trace(0x5EED0610, n, rules)
        mb = Mbufs(pk, n)
        fwo, _ = oracle_tables(rules)
        _, fo, _ = orc.process(pk, n, stages=DROPIN, fw=fwo)
        rx = L.cop_ring_create(16384)
        tx = L.cop_ring_create(65536)
        freed = []
        FREE = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p)
        cb = FREE(lambda m, arg: freed.append(mb.index(m)))
        stats = cg.NfStats()
        sent = done = 0
        out = []
        buf = (ctypes.c_void_p * 256)()
        polls = 0
        while done < n:
            # the fast path enqueues up to 3000 packets between two polls
            k_end = min(n, sent + 3000)
            while sent < k_end:
                k = min(32, k_end - sent)
                arr = (ctypes.c_void_p * k)(*[mb.ptr(j) for j in range(sent, sent + k)])
                if L.cop_ring_enqueue_bulk(rx, arr, k, None) != k:
                    break
                sent += k
            r = L.cop_coprocessor_poll_async(ctx, rx, tx, max_pkts, cb, None, ctypes.byref(stats))
            assert r >= 0
            done += r
            polls += 1
            assert polls < 10000
            while True:
                k = L.cop_ring_dequeue_burst(tx, buf, 256, None)
                if not k:
                    break
                out += [mb.index(buf[i]) for i in range(k)]
        assert L.cop_coprocessor_flush(ctx, tx, cb, None, ctypes.byref(stats)) == 0
        while True:
            k = L.cop_ring_dequeue_burst(tx, buf, 256, None)
            if not k:
                break
            out += [mb.index(buf[i]) for i in range(k)]
        assert out == list(fo)
        assert sorted(freed) == sorted(set(range(n)) - set(fo))
        assert stats.tx_packets == len(fo) and stats.tx_dropped == 0
        L.cop_ring_free(rx)
        L.cop_ring_free(tx)
    finally:
        L.coprocessor_teardown()


def unrouted_packet(src_ip, dst_low16, ethertype=0x0800):
    """One 64 B UDP/IPv4 frame whose destination get_next_hop would drop
    (routing_table[dst & 0xFFFF] == UNKNOWN_PORT for 0..4, init.c:51-53)."""
    f = np.zeros(64, np.uint8)
    f[12:14] = [ethertype >> 8, ethertype & 0xFF]
    f[14] = 0x45
    f[23] = 17
    f[26:30] = np.frombuffer(np.uint32(src_ip).byteswap().tobytes(), np.uint8)
    f[30:34] = np.frombuffer(np.uint32((0xC0A70000 | dst_low16)).byteswap().tobytes(), np.uint8)
    return f


def test_process_packet_unrouted_ipv4_gets_firewall_verdict(tmp_path):
    """process_packet on IPv4 packets with dst&0xFFFF in {0..4}, and on
    EtherType 0x86DD with an IPv4 header behind it: the reference's
    process_packet returns fw_packet_handler's verdict for them (it never
    looks at the route), so a source inside an action-0 rule forwards (0) and
    one inside a non-zero rule drops (-1)."""
    rules = np.zeros(2, dtype=cg.PREFIX_DT)
    rules["ip"] = [0x0A000000, 0x0B000000]
    rules["depth"] = [8, 8]
    rules["next_hop"] = [0, 7]
    f = tmp_path / "rules.json"
    cg.rules_write_json(str(f), rules)
    L = cg.lib()
    L.cop_set_mbuf_layout(0, 16)
    L.cop_set_rule_file(str(f).encode())
    assert L.coprocessor_setup() == 0
    try:
        frames, want = [], []
        for low in range(5):
            frames.append(unrouted_packet(0x0A010203, low)); want.append(0)
            frames.append(unrouted_packet(0x0B010203, low)); want.append(-1)
            frames.append(unrouted_packet(0x0C010203, low)); want.append(0)      # miss: nh 0 -> FORWARD
        frames.append(unrouted_packet(0x0A010203, 0x0A01, 0x86DD)); want.append(0)
        frames.append(unrouted_packet(0x0B010203, 0x0A01, 0x86DD)); want.append(-1)
        pk = np.concatenate(frames)
        n = len(want)
        mb = Mbufs(pk, n)
        got = [L.process_packet(ctypes.c_void_p(mb.ptr(i))) for i in range(n)]
        assert got == want
        fwo, _ = oracle_tables(rules)
        ro, _, _ = orc.process(pk, n, stages=DROPIN, fw=fwo)
        assert list(np.where(ro["verdict"] == 0, 0, -1)) == want
    finally:
        assert L.coprocessor_teardown() == 0


def _inject(ctx, what, count):
    fn = cg.lib().cop_debug_inject
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32]
    assert fn(ctx, what, count) == 0


@pytest.mark.parametrize("where", ["max_pkts", "submit", "async_submit", "async_wait"])
def test_dropin_error_paths_free_every_mbuf(rules_file, where):
    """A failure after packets left rx_q never strands them: each dequeued
    mbuf is forwarded or freed exactly once (switch.c:464-470 does one or the
    other for every packet). An oversized max_pkts is refused before any
    dequeue. Failures are injected with the library's test hook."""
    path, rules = rules_file
    L = cg.lib()
    L.cop_set_mbuf_layout(0, 16)
    L.cop_set_rule_file(path.encode())
    assert L.coprocessor_setup() == 0
    try:
        ctx = L.coprocessor_ctx()
        n = 4096
        pk = cg.gen_trace(0x5EED0620, n, rules)
        mb = Mbufs(pk, n)
        fwo, _ = oracle_tables(rules)
        _, fo, _ = orc.process(pk, n, stages=DROPIN, fw=fwo)
        rx = L.cop_ring_create(16384)
        tx = L.cop_ring_create(16384)
        freed = []
        FREE = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p)
        cb = FREE(lambda m, arg: freed.append(mb.index(m)))
        arr = (ctypes.c_void_p * n)(*[mb.ptr(j) for j in range(n)])
        assert L.cop_ring_enqueue_bulk(rx, arr, n, None) == n
        stats = cg.NfStats()
        if where == "max_pkts":
            assert L.cop_coprocessor_poll(ctx, rx, tx, 262145, cb, None, ctypes.byref(stats)) < 0
            assert L.cop_coprocessor_poll_async(ctx, rx, tx, 1 << 20, cb, None, ctypes.byref(stats)) < 0
            assert L.cop_ring_count(rx) == n and not freed     # nothing was dequeued
            return
        if where == "submit":
            _inject(ctx, 1, 1)
            assert L.cop_coprocessor_poll(ctx, rx, tx, 1000, cb, None, ctypes.byref(stats)) < 0
            lost = list(range(1000))
        elif where == "async_submit":
            _inject(ctx, 1, 1)
            assert L.cop_coprocessor_poll_async(ctx, rx, tx, 1000, cb, None, ctypes.byref(stats)) < 0
            lost = list(range(1000))
        else:
            assert L.cop_coprocessor_poll_async(ctx, rx, tx, 1000, cb, None, ctypes.byref(stats)) == 0
            _inject(ctx, 2, 1)
            # the second call submits packets 1000..1999, then completes the
            # first batch, whose wait fails: packets 0..999 are freed
            assert L.cop_coprocessor_poll_async(ctx, rx, tx, 1000, cb, None, ctypes.byref(stats)) < 0
            lost = list(range(1000))
        assert sorted(freed) == lost
        assert stats.tx_dropped == len(lost) and stats.tx_packets == 0
        # the loop recovers: the rest flows normally
        del freed[:]
        done = 0
        while True:
            r = L.cop_coprocessor_poll_async(ctx, rx, tx, 1000, cb, None, ctypes.byref(stats))
            assert r >= 0
            done += r
            if r == 0 and L.cop_ring_count(rx) == 0:
                break
        assert L.cop_coprocessor_flush(ctx, tx, cb, None, ctypes.byref(stats)) >= 0
        out = []
        buf = (ctypes.c_void_p * 256)()
        while True:
            k = L.cop_ring_dequeue_burst(tx, buf, 256, None)
            if not k:
                break
            out += [mb.index(buf[i]) for i in range(k)]
        rest = set(range(1000, n))
        assert out == [i for i in fo if i in rest]
        assert sorted(freed) == sorted(rest - set(out))
        L.cop_ring_free(rx)
        L.cop_ring_free(tx)
    finally:
        L.coprocessor_teardown()


def test_no_nf_chain_forwards_everything(rules_file):
    """process_packet without ENABLE_FW_NF forwards every packet
    (coprocessor.c:59-64); the drop-in takes that chain from
    cop_coprocessor_setup_stages(0) (what coprocessor_setup() expands to in
    a build with DISABLE_NF or COP_DROPIN_NO_NF), including packets the
    firewall would drop."""
    path, rules = rules_file
    L = cg.lib()
    L.cop_set_mbuf_layout(0, 16)
    L.cop_set_rule_file(path.encode())
    assert L.cop_coprocessor_setup_stages(0) == 0
    try:
        n = 4000
        pk = cg.gen_trace(0x5EED0510, n, rules)
        mb = Mbufs(pk, n)
        fwo, _ = oracle_tables(rules)
        ro, _, _ = orc.process(pk, n, stages=DROPIN, fw=fwo)
        assert np.sum(ro["verdict"] != 0) > 0          # the firewall would drop some
        ptrs = (ctypes.c_void_p * n)(*[mb.ptr(i) for i in range(n)])
        ret = np.full(n, 7, dtype=np.int32)
        assert L.process_burst(ptrs, n, ret.ctypes.data) == 0
        assert np.all(ret == 0)
    finally:
        assert L.coprocessor_teardown() == 0
        L.cop_set_dropin_stages(cg.STAGE_FW)


def test_coprocessor_poll_pmd_rings(rules_file):
    """Three coprocessor threads, each with its own rx/tx ring pair, on ONE
    poll-mode kernel (cop_pmd_host_create: the reference's coprocessor lcores
    each polling its own rx ring, main.c:92-94): per thread the tx_q order
    equals the oracle's forward list of that thread's packets, every drop is
    freed exactly once, and nothing is left in flight after the flush."""
    import threading
    path, rules = rules_file
    L = cg.lib()
    L.cop_set_mbuf_layout(0, 16)
    L.cop_set_rule_file(path.encode())
    assert L.coprocessor_setup() == 0
    try:
        ctx = L.coprocessor_ctx()
        R, n, max_pkts = 3, 20000, 4096
        hp = ctypes.c_void_p()
        assert L.cop_pmd_host_create(ctx, R, max_pkts, 4, ctypes.byref(hp)) == 0
        fwo, _ = oracle_tables(rules)
        FREE = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p)
        res = [None] * R

        def loop(r):
            pk = cg.gen_trace(0x5EED0620 + r, n, rules)
            mb = Mbufs(pk, n)
            _, fo, _ = orc.process(pk, n, stages=DROPIN, fw=fwo)
            rx = L.cop_ring_create(16384)
            tx = L.cop_ring_create(65536)
            freed = []
            cb = FREE(lambda m, arg: freed.append(mb.index(m)))
            stats = cg.NfStats()
            sent = done = polls = 0
            out = []
            buf = (ctypes.c_void_p * 256)()
            while done < n:
                k_end = min(n, sent + 2500 + 700 * r)
                while sent < k_end:
                    k = min(32, k_end - sent)
                    arr = (ctypes.c_void_p * k)(*[mb.ptr(j) for j in range(sent, sent + k)])
                    if L.cop_ring_enqueue_bulk(rx, arr, k, None) != k:
                        break
                    sent += k
                got = L.cop_coprocessor_poll_pmd(hp, r, rx, tx, max_pkts, cb, None, ctypes.byref(stats))
                assert got >= 0, got
                done += got
                polls += 1
                assert polls < 20000
                while True:
                    k = L.cop_ring_dequeue_burst(tx, buf, 256, None)
                    if not k:
                        break
                    out += [mb.index(buf[i]) for i in range(k)]
            assert L.cop_coprocessor_flush_pmd(hp, r, tx, cb, None, ctypes.byref(stats)) == 0
            while True:
                k = L.cop_ring_dequeue_burst(tx, buf, 256, None)
                if not k:
                    break
                out += [mb.index(buf[i]) for i in range(k)]
            L.cop_ring_free(rx)
            L.cop_ring_free(tx)
            res[r] = (out == list(fo), sorted(freed) == sorted(set(range(n)) - set(fo)),
                      stats.tx_packets == len(fo) and stats.tx_dropped == 0)

        th = [threading.Thread(target=loop, args=(r,)) for r in range(R)]
        for t in th:
            t.start()
        for t in th:
            t.join(180)
        assert not any(t.is_alive() for t in th)
        assert L.cop_pmd_host_destroy(hp) == 0
        assert res == [(True, True, True)] * R, res
    finally:
        L.coprocessor_teardown()


def test_pmd_host_odd_max_pkts_equal_to_max_batch(rules_file, gpu_ctx_factory):
    """cop_pmd_host_create with an odd max_pkts equal to the
    context's max_batch. The ring's batches hold max_pkts packets (its
    slots are max_pkts rounded up to even apart), so the start no longer
    fails with 'n > max_batch'; one full drain of max_pkts packets comes
    back in the oracle's forward order, its drops freed."""
    path, rules = rules_file
    L = cg.lib()
    L.cop_set_mbuf_layout(0, 16)
    n = 4097
    ctx = gpu_ctx_factory(stages=cg.STAGE_FW, max_batch=n)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    hp = ctypes.c_void_p()
    assert L.cop_pmd_host_create(ctx.handle, 1, n, 2, ctypes.byref(hp)) == 0
    try:
        fwo, _ = oracle_tables(rules)
        pk = cg.gen_trace(0x5EED0630, n, rules)
        mb = Mbufs(pk, n)
        _, fo, _ = orc.process(pk, n, stages=DROPIN, fw=fwo)
        rx = L.cop_ring_create(16384)
        tx = L.cop_ring_create(16384)
        FREE = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p)
        freed = []
        cb = FREE(lambda m, arg: freed.append(mb.index(m)))
        stats = cg.NfStats()
        for s in range(0, n, 32):
            k = min(32, n - s)
            arr = (ctypes.c_void_p * k)(*[mb.ptr(j) for j in range(s, s + k)])
            assert L.cop_ring_enqueue_bulk(rx, arr, k, None) == k
        got = L.cop_coprocessor_poll_pmd(hp, 0, rx, tx, n, cb, None, ctypes.byref(stats))
        assert got >= 0, got
        assert L.cop_coprocessor_flush_pmd(hp, 0, tx, cb, None, ctypes.byref(stats)) >= 0
        buf = (ctypes.c_void_p * 256)()
        out = []
        while True:
            k = L.cop_ring_dequeue_burst(tx, buf, 256, None)
            if not k:
                break
            out += [mb.index(buf[i]) for i in range(k)]
        assert out == list(fo)
        assert sorted(freed) == sorted(set(range(n)) - set(fo))
        L.cop_ring_free(rx)
        L.cop_ring_free(tx)
    finally:
        assert L.cop_pmd_host_destroy(hp) == 0
