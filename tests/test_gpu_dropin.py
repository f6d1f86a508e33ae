"""Drop-in coprocessor API on the GPU: coprocessor_setup / process_packet /
process_burst (coprocessor.c:21-65) with rte_mbuf-shaped descriptors, and
cop_coprocessor_poll, the GPU form of one coprocessor() call
(switch.c:443-474), over rte_ring-semantics rings."""
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
        ro, _, _ = orc.process(pk, n, stages=3, fw=fwo)
        want = np.where(ro["verdict"] == 0, 0, -1)
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
        ro, fo, _ = orc.process(pk, n, stages=3, fw=fwo)
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
        _, fo, _ = orc.process(pk, n, stages=3, fw=fwo)
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
