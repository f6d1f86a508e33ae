"""SPSC descriptor ring with rte_ring semantics (init.c:74-75; bulk enqueue
switch.c:225,268; burst dequeue switch.c:430,463)."""
import ctypes
import threading

import numpy as np

import copgpu as cg


def ring(n):
    r = cg.lib().cop_ring_create(n)
    assert r
    return r


def enq(r, vals):
    arr = (ctypes.c_void_p * len(vals))(*vals)
    free = ctypes.c_uint32()
    return cg.lib().cop_ring_enqueue_bulk(r, arr, len(vals), ctypes.byref(free)), free.value


def deq(r, n):
    arr = (ctypes.c_void_p * n)()
    avail = ctypes.c_uint32()
    k = cg.lib().cop_ring_dequeue_burst(r, arr, n, ctypes.byref(avail))
    return [arr[i] for i in range(k)], avail.value


def test_create_rejects_non_power_of_two():
    assert not cg.lib().cop_ring_create(1000)
    assert not cg.lib().cop_ring_create(0)


def test_capacity_is_size_minus_one_and_bulk_is_all_or_nothing():
    r = ring(16)
    sent, free = enq(r, list(range(1, 11)))
    assert sent == 10 and free == 5
    sent, free = enq(r, list(range(11, 17)))       # 6 > 5 free: nothing enqueued
    assert sent == 0 and free == 5
    sent, free = enq(r, list(range(11, 16)))
    assert sent == 5 and free == 0
    assert cg.lib().cop_ring_count(r) == 15
    got, avail = deq(r, 32)                        # burst: up to n
    assert got == list(range(1, 16)) and avail == 0
    got, _ = deq(r, 32)
    assert got == []
    cg.lib().cop_ring_free(r)


def test_wraparound_fifo_order():
    r = ring(8)
    out = []
    nxt = 1
    for _ in range(100):
        k = 3
        if enq(r, list(range(nxt, nxt + k)))[0] == k:
            nxt += k
        got, _ = deq(r, 2)
        out += got
    out += deq(r, 8)[0]
    assert out == list(range(1, nxt))
    cg.lib().cop_ring_free(r)


def test_spsc_threads():
    """One producer thread, one consumer thread (the fast path / coprocessor
    pairing): every object arrives exactly once, in order."""
    r = ring(1024)
    N = 200000
    got = []

    def producer():
        i = 1
        while i <= N:
            k = min(32, N - i + 1)
            if enq(r, list(range(i, i + k)))[0]:
                i += k

    def consumer():
        while len(got) < N:
            g, _ = deq(r, 32)
            got.extend(g)

    t1 = threading.Thread(target=producer)
    t2 = threading.Thread(target=consumer)
    t1.start()
    t2.start()
    t1.join(60)
    t2.join(60)
    assert np.array_equal(np.array(got, dtype=np.int64), np.arange(1, N + 1))
    cg.lib().cop_ring_free(r)
