#!/usr/bin/env python3
"""Diagnose the multi-ring drop-in loop (cop_pmd_host): per ring, how the
tx order and the freed set differ from the oracle's, single-threaded
(rings driven in turn) and with one thread per ring.
usage: rings_diag.py [R] [threads 0|1] [chunk]"""
import ctypes
import os
import sys
import tempfile
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ghost-dataplane_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), ROOT]
import copgpu as cg  # noqa: E402
import oracle as orc  # noqa: E402
from helpers import oracle_tables  # noqa: E402
from test_gpu_dropin import Mbufs  # noqa: E402


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    threaded = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    chunk = int(sys.argv[3]) if len(sys.argv) > 3 else 2500
    rules = cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)
    d = tempfile.mkdtemp()
    path = os.path.join(d, "rules.json")
    cg.rules_write_json(path, rules)
    L = cg.lib()
    L.cop_set_mbuf_layout(0, 16)
    L.cop_set_rule_file(path.encode())
    assert L.coprocessor_setup() == 0
    ctx = L.coprocessor_ctx()
    n, max_pkts = 20000, 4096
    hp = ctypes.c_void_p()
    assert L.cop_pmd_host_create(ctx, R, max_pkts, 4, ctypes.byref(hp)) == 0
    fwo, _ = oracle_tables(rules)
    FREE = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p)
    st = {}
    for r in range(R):
        pk = cg.gen_trace(0x5EED0620 + r, n, rules)
        mb = Mbufs(pk, n)
        _, fo, _ = orc.process(pk, n, stages=cg.STAGE_FW, fw=fwo)
        s = dict(mb=mb, fo=list(fo), rx=L.cop_ring_create(16384), tx=L.cop_ring_create(65536), freed=[], out=[],
                 sent=0, done=0, stats=cg.NfStats(), batches=[])
        s["cb"] = FREE(lambda m, arg, s=s: s["freed"].append(s["mb"].index(m)))
        st[r] = s
    buf = (ctypes.c_void_p * 256)()

    def step(r):
        s = st[r]
        k_end = min(n, s["sent"] + chunk + 700 * r)
        while s["sent"] < k_end:
            k = min(32, k_end - s["sent"])
            arr = (ctypes.c_void_p * k)(*[s["mb"].ptr(j) for j in range(s["sent"], s["sent"] + k)])
            if L.cop_ring_enqueue_bulk(s["rx"], arr, k, None) != k:
                break
            s["sent"] += k
        got = L.cop_coprocessor_poll_pmd(hp, r, s["rx"], s["tx"], max_pkts, s["cb"], None, ctypes.byref(s["stats"]))
        assert got >= 0, got
        s["done"] += got
        s["batches"].append(got)
        while True:
            k = L.cop_ring_dequeue_burst(s["tx"], buf, 256, None)
            if not k:
                break
            s["out"] += [s["mb"].index(buf[i]) for i in range(k)]

    def finish(r):
        s = st[r]
        assert L.cop_coprocessor_flush_pmd(hp, r, s["tx"], s["cb"], None, ctypes.byref(s["stats"])) >= 0
        while True:
            k = L.cop_ring_dequeue_burst(s["tx"], buf, 256, None)
            if not k:
                break
            s["out"] += [s["mb"].index(buf[i]) for i in range(k)]

    if threaded:
        def loop(r):
            while st[r]["done"] < n:
                step(r)
            finish(r)
        th = [threading.Thread(target=loop, args=(r,)) for r in range(R)]
        for t in th:
            t.start()
        for t in th:
            t.join(120)
    else:
        while any(st[r]["done"] < n for r in range(R)):
            for r in range(R):
                if st[r]["done"] < n:
                    step(r)
        for r in range(R):
            finish(r)
    assert L.cop_pmd_host_destroy(hp) == 0
    for r in range(R):
        s = st[r]
        out, fo = s["out"], s["fo"]
        bad = next((i for i in range(min(len(out), len(fo))) if out[i] != fo[i]), None)
        fr = sorted(s["freed"])
        want_fr = sorted(set(range(n)) - set(fo))
        print(f"ring {r}: out {len(out)} want {len(fo)} first diff {bad} "
              f"(got {out[bad] if bad is not None else '-'} want {fo[bad] if bad is not None else '-'}) "
              f"freed {len(fr)} want {len(want_fr)} ok {out == fo and fr == want_fr} "
              f"tx {s['stats'].tx_packets} batches {s['batches'][:12]}", flush=True)
        if bad is not None:
            extra = sorted(set(out) - set(fo))[:10]
            missing = sorted(set(fo) - set(out))[:10]
            print(f"   forwarded but dropped by oracle: {extra}  missing: {missing}", flush=True)
    L.coprocessor_teardown()


if __name__ == "__main__":
    main()
