#!/usr/bin/env python3
"""Latency of the synchronous host path (cop_process_host: what
process_packet / process_burst / cop_coprocessor_poll call): packets in an
mbuf-like host pool, per-call wall time for batch sizes from one packet to
64k, median of 200 calls (50 for the largest). $COP_ZC_MAX selects the
zero-copy form (mapped pinned memory, default up to 65536 packets) or, at 0,
the copy-engine form. Results are checked against the oracle once per size.
"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ghost-dataplane_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import copgpu as cg  # noqa: E402
import oracle as orc  # noqa: E402

NB, STRIDE, HEADROOM = 65536, 2176, 128


def main():
    fw = cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)
    pk = cg.gen_trace(0x5EED0002, NB, fw)
    pool = np.zeros(NB * STRIDE, np.uint8)
    pool.reshape(NB, STRIDE)[:, HEADROOM:HEADROOM + 64] = pk.reshape(NB, 64)
    ptrs = (pool.ctypes.data + HEADROOM + np.arange(NB, dtype=np.uint64) * STRIDE).astype(np.uint64)
    o = orc.OracleLpm(1024, 24)
    o.setup(fw["ip"], fw["depth"], fw["next_hop"])
    ro, _, _ = orc.process(pk, NB, stages=3, fw=o)
    ctx = cg.Context(stages=cg.STAGE_PARSE | cg.STAGE_FW)
    ctx.set_fw_table(cg.LpmTable(fw, 1024, 24))
    L = cg.lib()
    res = np.zeros(NB, cg.RESULT_DT)
    pp = ctypes.cast(ptrs.ctypes.data, ctypes.POINTER(ctypes.c_void_p))
    mode = os.environ.get("COP_ZC_MAX", "65536 (default)")
    print(f"COP_ZC_MAX={mode}")
    for n in (1, 32, 256, 4096, 16384, 65536):
        reps = 50 if n >= 65536 else 200
        rc = L.cop_process_host(ctx.handle, pp, n, res.ctypes.data, None, None)
        assert rc == 0, rc
        ok = np.array_equal(res[:n].view(np.uint8), ro[:n].view(np.uint8))
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            L.cop_process_host(ctx.handle, pp, n, res.ctypes.data, None, None)
            ts.append(time.perf_counter() - t0)
        med = float(np.median(ts)) * 1e6
        print(f"  n {n:6d}: {med:8.1f} us per call, {n / med:8.1f} Mpkt/s  {'ok' if ok else 'MISMATCH'}",
              flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
