#!/usr/bin/env python3
"""End-to-end rate of the host-memory path (north star: "packets start and
end in host memory ... pinned hipMemcpyAsync in and out"): packets sit in an
mbuf-like host pool (NB_MBUF = 131072 buffers at 2176 B stride, data at
128 B headroom, init.h:38-44); cop_process_host_stream packs each batch's
16-byte header records (COP_HDR16_STRIDE: frame bytes 12..15, 24..35) into
pinned staging, copies H2D, runs the pipeline,
copies the 8-byte records D2H, with the lanes overlapping; the gather runs
on 1..16 host threads (cop_set_host_threads). Results of the first pool
pass are checked bit-exactly against the oracle.
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ghost-dataplane_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import copgpu as cg  # noqa: E402

NB_MBUF, STRIDE, HEADROOM = 131072, 2176, 128


def main():
    fw = cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)
    pk = cg.gen_trace(0x5EED0002, NB_MBUF, fw)
    pool = np.zeros(NB_MBUF * STRIDE, dtype=np.uint8)
    pool.reshape(NB_MBUF, STRIDE)[:, HEADROOM:HEADROOM + 64] = pk.reshape(NB_MBUF, 64)
    base = pool.ctypes.data + HEADROOM
    n = 16 * NB_MBUF
    ptrs = (base + (np.arange(n, dtype=np.uint64) % NB_MBUF) * STRIDE).astype(np.uint64)

    import oracle as orc
    o = orc.OracleLpm(1024, 24)
    o.setup(fw["ip"], fw["depth"], fw["next_hop"])
    ro, _, _ = orc.process(pk, NB_MBUF, stages=3, fw=o)

    print(f"{'lanes':>5s} {'thr':>3s} {'batch':>7s} {'Mpkt/s':>9s} {'GB/s H2D':>9s}  parity")
    for lanes, threads in ((1, 1), (2, 1), (4, 1), (2, 4), (4, 4), (2, 8), (4, 8), (2, 16), (4, 16)):
        ctx = cg.Context(stages=cg.STAGE_PARSE | cg.STAGE_FW, n_streams=lanes)
        ctx.set_fw_table(cg.LpmTable(fw, 1024, 24))
        ctx.set_host_threads(threads)
        for batch in (16384, 65536, 262144):
            res = ctx.process_host_stream(ptrs[:NB_MBUF], batch)    # warm + parity
            ok = np.array_equal(res.view(np.uint8), ro.view(np.uint8))
            t0 = time.perf_counter()
            res = ctx.process_host_stream(ptrs, batch)
            dt = time.perf_counter() - t0
            print(f"{lanes:5d} {threads:3d} {batch:7d} {n / dt / 1e6:9.1f} {n * cg.HDR16_STRIDE / dt / 1e9:9.2f}  "
                  f"{'ok' if ok else 'MISMATCH'}", flush=True)
        ctx.close()
    # synchronous single-batch path (cop_process_host) for reference
    ctx = cg.Context(stages=cg.STAGE_PARSE | cg.STAGE_FW)
    ctx.set_fw_table(cg.LpmTable(fw, 1024, 24))
    res, fwd = ctx.process_host(pk, 65536)
    t0 = time.perf_counter()
    for _ in range(8):
        ctx.process_host(pk, 65536)
    dt = time.perf_counter() - t0
    print(f"cop_process_host (sync, 64k, incl. Python pointer list): {8 * 65536 / dt / 1e6:.1f} Mpkt/s")
    # the CPU baseline on the same box, same run, per core count: the oracle's
    # restatement of the reference's coprocessor() loop (bench.py's
    # cpu_baseline), so the host paths above read per core against it
    trace = cg.gen_trace(0x5EED0001, NB_MBUF, fw, None)
    for cores in (1, 4, 8, 16):
        rate, pk_n, secs = orc.coprocessor_bench(trace, NB_MBUF, o, 3.0, cores, max(os.sched_getaffinity(0)) if cores == 1
                                                 else -1)
        print(f"cpu baseline: restated coprocessor() loop, {cores:2d} thread(s): {rate:9.1f} Mpkt/s "
              f"({rate / cores:.1f} per core)", flush=True)


if __name__ == "__main__":
    main()
