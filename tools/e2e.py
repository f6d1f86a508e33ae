#!/usr/bin/env python3
"""End-to-end rate of the host-memory path (north star: "packets start and
end in host memory ... pinned hipMemcpyAsync in and out"): packets sit in an
mbuf-like host pool (NB_MBUF = 131072 buffers at 2176 B stride, data at
128 B headroom, init.h:38-44); cop_process_host_stream packs each batch's
12-byte header records (COP_HDR12_STRIDE: frame bytes 12..15, 26..33; or 16,
$COP_STREAM_REC) into
pinned staging, copies H2D, runs the pipeline,
copies the 8-byte records D2H, with the lanes overlapping (or, zc, the
kernel reads and writes mapped pinned memory: $COP_STREAM_ZC); the gather
runs on 1..16 host threads (cop_set_host_threads), never more than the
job's CPU share. Results of the first pool pass are checked bit-exactly
against the oracle.
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
    n = 64 * NB_MBUF
    ptrs = (base + (np.arange(n, dtype=np.uint64) % NB_MBUF) * STRIDE).astype(np.uint64)
    out = np.zeros(n, dtype=cg.RESULT_DT)

    import oracle as orc
    o = orc.OracleLpm(1024, 24)
    o.setup(fw["ip"], fw["depth"], fw["next_hop"])
    ro, _, _ = orc.process(pk, NB_MBUF, stages=3, fw=o)

    # host threads never above the job's CPU share ($OMP_NUM_THREADS, 16 on
    # the pool's one-GPU boxes): more gather threads than cores collapse
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
    rec_b = int(os.environ.get("COP_STREAM_REC", "12"))
    lanes_l = [int(x) for x in os.environ.get("E2E_LANES", "2,4").split(",")]
    thr_l = [int(x) for x in os.environ.get("E2E_THREADS", "1,2,4,8,12,16").split(",")]
    print(f"{'lanes':>5s} {'thr':>3s} {'zc':>2s} {'batch':>7s} {'Mpkt/s':>9s} {'GB/s H2D':>9s}  parity", flush=True)
    for zc in (int(x) for x in os.environ.get("E2E_MODES", "0,1,2").split(",")):
        os.environ["COP_STREAM_ZC"] = str(zc)
        for lanes in lanes_l:
            for threads in thr_l:
                if threads > share:
                    continue
                batch = int(os.environ.get("E2E_BATCH", "262144"))
                ctx = cg.Context(stages=cg.STAGE_PARSE | cg.STAGE_FW, n_streams=lanes, max_batch=batch)
                ctx.set_fw_table(cg.LpmTable(fw, 1024, 24))
                ctx.set_host_threads(threads)
                res = ctx.process_host_stream(ptrs[:NB_MBUF], batch)    # warm + parity
                ok = np.array_equal(res.view(np.uint8), ro.view(np.uint8))
                ts = []
                for _ in range(5):
                    t0 = time.perf_counter()
                    ctx.process_host_stream(ptrs, batch, out=out)
                    ts.append(time.perf_counter() - t0)
                dt = float(np.median(ts))
                print(f"{lanes:5d} {threads:3d} {zc:2d} {batch:7d} {n / dt / 1e6:9.1f} {n * rec_b / dt / 1e9:9.2f}  "
                      f"{'ok' if ok else 'MISMATCH'}", flush=True)
                ctx.close()
    # batch size at the default mode (larger copies, fewer per-batch calls)
    os.environ["COP_STREAM_ZC"] = "2"
    for lanes, threads, batch in ((4, share, 524288), (4, share, 131072), (4, share, 65536), (3, share, 131072),
                                  (4, 8, 131072), (4, 4, 131072)):
        ctx = cg.Context(stages=cg.STAGE_PARSE | cg.STAGE_FW, n_streams=lanes, max_batch=batch)
        ctx.set_fw_table(cg.LpmTable(fw, 1024, 24))
        ctx.set_host_threads(threads)
        res = ctx.process_host_stream(ptrs[:NB_MBUF], batch)
        ok = np.array_equal(res.view(np.uint8), ro.view(np.uint8))
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            ctx.process_host_stream(ptrs, batch, out=out)
            ts.append(time.perf_counter() - t0)
        dt = float(np.median(ts))
        print(f"{lanes:5d} {threads:3d}  2 {batch:7d} {n / dt / 1e6:9.1f} {n * rec_b / dt / 1e9:9.2f}  "
              f"{'ok' if ok else 'MISMATCH'}", flush=True)
        ctx.close()
    # 16-byte records against the default 12-byte ones ($COP_STREAM_REC)
    for rec in (16, 12, 16, 12):
        os.environ["COP_STREAM_REC"] = str(rec)
        ctx = cg.Context(stages=cg.STAGE_PARSE | cg.STAGE_FW, n_streams=4, max_batch=131072)
        ctx.set_fw_table(cg.LpmTable(fw, 1024, 24))
        ctx.set_host_threads(share)
        res = ctx.process_host_stream(ptrs[:NB_MBUF], 131072)
        ok = np.array_equal(res.view(np.uint8), ro.view(np.uint8))
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            ctx.process_host_stream(ptrs, 131072, out=out)
            ts.append(time.perf_counter() - t0)
        dt = float(np.median(ts))
        print(f"records {rec:2d} B, 4 lanes, {share} threads, 131072: {n / dt / 1e6:.1f} Mpkt/s, "
              f"{n * rec / dt / 1e9:.2f} GB/s H2D  {'ok' if ok else 'MISMATCH'}", flush=True)
        ctx.close()
    os.environ.pop("COP_STREAM_REC", None)
    # timing ablations at the default mode: no H2D copy ($COP_DBG 0x100;
    # results wrong), and no gather (the same 131072 records every batch)
    for what, env in (("no H2D copy", {"COP_DBG": "0x100"}),):
        os.environ.update(env)
        ctx = cg.Context(stages=cg.STAGE_PARSE | cg.STAGE_FW, n_streams=4, max_batch=131072)
        ctx.set_fw_table(cg.LpmTable(fw, 1024, 24))
        ctx.set_host_threads(share)
        ctx.process_host_stream(ptrs[:NB_MBUF], 131072)
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            ctx.process_host_stream(ptrs, 131072, out=out)
            ts.append(time.perf_counter() - t0)
        print(f"ablation ({what}), 4 lanes, {share} threads, 131072: {n / float(np.median(ts)) / 1e6:.1f} Mpkt/s",
              flush=True)
        ctx.close()
        for k in env:
            os.environ.pop(k, None)
    os.environ.pop("COP_STREAM_ZC", None)
    # the H2D copy alone: pinned staging -> HBM, 4 MiB chunks, the copy engine's rate
    ctx = cg.Context(stages=cg.STAGE_PARSE | cg.STAGE_FW)
    lib = cg.lib()
    import ctypes
    hp = ctypes.c_void_p()
    nbytes = 64 << 20
    if lib.cop_host_alloc_pinned(ctx.handle, nbytes, ctypes.byref(hp)) == 0:
        d = ctx.alloc(nbytes)
        f = lib.cop_memcpy_h2d
        t0 = time.perf_counter()
        reps = 20
        for _ in range(reps):
            f(ctx.handle, ctypes.c_void_p(d.addr), hp, ctypes.c_uint64(nbytes))
        ctx.sync()
        dt = time.perf_counter() - t0
        print(f"pinned H2D copy, {nbytes >> 20} MiB x {reps}: {reps * nbytes / dt / 1e9:.1f} GB/s", flush=True)
        lib.cop_host_free_pinned(ctx.handle, hp)
    ctx.close()
    # the CPU baseline on the same box, same run, per core count: the oracle's
    # restatement of the reference's coprocessor() loop (bench.py's
    # cpu_baseline), so the host paths above read per core against it
    trace = cg.gen_trace(0x5EED0001, NB_MBUF, fw, None)
    for cores in (1, 4, 8, 16):
        if cores > share:
            continue
        rate, pk_n, secs = orc.coprocessor_bench(trace, NB_MBUF, o, 3.0, cores, max(os.sched_getaffinity(0)) if cores == 1
                                                 else -1)
        print(f"cpu baseline: restated coprocessor() loop, {cores:2d} thread(s): {rate:9.1f} Mpkt/s "
              f"({rate / cores:.1f} per core)", flush=True)


if __name__ == "__main__":
    main()
