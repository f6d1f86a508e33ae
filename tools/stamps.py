#!/usr/bin/env python3
"""Diagnostic: per-workgroup phase timeline of one launch (COP_DBG bit 8,
s_memrealtime at 100 MHz). Reports, over workgroups, the median / p90 of
each phase and the launch span. Timing-only build flag; outputs of that
launch are still checked by nothing here.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ghost-dataplane_amd"))
os.environ["COP_DBG"] = str(8 | int(os.environ.get("EXTRA_DBG", "0")))
import copgpu as cg  # noqa: E402

S, F, L = cg.STAGE_PARSE, cg.STAGE_FW, cg.STAGE_LPM
PH = ["ticket+stage", "loads+P", "lookups", "store", "compact", "tail"]


def run(stages, Lb, compact, label, ring=False):
    fw = cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)
    routes = cg.gen_rules(0x5EED2004, 100000, cg.GEN_ROUTES, 0)
    ctx = cg.Context(stages=stages)
    ctx.set_fw_table(cg.LpmTable(fw, 1024, 24))
    ctx.set_route_lpm(cg.LpmTable(routes, 1 << 20, 1 << 16, False))
    B = 65536
    P = 100 if ring else 64
    dp = ctx.alloc(P * B * 64)
    for i in range(0, P, 16):
        k = min(16, P - i)
        dp.upload(cg.gen_trace(0x5EED0002 + i, k * B, fw, routes), i * B * 64)
    dr = ctx.alloc(P * B * 8)
    df = ctx.alloc(P * B * 4)
    dc = ctx.alloc(P * 4)
    rg = cg.make_ring(dp, P, B, dr, B * 64, fwd_idx=df if compact else None, fwd_count=dc if compact else None)
    for it in range(6):
        if ring:
            ctx.submit_ring(rg, 0, Lb)
            continue
        bl = []
        for j in range(Lb):
            i = (it * Lb + j) % P
            bl.append(cg.make_batch(dp.addr + i * B * 64, B, dr.addr + i * B * 8,
                                    fwd_idx=(df.addr + i * B * 4) if compact else None,
                                    fwd_count=(dc.addr + i * 4) if compact else None))
        ctx.submit(bl)
    ctx.sync()
    lib = cg.lib()
    lib.cop_debug_stamps.restype = ctypes.c_int
    lib.cop_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
    n = 65536 * 8
    buf = np.zeros(n, dtype=np.uint64)
    k = lib.cop_debug_stamps(ctx.handle, buf.ctypes.data_as(ctypes.c_void_p), n)
    st = buf[:k].reshape(-1, 8).astype(np.int64)
    st = st[st[:, 0] > 0]
    t0 = st[:, 0].min()
    span = (st[:, 6].max() - t0) * 10 / 1000
    print(f"== {label}: {len(st)} workgroups, span {span:.2f} us")
    starts = (st[:, 0] - t0) * 10 / 1000
    print(f"   start spread  median {np.median(starts):.2f}  p90 {np.percentile(starts, 90):.2f}  max {starts.max():.2f} us")
    ends = (st[:, 6] - t0) * 10 / 1000
    print(f"   end           min {ends.min():.2f}  median {np.median(ends):.2f}  max {ends.max():.2f} us")
    for a, name in enumerate(PH):
        b = a + 1
        if not compact and a == 4:
            d = (st[:, 6] - st[:, 4]) * 10 / 1000
            print(f"   {'store->end':14s} median {np.median(d):6.2f}  p90 {np.percentile(d, 90):6.2f} us")
            break
        d = (st[:, b] - st[:, a]) * 10 / 1000
        print(f"   {name:14s} median {np.median(d):6.2f}  p90 {np.percentile(d, 90):6.2f} us")
    # workgroups in flight over the launch (5 us buckets)
    t_end = (st[:, 6] - t0) * 10 / 1000
    edges = np.arange(0, t_end.max() + 5, 5)
    act = [int(((starts < e + 5) & (t_end > e)).sum()) for e in edges]
    print("   active WGs per 5us:", act)
    ctx.close()


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "short":
        # the driver's short timed region: one ring launch of 20 batches; one batch
        run(S | F, 20, True, "fw ring L20 compact", ring=True)
        run(S | F, 1, True, "fw ring L1 compact", ring=True)
        run(S | F, 1, False, "fw ring L1 no-compact", ring=True)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "ring":
        run(S | F, 96, True, "fw ring L96 compact", ring=True)
        run(S | F | L, 96, True, "fw+lpm ring L96 compact", ring=True)
        sys.exit(0)
    run(S | F, 16, True, "fw L16 compact")
    run(S | F, 16, False, "fw L16 no-compact")
    run(S | F, 1, True, "fw L1 compact")
    run(S | F | L, 16, True, "fw+lpm L16 compact")
