#!/usr/bin/env python3
"""Diagnostic: where the time of a SHORT timed region goes (the driver runs
bench.py --steps 20: one ring launch of 20 x 64k batches). For each tile
size (COP_PPT) and launch length: the host's submit->sync wall time
(median) and the kernel's own duration (HIP events on its stream).

usage: python tools/short_probe.py [--iters 50]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ghost-dataplane_amd"))
import copgpu as cg  # noqa: E402

S, F = cg.STAGE_PARSE, cg.STAGE_FW


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--ppts", default="0,1,4,8")
    ap.add_argument("--lens", default="1,4,20,64")
    args = ap.parse_args()
    fw = cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)
    B = 65536
    P = 128
    base = cg.Context(stages=S | F, max_batch=B)
    base.set_fw_table(cg.LpmTable(fw, 1024, 24))
    dp = base.alloc(P * B * 64)
    for i in range(0, P, 16):
        dp.upload(cg.gen_trace(0x5EED0002 + i, 16 * B, fw, None), i * B * 64)
    dr = base.alloc(P * B * 8)
    df = base.alloc(P * B * 4)
    dc = base.alloc(P * 4 + 16)
    ring = cg.make_ring(dp, P, B, dr, B * 64, stride=64, fwd_idx=df, fwd_count=dc)
    for ppt in [int(x) for x in args.ppts.split(",")]:
        if ppt:
            os.environ["COP_PPT"] = str(ppt)
        else:
            os.environ.pop("COP_PPT", None)
        ctx = cg.Context(stages=S | F, max_batch=B, n_streams=1)
        ctx.set_fw_table(cg.LpmTable(fw, 1024, 24))
        for L in [int(x) for x in args.lens.split(",")]:
            for w in range(5):
                ctx.submit_ring(ring, (w * L) % P, L)
            ctx.sync()
            host = []
            ctx.launch_timing(True)
            for i in range(args.iters):
                t0 = time.perf_counter()
                ctx.submit_ring(ring, (i * L) % P, L)
                ctx.sync()
                host.append((time.perf_counter() - t0) * 1e6)
            k_ms, n = ctx.launch_timing_read(reset=True)
            ctx.launch_timing(False)
            h = float(np.median(host))
            print(f"ppt {ppt or 'auto':>4} L {L:4d}: host submit->sync median {h:8.1f} us, kernel {k_ms * 1e3:8.1f} us "
                  f"-> {L * B / h:9.1f} Mpkt/s host, {L * B / (k_ms * 1e3):9.1f} Mpkt/s kernel", flush=True)
        ctx.close()
    base.close()


if __name__ == "__main__":
    main()
