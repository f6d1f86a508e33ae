#!/usr/bin/env python3
"""Diagnostic: where a poll-mode post spends its time. Posts of 1 and 20
batches (fw1k, 64k packets), host post->wait time, and the kernel's phase
stamps ($COP_PMD_STAMPS, s_memrealtime 100 MHz) for the last post: doorbell
relay -> first/last tile start -> tile bodies -> last tile counted.

usage: python tools/pmd_probe.py [--iters 30]
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ghost-dataplane_amd"))
os.environ.setdefault("COP_PMD_STAMPS", "1")   # 1: tile stamps (production kernel); 2: + body phases (EXT kernel)
import copgpu as cg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--posts", default="1,20,64,128")
    ap.add_argument("--lists", default="seg", choices=("seg", "dense"))
    ap.add_argument("--dump", default="", help="save each post's raw stamps to <prefix>_post<k>.npz")
    ap.add_argument("--rules", type=int, default=1000, help="firewall rules (fw1k: 1000)")
    args = ap.parse_args()
    fw = cg.gen_rules(0x5EED1002, args.rules, cg.GEN_FW, 20 if args.rules >= 20 else 0)
    B, P = 65536, 128
    ctx = cg.Context(stages=cg.STAGE_PARSE | cg.STAGE_FW, max_batch=B,
                     flags=cg.CFG_SEG_LISTS if args.lists == "seg" else 0)
    ctx.set_fw_table(cg.LpmTable(fw, 1024, 24))
    dp = ctx.alloc(P * B * 64)
    for i in range(0, P, 16):
        dp.upload(cg.gen_trace(0x5EED0002 + i, 16 * B, fw, None), i * B * 64)
    dr = ctx.alloc(P * B * 8)
    df = ctx.alloc(P * B * 4)
    dc = ctx.alloc(P * (B // cg.SEG_PKTS) * 4 + 16)
    ring = cg.make_ring(dp, P, B, dr, B * 64, stride=64, fwd_idx=df, fwd_count=dc)
    m = ctx.pmd_start(ring)
    info = m.info()
    print("pmd:", info, "fw rules", args.rules, "intervals", ctx.fw_intervals() if hasattr(ctx, "fw_intervals") else "?",
          flush=True)
    lib = cg.lib()
    lib.cop_debug_pmd_stamps.restype = ctypes.c_int
    lib.cop_debug_pmd_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
    G = info["workers"]
    for k in [int(x) for x in args.posts.split(",")]:
        m.post(k)
        m.wait()
        host = []
        for _ in range(args.iters):
            t0 = time.perf_counter()
            m.post(k)
            m.wait()
            host.append((time.perf_counter() - t0) * 1e6)
        buf = np.zeros(G * 16 + 128, np.uint64)
        n = lib.cop_debug_pmd_stamps(m.handle, buf.ctypes.data, buf.size)
        st = buf[:G * 8].reshape(G, 8).astype(np.int64)
        relay = buf[G * 8:G * 8 + 128].reshape(64, 2).astype(np.int64)
        posted = m.posted
        last_batches = set(range(posted - k, posted))
        mine = st[np.isin(st[:, 4], list(last_batches))]
        r = relay[posted % 64]
        assert r[0] == posted, (r, posted)
        t_relay = r[1]
        us = lambda x: x * 10 / 1000.0  # noqa: E731
        seen = mine[:, 1] - t_relay
        body = mine[:, 2] - mine[:, 1]
        drain = mine[:, 3] - mine[:, 2]
        end = mine[:, 3] - t_relay
        if n > G * 8 + 128:
            ts = buf[G * 8 + 128:G * 16 + 128].reshape(G, 8).astype(np.int64)
            sel = np.isin(st[:, 4], list(last_batches))
            tb = ts[sel]
            ph = {"seen->pass1 (loads+P+lookups)": tb[:, 2] - mine[:, 1], "pass2": tb[:, 3] - tb[:, 2],
                  "compaction+records": tb[:, 5] - tb[:, 3], "counters": tb[:, 6] - tb[:, 5]}
            print("   body phases (median/max us): " + "; ".join(f"{k2} {us(np.median(v)):.2f}/{us(v.max()):.2f}"
                                                              for k2, v in ph.items()))
        if args.dump:
            # raw stamps of this post's tiles (worker = row index), for offline analysis
            sel = np.isin(st[:, 4], list(last_batches))
            extra = buf[G * 8 + 128:G * 16 + 128].reshape(G, 8).astype(np.int64) if n > G * 8 + 128 else None
            np.savez(f"{args.dump}_post{k}.npz", stamps=st, sel=sel, relay=t_relay, phases=extra)
        # when the tiles of the post finished, relative to the relay (us): quantiles
        q = np.percentile(end, [10, 50, 90, 99, 100])
        sq = np.percentile(seen, [10, 50, 90, 100])
        print("   tile counted at (p10/p50/p90/p99/max us after relay): " + " ".join(f"{us(x):.1f}" for x in q)
              + "; seen at (p10/p50/p90/max): " + " ".join(f"{us(x):.1f}" for x in sq))
        print(f"post {k:3d}: host post->done median {np.median(host):7.1f} us (min {min(host):.1f}); "
              f"{len(mine)} tiles; relay->seen min {us(seen.min()):.2f} med {us(np.median(seen)):.2f} "
              f"max {us(seen.max()):.2f}; body med {us(np.median(body)):.2f} max {us(body.max()):.2f}; "
              f"drain+count med {us(np.median(drain)):.2f} max {us(drain.max()):.2f}; relay->last counted "
              f"{us(end.max()):.2f} us", flush=True)
    m.stop()
    ctx.close()


if __name__ == "__main__":
    main()
