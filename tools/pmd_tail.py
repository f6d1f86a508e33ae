#!/usr/bin/env python3
"""Diagnostic: where the tail of the driver's 20-batch poll-mode post comes
from. Posts `--posts` bursts of 20 fw1k batches (64k packets) to a 1024-slot
ring and, after each, reads the kernel's per-worker stamps ($COP_PMD_STAMPS:
tile start, batch seen, body done, counted; s_memrealtime, 100 MHz). Each
worker serves one 1024-packet tile per 20-batch post in the static order, so
per post every worker has one "counted" time after the doorbell relay.

Reports: the host post->done times; per XCD (worker % 8, workgroups being
dealt round-robin over the XCDs) the median / p90 / max of the counted
times; how often each XCD holds the post's slowest 5 % of tiles; whether a
worker that is slow in one post is slow in the next (rank correlation of
the per-worker times between posts); and the same split by the CU slot
within the XCD (worker // 8 % 32) and by the worker's slot on its CU
(worker // 256). Raw arrays go to --dump (npz) for offline analysis.

usage: python tools/pmd_tail.py [--posts 40] [--dump out.npz]
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ghost-dataplane_amd"))
os.environ.setdefault("COP_PMD_STAMPS", "1")
import copgpu as cg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--posts", type=int, default=40)
    ap.add_argument("--batches", type=int, default=20)
    ap.add_argument("--dump", default="")
    args = ap.parse_args()
    fw = cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)
    B, P = 65536, 1024
    ctx = cg.Context(stages=cg.STAGE_PARSE | cg.STAGE_FW, max_batch=B, flags=cg.CFG_SEG_LISTS)
    ctx.set_fw_table(cg.LpmTable(fw, 1024, 24))
    dp = ctx.alloc(P * B * 64)
    for i in range(0, P, 16):
        dp.upload(cg.gen_trace(0x5EED0002 + i, 16 * B, fw, None), i * B * 64)
    dr = ctx.alloc(P * B * 8)
    df = ctx.alloc(P * B * 4)
    dc = ctx.alloc(P * (B // cg.SEG_PKTS) * 4 + 16)
    ring = cg.make_ring(dp, P, B, dr, B * 64, stride=64, fwd_idx=df, fwd_count=dc)
    m = ctx.pmd_start(ring, cg.PMD_STATIC_SLOTS)
    info = m.info()
    G = info["workers"]
    print("pmd:", info, flush=True)
    lib = cg.lib()
    lib.cop_debug_pmd_stamps.restype = ctypes.c_int
    lib.cop_debug_pmd_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
    k = args.batches
    m.run(5)   # warm
    host, ends, seens, bodies = [], [], [], []
    buf = np.zeros(G * 8 + 128, np.uint64)
    for it in range(args.posts):
        t0 = time.perf_counter()
        m.post(k)
        m.wait()
        host.append((time.perf_counter() - t0) * 1e6)
        lib.cop_debug_pmd_stamps(m.handle, buf.ctypes.data, buf.size)
        st = buf[:G * 8].reshape(G, 8).astype(np.int64)
        relay = buf[G * 8:G * 8 + 128].reshape(64, 2).astype(np.int64)
        posted = m.posted
        r = relay[posted % 64]
        if r[0] != posted:
            continue
        mine = np.isin(st[:, 4], np.arange(posted - k, posted))
        end = np.full(G, np.nan)
        seen = np.full(G, np.nan)
        body = np.full(G, np.nan)
        end[mine] = (st[mine, 3] - r[1]) / 100.0      # us after the relay
        seen[mine] = (st[mine, 1] - r[1]) / 100.0
        body[mine] = (st[mine, 2] - st[mine, 1]) / 100.0
        ends.append(end)
        seens.append(seen)
        bodies.append(body)
        time.sleep(0.002)
    m.stop()
    ctx.close()
    E = np.array(ends)   # posts x workers
    print(f"{len(E)} posts of {k} batches; host post->done median {np.median(host):.1f} us "
          f"(p10 {np.percentile(host, 10):.1f}, p90 {np.percentile(host, 90):.1f})")
    allv = E[~np.isnan(E)]
    print("tile counted after the relay (us) p10/p50/p90/p99/max: "
          + " ".join(f"{np.percentile(allv, q):.1f}" for q in (10, 50, 90, 99, 100)))
    w = np.arange(E.shape[1])

    def split(name, key, nk):
        print(f"by {name}:")
        slow = E >= np.nanpercentile(E, 95, axis=1, keepdims=True)
        for g in range(nk):
            sel = key == g
            v = E[:, sel]
            v = v[~np.isnan(v)]
            if not len(v):
                continue
            share = slow[:, sel].sum() / max(1, slow.sum())
            sv, bv = np.array(seens)[:, sel], np.array(bodies)[:, sel]
            print(f"  {name} {g:2d}: workers {sel.sum():4d}  median {np.median(v):5.1f}  p90 {np.percentile(v, 90):5.1f}"
                  f"  max {v.max():5.1f}  share of the slowest 5 % {share:5.3f}"
                  f"  (seen {np.nanmedian(sv):4.2f}, body {np.nanmedian(bv):5.2f}, counted after body "
                  f"{np.nanmedian(v - (sv + bv)[~np.isnan(E[:, sel])]):4.2f})")

    split("XCD (w % 8)", w % 8, 8)
    split("slot on CU (w // 256)", w // 256, 5)
    # is a worker slow consistently? rank correlation of per-worker times
    # between consecutive posts
    cors = []
    for a, b in zip(E[:-1], E[1:]):
        ok = ~np.isnan(a) & ~np.isnan(b)
        ra = np.argsort(np.argsort(a[ok]))
        rb = np.argsort(np.argsort(b[ok]))
        cors.append(np.corrcoef(ra, rb)[0, 1])
    print(f"rank correlation of per-worker counted times between consecutive posts: median {np.median(cors):.3f}")
    S = np.array(seens)
    Bd = np.array(bodies)
    print("relay->seen (us) median/p90/max: "
          f"{np.nanmedian(S):.2f} {np.nanpercentile(S, 90):.2f} {np.nanmax(S):.2f}; body median/p90/max: "
          f"{np.nanmedian(Bd):.2f} {np.nanpercentile(Bd, 90):.2f} {np.nanmax(Bd):.2f}")
    if args.dump:
        np.savez(args.dump, ends=E, seens=S, bodies=Bd, host=np.array(host))


if __name__ == "__main__":
    main()
