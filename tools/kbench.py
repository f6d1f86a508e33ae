#!/usr/bin/env python3
"""A/B kernel experiments (not the contract bench): per-launch kernel time
and algorithmic GB/s for several variants, interleaved rounds in one
process (cdna_hip_programming.md §5.4 rule 24).

usage: python tools/kbench.py [--rounds 5] [--variants a,b,...]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ghost-dataplane_amd"))
import copgpu as cg  # noqa: E402

S, F, L = cg.STAGE_PARSE, cg.STAGE_FW, cg.STAGE_LPM


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=40)
    ap.add_argument("--variants", default="")
    args = ap.parse_args()

    fw_rules = cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)
    routes = cg.gen_rules(0x5EED2004, 100000, cg.GEN_ROUTES, 0)
    B = 65536
    P = 100
    ctxs = {}

    def ctx_for(stages, flags, env=()):
        key = (stages, flags, env)
        if key not in ctxs:
            saved = {k: os.environ.get(k) for k, _ in env}
            os.environ.update(dict(env))
            c = cg.Context(stages=stages, flags=flags, max_batch=262144)
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            c.set_fw_table(cg.LpmTable(fw_rules, 1024, 24))
            c.set_route_lpm(cg.LpmTable(routes, 1 << 20, 1 << 16, False))
            ctxs[key] = c
        return ctxs[key]

    base = ctx_for(S | F, 0)
    d_pk = base.alloc(P * B * 64)
    for i in range(0, P, 20):
        d_pk.upload(cg.gen_trace(0x5EED0002 + i, 20 * B, fw_rules, routes), i * B * 64)
    d_res = base.alloc(P * B * 8)
    d_fwd = base.alloc(P * B * 4)
    d_cnt = base.alloc(P * 4)

    variants = {
        # name: (stages, flags, per_launch, compact)
        "fw_L16": (S | F, 0, 16, True),
        "fw_L16_nocompact": (S | F, 0, 16, False),
        "fw_L1": (S | F, 0, 1, True),
        "fw_L4": (S | F, 0, 4, True),
        "fw_L32": (S | F, 0, 32, True),
        "fw_dir_L16": (S | F, cg.CFG_FW_FORCE_DIR24, 16, True),
        "p_only_L16": (S, 0, 16, True),
        "fw_lpm_L16": (S | F | L, 0, 16, True),
    }
    for ppt in (1, 4, 8):
        variants[f"fw_L16_p{ppt}"] = (S | F, 0, 16, True, (("COP_PPT", str(ppt)),))
    for ns in (1, 2, 4):
        variants[f"fw_L16_s{ns}"] = (S | F, 0, 16, True, (("COP_STREAMS", str(ns)),))
        variants[f"fw_L32_s{ns}"] = (S | F, 0, 32, True, (("COP_STREAMS", str(ns)),))
    # timing-only ablations (COP_DBG bits: 1 no counter atomics, 2 static tiles, 4 no LDS staging)
    for dbg in (1, 2, 3, 7):
        variants[f"nc_dbg{dbg}"] = (S | F, 0, 16, False, (("COP_DBG", str(dbg)),))
    variants["c_dbg1"] = (S | F, 0, 16, True, (("COP_DBG", "1"),))
    for Lr in (16, 32, 64, 100):
        for ns in (1, 2):
            variants[f"ring_L{Lr}_s{ns}"] = (S | F, 0, Lr, True, (("COP_STREAMS", str(ns)),), "ring")
    variants["ring_lpm_L64_s1"] = (S | F | L, 0, 64, True, (("COP_STREAMS", "1"),), "ring")
    variants["ring_L96_s1"] = (S | F, 0, 96, True, (("COP_STREAMS", "1"),), "ring")
    variants["ring_L96_s1_static"] = (S | F, 0, 96, True, (("COP_STREAMS", "1"), ("COP_DBG", "2")), "ring")
    variants["ring_L96_s1_nocompact"] = (S | F, 0, 96, False, (("COP_STREAMS", "1"),), "ring")
    variants["ring_L96_s1_p4"] = (S | F, 0, 96, True, (("COP_STREAMS", "1"), ("COP_PPT", "4")), "ring")
    variants["ring_lpm_L96_s1"] = (S | F | L, 0, 96, True, (("COP_STREAMS", "1"),), "ring")
    variants["ring_lpm_L96_s1_static"] = (S | F | L, 0, 96, True, (("COP_STREAMS", "1"), ("COP_DBG", "2")), "ring")
    names = [v for v in args.variants.split(",") if v] or list(variants)
    res = {n: [] for n in names}
    for r in range(args.rounds):
        for n in names:
            stages, flags, Lb, compact, *env = variants[n]
            ctx = ctx_for(stages, flags, env[0] if env else ())
            is_ring = len(env) > 1 and env[1] == "ring"
            ring = cg.make_ring(d_pk, P, B, d_res, B * 64, fwd_idx=d_fwd if compact else None,
                                fwd_count=d_cnt if compact else None)

            def sub_ring(i0):
                ctx.submit_ring(ring, i0 % P, Lb)

            def sub_desc(i0):
                bl = []
                for j in range(Lb):
                    i = (i0 + j) % P
                    bl.append(cg.make_batch(d_pk.addr + i * B * 64, B, d_res.addr + i * B * 8,
                                            fwd_idx=(d_fwd.addr + i * B * 4) if compact else None,
                                            fwd_count=(d_cnt.addr + i * 4) if compact else None))
                ctx.submit(bl)
            sub = sub_ring if is_ring else sub_desc
            for w in range(3):
                sub(w * Lb)
            ctx.sync()
            ctx.launch_timing(True)
            for k in range(args.launches):
                sub(k * Lb)
            ctx.sync()
            ms, nl = ctx.launch_timing_read(reset=True)
            ctx.launch_timing(False)
            ctx.timer_start()
            for k in range(args.launches):
                sub(k * Lb)
            wall = ctx.timer_stop()
            res[n].append((ms, wall / args.launches))
    print(f"{'variant':22s} {'kern_us':>9s} {'GB/s':>8s} {'frac':>6s} {'Mpkt/s(stream)':>15s}")
    for n in names:
        stages, flags, Lb, compact, *_ = variants[n]
        k = np.median([a for a, _ in res[n]])
        w = np.median([b for _, b in res[n]])
        gbs = 72 * B * Lb / (k * 1e-3) / 1e9
        print(f"{n:22s} {k * 1e3:9.1f} {gbs:8.1f} {gbs / 8000:6.3f} {B * Lb / (w * 1e-3) / 1e6:15.1f}")


if __name__ == "__main__":
    main()
