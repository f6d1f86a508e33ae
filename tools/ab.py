#!/usr/bin/env python3
"""Interleaved A/B of kernel variants in one process (not the contract
bench): every variant is a context created under its own environment
($COP_KERNEL, $COP_PPT, $COP_DBG, ...); rounds rotate over the variants so
box-to-box and drift effects cancel, and the median per-launch kernel time
(HIP events on the launch stream) is reported.

usage: python tools/ab.py [--workload fw1k|fw_lpm|imix|fw_lpm_1m] [--rounds 7]
           [--per-launch 384] [--launches 8] [--rule-counters] VARIANT...
VARIANT = name[:KEY=VAL[,KEY=VAL...]][/nocompact]
e.g.  python tools/ab.py base stage0:COP_STAGE_LISTS=0 p8:COP_PPT=8
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ghost-dataplane_amd"))
import copgpu as cg  # noqa: E402

S, F, L = cg.STAGE_PARSE, cg.STAGE_FW, cg.STAGE_LPM


def parse_variant(spec):
    compact = True
    if spec.endswith("/nocompact"):
        compact = False
        spec = spec[: -len("/nocompact")]
    name, _, envs = spec.partition(":")
    env = dict(kv.split("=", 1) for kv in envs.split(",") if kv)
    return name, env, compact


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="fw1k", choices=["fw1k", "fw_lpm", "imix", "fw_lpm_1m"])
    ap.add_argument("--rule-counters", action="store_true", help="per-rule hit counters (COP_CFG_RULE_COUNTERS)")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--per-launch", type=int, default=384)
    ap.add_argument("--launches", type=int, default=8)
    ap.add_argument("variants", nargs="+")
    args = ap.parse_args()

    big = args.workload == "fw_lpm_1m"   # BASELINE configs[4]: 1M ACL rules + 1M prefixes, 256k batches
    if big:
        fw_rules = cg.gen_rules(0x5EED1005, 1000000, cg.GEN_FW, 0)
        routes = cg.gen_rules(0x5EED2005, 1000000, cg.GEN_ROUTES, 0)
        fw_tab = cg.LpmTable(fw_rules, 1000000, 1 << 20, False)
        rt_tab = cg.LpmTable(routes, 1 << 20, 1 << 20, False)
    else:
        fw_rules = cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)
        routes = cg.gen_rules(0x5EED2004, 100000, cg.GEN_ROUTES, 0) if args.workload != "fw1k" else None
        fw_tab = cg.LpmTable(fw_rules, 1024, 24, True)
        rt_tab = cg.LpmTable(routes, 1 << 20, 1 << 16, False) if routes is not None else None
    stages = S | F | (L if routes is not None else 0)
    B = 262144 if big else 65536
    flags = cg.CFG_RULE_COUNTERS if args.rule_counters else 0
    Lb = args.per_launch
    variants = [parse_variant(v) for v in args.variants]
    ctxs = []
    for name, env, compact in variants:
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        c = cg.Context(stages=stages, max_batch=B, n_streams=1, flags=flags)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        c.set_fw_table(fw_tab)
        if rt_tab is not None:
            c.set_route_lpm(rt_tab)
        ctxs.append(c)
    base = ctxs[0]
    if args.workload == "imix":
        slab, offs = cg.gen_imix(0x5EED0003, B, fw_rules, routes)
        per = slab.nbytes + offs.nbytes
        P = Lb
        d_pk = base.alloc(P * per)
        for i in range(P):
            d_pk.upload(slab, i * per)
            d_pk.upload(offs, i * per + slab.nbytes)
    else:
        per = B * 64
        P = max(Lb, (400 << 20) // per)
        d_pk = base.alloc(P * per)
        for i in range(0, P, 16):
            k = min(16, P - i)
            d_pk.upload(cg.gen_trace(0x5EED0002 + i, k * B, fw_rules, routes), i * per)
    d_res = base.alloc(P * B * 8)
    d_fwd = base.alloc(P * B * 4)
    d_cnt = base.alloc(P * 4)
    res = {v[0]: [] for v in variants}
    for r in range(args.rounds):
        for (name, env, compact), ctx in zip(variants, ctxs):
            if args.workload == "imix":
                ring = cg.make_ring(d_pk, P, B, d_res, per, offsets=d_pk.addr + slab.nbytes,
                                    offsets_slot_words=per // 4, fwd_idx=d_fwd if compact else None,
                                    fwd_count=d_cnt if compact else None)
            else:
                ring = cg.make_ring(d_pk, P, B, d_res, per, stride=64, fwd_idx=d_fwd if compact else None,
                                    fwd_count=d_cnt if compact else None)
            ctx.submit_ring(ring, 0, Lb)
            ctx.sync()
            ctx.launch_timing(True)
            for k in range(args.launches):
                ctx.submit_ring(ring, (k * Lb) % P, Lb)
            ctx.sync()
            ms, _ = ctx.launch_timing_read(reset=True)
            ctx.launch_timing(False)
            res[name].append(ms)
    alg = (76 if args.workload == "imix" else 72) * B * Lb
    print(f"workload {args.workload}, {Lb} x {B} per launch, {args.rounds} rounds x {args.launches} launches")
    print(f"{'variant':28s} {'median_us':>10s} {'min_us':>8s} {'GB/s(72B)':>10s} {'Gpkt/s':>8s}")
    for name, _, _ in variants:
        m = float(np.median(res[name]))
        print(f"{name:28s} {m * 1e3:10.1f} {min(res[name]) * 1e3:8.1f} {alg / (m * 1e-3) / 1e9:10.1f} "
              f"{B * Lb / (m * 1e-3) / 1e9:8.2f}", flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
