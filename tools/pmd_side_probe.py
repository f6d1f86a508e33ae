#!/usr/bin/env python3
"""Which side kernels complete beside a running poll-mode kernel, and how
fast (the round-3 config-5 stall: cop_hit_count beside cop_pmd). One case
per process (fresh streams and queues):

  rules N   per-rule counters on, N firewall rules (N > 8192: DIR-24-8, the
            EXT kernel with binned hits, 4 workers per CU)
Prints, for each call made while the kernel idles with posted work done,
its host wall time; a call that waits for the kernel's idle exit takes
about $COP_PMD_IDLE_MS.
usage: pmd_side_probe.py <rules> [--bins 0|1]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ghost-dataplane_amd"))
import copgpu as cg  # noqa: E402


def main():
    n_rules = int(sys.argv[1])
    S, F = cg.STAGE_PARSE, cg.STAGE_FW
    rules = cg.gen_rules(0x5EED1077, n_rules, cg.GEN_FW, 20 if n_rules <= 1000 else 0)
    ctx = cg.Context(stages=S | F, flags=cg.CFG_SEG_LISTS | cg.CFG_RULE_COUNTERS, max_batch=65536)
    if n_rules <= 1000:
        ctx.set_fw_table(cg.LpmTable(rules, 1024, 24, True))
    else:
        ctx.set_fw_table(cg.LpmTable(rules, n_rules, 1 << 16, False))
    B, P = 65536, 8
    pk = cg.gen_trace(0x5EED5E30, B * P, rules)
    dp = ctx.alloc(pk.nbytes)
    dp.upload(pk)
    dr, df, dc = ctx.alloc(B * P * 8), ctx.alloc(B * P * 4), ctx.alloc(P * 256 * 4)
    ring = cg.make_ring(dp, P, B, dr, B * 64, fwd_idx=df, fwd_slot=B, fwd_count=dc)
    out = {"rules": n_rules, "env": {k: os.environ[k] for k in os.environ if k.startswith(("COP_", "GPU_MAX"))}}
    m = ctx.pmd_start(ring)
    out["pmd"] = m.info()
    t = []
    for what in ("snapshot", "rule_counters", "snapshot", "rule_counters", "counters_reset"):
        m.post(2)
        m.wait()
        t0 = time.perf_counter()
        if what == "snapshot":
            ctx.snapshot(reset=True)
        elif what == "rule_counters":
            ctx.rule_counters(reset=True)
        else:
            ctx.counters(reset=True)
        t.append((what, round((time.perf_counter() - t0) * 1e3, 3), m.info()["launches"]))
    out["calls_ms_launches"] = t
    m.stop()
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
