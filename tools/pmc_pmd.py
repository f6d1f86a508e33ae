#!/usr/bin/env python3
"""PMC traffic of the poll-mode kernel per posted batch.

A persistent kernel's counters cover its whole lifetime, idle polling
included, so the bench's own runs (many posts, idle spells between them)
cannot be divided by a batch count. This tool gives the kernel a lifetime
that serves exactly K posted batches: start, one post of K batches, wait,
stop at once (no idle spell). rocprofv3 --pmc then reports the lifetime's
FETCH_SIZE / WRITE_SIZE (separate passes); divided by K they are the
traffic per batch (the start-up census and table staging included, a few
KiB).

  run      [--workload fw1k|fw_lpm|fw_lpm_imix|fw_lpm_1m] [--batches K] [--lists seg|dense]
           the workload, meant to run under rocprofv3 --pmc
  reduce   <fetch.csv> <write.csv> <fetch_mb.csv> <write_mb.csv> <out.json> --batches K [--pkts-per-batch B]
           bytes per batch, read factor calibrated on tools/membench as in
           tools/pmc_traffic.py (same method)
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ghost-dataplane_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def run(a):
    """Build the workload exactly as bench.py's measure() does (same seeds,
    tables, context flags, batch layout and slot declaration), then one
    kernel lifetime that serves exactly K posted batches."""
    import copgpu as cg
    import copdist
    sys.path.insert(0, ROOT)
    from bench import WORKLOADS
    W = WORKLOADS[a.workload]
    B, cid = W["batch"], W["cid"]
    rc_on = bool(W.get("rule_counters"))
    fw_rules = cg.gen_rules(0x5EED1000 + cid, W["fw"], cg.GEN_FW, 20 if W["fw"] <= 1000 else 0)
    routes = cg.gen_rules(0x5EED2000 + cid, W["routes"], cg.GEN_ROUTES, 0) if W["routes"] else None
    seg = a.lists == "seg"
    ctx = cg.Context(device=0, stages=W["stages"], max_batch=B, max_batches=32,
                     flags=(cg.CFG_SEG_LISTS if seg else 0) | (cg.CFG_RULE_COUNTERS if rc_on else 0))
    if W["fw"] <= 1024:
        ctx.set_fw_table(cg.LpmTable(fw_rules, 1024, 24, True))
    else:
        ctx.set_fw_table(cg.LpmTable(fw_rules, W["fw"], 1 << 20, False))
    if routes is not None:
        ctx.set_route_lpm(cg.LpmTable(routes, max(W["routes"], 1), 1 << 20, False))
    P = a.batches
    if W["imix"]:
        slab, offs = cg.gen_imix(copdist.shard_seed(0x5EED0000 + cid, 0), B, fw_rules, routes)
        per_batch = slab.nbytes + offs.nbytes
    else:
        per_batch = B * 64
    dp = ctx.alloc(P * per_batch)
    if W["imix"]:
        for i in range(P):
            dp.upload(slab, i * per_batch)
            dp.upload(offs, i * per_batch + slab.nbytes)
    else:
        for i in range(0, P, 16):
            k = min(16, P - i)
            dp.upload(cg.gen_trace(copdist.shard_seed(0x5EED0000 + cid, 0, i), k * B, fw_rules, routes),
                      i * per_batch)
    dr = ctx.alloc(P * B * 8)
    df = ctx.alloc(P * B * 4)
    dc = ctx.alloc(P * ((B + cg.SEG_PKTS - 1) // cg.SEG_PKTS if seg else 1) * 4 + 16)
    if W["imix"]:
        ring = cg.make_ring(dp, P, B, dr, per_batch, offsets=dp.addr + slab.nbytes,
                            offsets_slot_words=per_batch // 4, fwd_idx=df, fwd_count=dc)
    else:
        ring = cg.make_ring(dp, P, B, dr, per_batch, stride=64, fwd_idx=df, fwd_count=dc)
    # bench.py's pool is written once before the kernel starts (--slots static)
    m = ctx.pmd_start(ring, cg.PMD_STATIC_SLOTS)
    m.post(P)
    m.wait()
    info = m.info()
    m.stop()
    c = ctx.counters()
    print(json.dumps({"workload": a.workload, "batches": P, "pkts_per_batch": B, "rx": int(c["rx"]),
                      "forward": int(c["forward"]), "ok": int(c["rx"]) == P * B,
                      "workers": info["workers"], "packets_per_tile": info["packets_per_tile"]}))
    ctx.close()


def reduce(a):
    from pmc_traffic import load, MB_PKTS
    fb, wb, fm, wm = load(a.fetch), load(a.write), load(a.fetch_mb), load(a.write_mb)
    rf = wf = None
    for name, vals in fm.items():
        if name.startswith("void kA<4>"):
            rf = (MB_PKTS * 64 / 1024) / statistics.median(v for _, v in vals)
    for name, vals in wm.items():
        if name.startswith("void kA<4>"):
            wf = (MB_PKTS * 4 / 1024) / statistics.median(v for _, v in vals)
    pmd = [k for k in fb if "cop_pmd" in k]
    assert len(pmd) == 1, pmd
    name = pmd[0]
    f = sum(v for _, v in fb[name])
    w = sum(v for _, v in wb.get(name, []))
    rd, wr = f * 1024 * rf, w * 1024 * wf
    K, B = a.batches, a.pkts_per_batch
    doc = {"kernel": name, "batches": K, "pkts_per_batch": B, "dispatches": len(fb[name]),
           "read_bytes_total": rd, "write_bytes_total": wr,
           "hbm_bytes_per_batch": (rd + wr) / K, "read_bytes_per_pkt": rd / K / B, "write_bytes_per_pkt": wr / K / B,
           "calibration": {"kA_strided_read_factor": rf, "kA_dword_write_factor": wf},
           "method": "one poll-mode kernel lifetime serving exactly K posted batches, then stopped at once "
                     "(tools/pmc_pmd.py run); rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; read "
                     "factor calibrated on tools/membench kA"}
    json.dump(doc, open(a.out, "w"), indent=1)
    print(json.dumps(doc, indent=1))


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--workload", default="fw1k", choices=("fw1k", "fw_lpm", "fw_lpm_imix", "fw_lpm_1m"))
    r.add_argument("--batches", type=int, default=1024)
    r.add_argument("--lists", default="seg", choices=("seg", "dense"))
    d = sub.add_parser("reduce")
    for k in ("fetch", "write", "fetch_mb", "write_mb", "out"):
        d.add_argument(k)
    d.add_argument("--batches", type=int, required=True)
    d.add_argument("--pkts-per-batch", type=int, default=65536)
    a = ap.parse_args()
    run(a) if a.cmd == "run" else reduce(a)


if __name__ == "__main__":
    main()
