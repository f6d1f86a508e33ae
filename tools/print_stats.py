#!/usr/bin/env python3
"""Live telemetry demo: print_stats (switch.c:33-90) over a running GPU
pipeline. The device processes ring launches back to back; every
PRINT_DELAY seconds (switch.h:23) the host takes cop_counters_snapshot
with reset (a read-and-zero that runs concurrently with the launches) and
prints the reference's two tables: per-port packet statistics and per-NF
coprocessor_stats, plus the interval's rate. At the end the snapshots'
sum is checked against the exact number of packets submitted.

usage: python tools/print_stats.py [--seconds 6] [--delay 2]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ghost-dataplane_amd"))
import copgpu as cg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--delay", type=float, default=2.0)
    args = ap.parse_args()
    P = 5
    rules = cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)
    ctx = cg.Context(stages=cg.STAGE_PARSE | cg.STAGE_FW, flags=cg.CFG_PORT_STATS | cg.CFG_DEMUX_PORTS,
                     n_streams=2)
    ctx.set_fw_table(cg.LpmTable(rules, 1024, 24))
    B, NS = 65536, 64
    dp = ctx.alloc(NS * B * 64)
    for i in range(0, NS, 16):
        dp.upload(cg.gen_trace(0x5EED0F00 + i, 16 * B, rules), i * B * 64)
    dr = ctx.alloc(NS * B * 8)
    df = ctx.alloc(NS * B * P * 4)
    dc = ctx.alloc(NS * P * 4)
    ring = cg.make_ring(dp, NS, B, dr, B * 64, fwd_idx=df, fwd_count=dc, fwd_slot=B * P)
    ctx.snapshot(reset=True, ports=P)
    submitted = 0
    totals = 0
    t_start = t_last = time.time()
    while time.time() - t_start < args.seconds:
        for _ in range(4):
            ctx.submit_ring(ring, 0, NS)
            submitted += NS * B
        now = time.time()
        if now - t_last >= args.delay:
            # taken while the launches just submitted are running
            c, ps = ctx.snapshot(reset=True, ports=P)
            totals += c["rx"]
            dt = now - t_last
            t_last = now
            print("\x1b[2J\x1b[1;1H" if sys.stdout.isatty() else "", end="")
            print("\n**Coprocessor (vport) statistics**   interval %.2f s, %.1f Mpkt/s" % (dt, c["rx"] / dt / 1e6))
            print("======  ============  ============  ============  ============")
            print(" NF      rx_packets    rx_dropped     tx_packets    tx_dropped")
            print("------  ------------  ------------  ------------  ------------")
            for q, st in enumerate(ps):
                print("%7d %13d %13d %13d %13d" % (q, st["rx_packets"], st["rx_dropped"], st["tx_packets"],
                                                  st["tx_dropped"]))
            print("======  ============  ============  ============  ============")
            print(" parse_err %d   no_port %d   fw drops %d   not_ipv4 %d" % (c["parse_err"], c["no_port"],
                                                                          c["pkt_drop"], c["pkt_not_ipv4"]),
                  flush=True)
        wait_idle(ctx)      # throttle the producer
    ctx.sync()
    c, _ = ctx.snapshot(reset=True, ports=P)
    totals += c["rx"]
    print(f"\nsubmitted {submitted} packets, snapshots summed to {totals}: "
          f"{'exact' if totals == submitted else 'MISMATCH'}")
    ctx.close()
    sys.exit(0 if totals == submitted else 1)


def wait_idle(ctx):
    while cg.lib().cop_poll(ctx.handle) == -11:   # -EAGAIN: launches still in flight
        time.sleep(0.0002)


if __name__ == "__main__":
    main()
