#!/usr/bin/env python3
"""Print the key fields of bench.py JSON lines in the given logs (diagnostic)."""
import json
import sys

for f in sys.argv[1:]:
    for line in open(f):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        r = d["roofline"]
        rl = d.get("roofline_launch", r)
        bc = rl.get("box_ceiling") or {}
        print(f"{f}: {d['config']['workload']} {d['config'].get('engine')} value {d['value']:.1f} runs_us "
              f"{[round(x * 1e3, 1) for x in d['runs_ms']]} frac {r['frac']} (traffic x{r.get('traffic_per_algorithmic')}) "
              f"launch frac {rl['frac']} kernel_ms {rl['kernel_ms_per_launch']} ceiling {bc.get('achieved')} "
              f"({bc.get('best_pattern')})")
        if "pmd" in d:
            p = d["pmd"]
            print(f"   pmd steady {p['steady_mpkt_s']:.0f} ({p['steady_frac']}), 1-batch post {p['single_batch_post_to_done_us_median']} us, "
                  f"one-batch posts {p['one_batch_posts']['mpkt_s']:.0f}")
        if "single_batch_latency" in d:
            print(f"   single batch {d['single_batch_latency']}")
        for k in ("secondary", "counter_reduce", "counter_allreduce_check"):
            if k in d:
                print(f"   {k}: {json.dumps(d[k])[:400]}")
