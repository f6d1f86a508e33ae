#!/usr/bin/env python3
"""Generate the committed fixtures (tests/golden/*.npz).

Only g1 holds a REFERENCE fixture: the reference's own rules.json
(reference_rules.json: both rules accept, so every IPv4 packet that reaches
the coprocessor is forwarded). g2-g6 are ORACLE REGRESSION VECTORS, not
reference goldens: the reference ships no vectors for this path (SURVEY.md
§4) and cannot be built here (DPDK absent), so they are produced by the
oracle's C restatement (oracle/cop_oracle.c) on small seeded inputs. They
pin the product and the oracle against later changes of either; parity with
the reference's own outputs stays unpinned beyond g1.
Each .npz holds inputs (rules, packets, routing table, stage mask) and the
expected outputs (8-byte result records, ordered forward list, counters).

Run from the repo root:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "ghost-dataplane_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import copgpu as cg  # noqa: E402  (generator only: trace/rule synthesis)
import oracle as orc  # noqa: E402

S, F, L = cg.STAGE_PARSE, cg.STAGE_FW, cg.STAGE_LPM


def rules_arrays(r):
    return np.ascontiguousarray(r["ip"]), np.ascontiguousarray(r["depth"]), np.ascontiguousarray(r["next_hop"])


def emit(name, pkts, n, stages, fw_rules, routes, fw_cfg=(1024, 24, True), rt=None, offsets=None):
    fw = orc.OracleLpm(fw_cfg[0], fw_cfg[1])
    if fw_rules is not None and len(fw_rules):
        fw.setup(*rules_arrays(fw_rules), stop_at_error=fw_cfg[2])
    route = orc.OracleLpm(1 << 20, 1 << 16)
    if routes is not None and len(routes):
        route.setup(*rules_arrays(routes), stop_at_error=False)
    if rt is None:
        rt = orc.route_table_default(5)
    res, fwd, cnt = orc.process(pkts, n, offsets=offsets, rt=rt, stages=stages, fw=fw, route=route)
    empty = np.zeros(0, dtype=np.uint32)
    np.savez_compressed(
        os.path.join(HERE, name + ".npz"),
        pkts=pkts, n=np.uint32(n), stages=np.uint32(stages), rt=rt,
        offsets=offsets if offsets is not None else empty,
        fw_ip=fw_rules["ip"] if fw_rules is not None else empty,
        fw_depth=fw_rules["depth"] if fw_rules is not None else empty.astype(np.uint8),
        fw_nh=fw_rules["next_hop"] if fw_rules is not None else empty,
        fw_cfg=np.array(fw_cfg, dtype=np.uint32),
        rt_ip=routes["ip"] if routes is not None else empty,
        rt_depth=routes["depth"] if routes is not None else empty.astype(np.uint8),
        rt_nh=routes["next_hop"] if routes is not None else empty,
        res=res.view(np.uint8).reshape(-1, 8), fwd=fwd,
        counters=np.array([cnt[k] for k in sorted(cnt)], dtype=np.uint64),
        counter_names=np.array(sorted(cnt)))
    print(f"{name}: {n} pkts, {len(fwd)} forwarded")


def main():
    # 1. the reference's own fixture: rules.json (2 accept rules)
    ref = cg.rules_load_json(os.path.join(HERE, "reference_rules.json"))
    pk = cg.gen_trace(0x5EED0001, 2048, None, None)
    emit("g1_reference_rules", pk, 2048, S | F, ref, None)
    # 2. 1k-rule firewall (BASELINE configs[1] shape, small n)
    fw = cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)
    pk = cg.gen_trace(0x5EED0002, 4096, fw, None)
    emit("g2_fw1k", pk, 4096, S | F, fw, None)
    # 3. firewall + route LPM (5k prefixes to keep the fixture small)
    routes = cg.gen_rules(0x5EED2003, 5000, cg.GEN_ROUTES, 0)
    pk = cg.gen_trace(0x5EED0003, 4096, fw, routes)
    emit("g3_fw_lpm", pk, 4096, S | F | L, fw, routes)
    # 4. edge traffic: bad versions, non-IPv4, unknown dsts, custom routes
    rt = orc.route_table_default(5)
    rt[0x1234] = 7
    rt[0x2000:0x2100] = 3
    opts = cg.trace_opts(pct_bad_version=10, pct_non_ipv4=10, pct_unknown_dst=10)
    pk = cg.gen_trace(0x5EED0077, 3000, fw, None, opts=opts)
    for i in range(0, 3000, 97):
        pk[i * 64 + 32] = 0x12
        pk[i * 64 + 33] = 0x34
    emit("g4_edges", pk, 3000, S | F, fw, None, rt=rt)
    # 5. lpm_setup truncation: 30 /25 parents with number_tbl8s = 24
    ip = [(10 << 24) | (k << 8) | 0x80 for k in range(30)] + [0x0B000000]
    rules = cg.prefixes(ip, [25] * 30 + [8], list(range(1, 31)) + [9])
    pk = cg.gen_trace(0x5EED0300, 2048, rules, None)
    emit("g5_tbl8_exhaustion", pk, 2048, S | F, rules, None)
    # 6. IMIX slab
    slab, offs = cg.gen_imix(0x5EED0003, 1500, fw, routes)
    emit("g6_imix", slab, 1500, S | F | L, fw, routes, offsets=offs)


if __name__ == "__main__":
    main()
