#!/usr/bin/env python3
"""Per-launch HBM traffic of the pipeline kernel from rocprofv3 PMC passes.

Method (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): FETCH_SIZE
and WRITE_SIZE are collected in separate --pmc passes (they do not fit one
pass); both are in KiB per dispatch. On gfx950 FETCH_SIZE under-counts wide
streaming reads by 2x and other widths are uncalibrated, so the read factor
is calibrated here on tools/membench, whose kernels read a known byte count
with the pipeline's exact access pattern (kA: dword@12 + dwordx3@24 per
64-byte slot) and with dwordx4 streaming (kD).

usage: pmc_traffic.py <fetch_bench.csv> <write_bench.csv> <fetch_mb.csv> <write_mb.csv> <out.json>

Every L2 read request to the fabric on gfx950 is 128 bytes, and FETCH_SIZE
tallies each at 64 B: a streaming read makes one request per 128 B
(tools/membench kA: 2,621,805 TCC_EA0_RDREQ for 320 MiB), and an isolated
random dword probe one request (tools/probebench: 0.94-1.00 per probe; two
dword loads into the two 64-byte halves of one line, issued together, merge
into one request). So the calibrated factor 2 applies to the probe share of
the traffic as well (profiles/r03/calib/).
"""
import collections
import csv
import json
import statistics
import sys

MB_PKTS = 5 << 20           # tools/membench: 5 Mi packets of 64 B
MB_SLICE = 1 << 20          # its 1 Mi-packet slice runs


def load(path):
    """{kernel: [(grid, value)]}; path#RDREQ / path#DRAM pick one counter of
    a two-counter pass (TCC_EA0_RDREQ_sum / TCC_EA0_RDREQ_DRAM_sum)."""
    path, _, which = path.partition("#")
    want = {"RDREQ": "TCC_EA0_RDREQ_sum", "DRAM": "TCC_EA0_RDREQ_DRAM_sum"}.get(which)
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if want and r["Counter_Name"] != want:
            continue
        d[r["Kernel_Name"]].append((int(r["Grid_Size"]), float(r["Counter_Value"])))
    return d


def main():
    fb, wb, fm, wm, out = sys.argv[1:6]
    fetch_mb, write_mb = load(fm), load(wm)
    # calibration on kA<4> (whole 320 MiB: 5 Mi packets) and kD (dwordx4)
    cal = {}
    for name, vals in fetch_mb.items():
        if name.startswith("void kA<4>"):
            cal["kA_strided_read_factor"] = (MB_PKTS * 64 / 1024) / statistics.median(v for _, v in vals)
        if name.startswith("kD("):
            cal["kD_stream_read_factor"] = (MB_PKTS * 64 / 1024) / statistics.median(v for _, v in vals)
    for name, vals in write_mb.items():
        if name.startswith("void kA<4>"):
            cal["kA_dword_write_factor"] = (MB_PKTS * 4 / 1024) / statistics.median(v for _, v in vals)
    rf = cal["kA_strided_read_factor"]
    wf = cal["kA_dword_write_factor"]
    fb_, wb_ = load(fb), load(wb)
    # one group per (kernel, grid size): the bench's main launches, its
    # single-batch latency launches and any partial launch are told apart by
    # their grids; the main launches are the group with the most bytes
    res = {}
    for name in fb_:
        if "cop_pipeline" not in name and "cop_hit_count" not in name:
            continue
        for grid in sorted({g for g, _ in fb_[name]}):
            fv = [v for g, v in fb_[name] if g == grid]
            wv = [v for g, v in wb_.get(name, []) if g == grid] or [0.0]
            f = statistics.median(fv)
            w = statistics.median(wv)
            res[f"{name} grid={grid}"] = {
                "dispatches": len(fv), "fetch_kib_raw": f, "write_kib_raw": w, "total_fetch_kib": sum(fv),
                "read_bytes": f * 1024 * rf, "write_bytes": w * 1024 * wf,
                "hbm_bytes_per_launch": f * 1024 * rf + w * 1024 * wf}
    # the poll-mode kernel (one dispatch per launch, serving many batches):
    # its total traffic, for bytes per packet over the packets it served
    pmd = {}
    for name in fb_:
        if "cop_pmd" not in name:
            continue
        fv = [v for _, v in fb_[name]]
        wv = [v for _, v in wb_.get(name, [])] or [0.0]
        pmd[name] = {"dispatches": len(fv), "read_bytes_total": sum(fv) * 1024 * rf,
                     "write_bytes_total": sum(wv) * 1024 * wf}
    main_k = max((k for k in res if "cop_pipeline" in k), key=lambda k: res[k]["total_fetch_kib"])
    doc = {"kernel": main_k, "hbm_bytes_per_launch": res[main_k]["hbm_bytes_per_launch"],
           "read_bytes_per_launch": res[main_k]["read_bytes"], "write_bytes_per_launch": res[main_k]["write_bytes"],
           "calibration": cal, "kernels": res, "pmd": pmd,
           # binned per-rule counters: the count kernel after each launch
           # (the group dispatched as often as the main launches)
           "hit_count": max(({"kernel": k, **v} for k, v in res.items() if "cop_hit_count" in k),
                            key=lambda d: (d["dispatches"] == res[main_k]["dispatches"], d["total_fetch_kib"]),
                            default=None),
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; KiB per dispatch; "
                     "read factor calibrated on tools/membench kA (same access pattern, known bytes)"}
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps({k: doc[k] for k in ("kernel", "hbm_bytes_per_launch", "calibration")}, indent=1))


if __name__ == "__main__":
    main()
