#!/usr/bin/env python3
"""Benchmark: device-resident coprocessor NF pipeline, Mpkt/s (BASELINE.json).

A step = one pass of the pipeline over one batch of synthetic packets that
are already resident in HBM. Default workload = BASELINE configs[1]:
firewall ACL (1k rules), 64 B packets, batch 64k. The timed region rotates
over a pool of distinct batches larger than the 256 MiB Infinity Cache, so
every step reads its packets from HBM.

Multi-GPU: one process per GPU, each with its own context, batches and
tables (the path shards with no data-path collective: weak scaling). A
gloo barrier brackets the timed region and the max elapsed time over ranks
is used. Launched either by python -m torch.distributed.run ... bench.py
--gpus N (RANK/WORLD_SIZE set: WORLD_SIZE must equal --gpus), or as plain
python bench.py --gpus N: the parent then spawns N rank processes with
RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, before anything touches a GPU, and
exits with their status (rank 0 prints the line). Every rank needs its own
GPU: ranks that would share one are refused unless --allow-shared-gpu.

Also reported (rank 0):
  roofline      algorithmic bytes per launch / mean kernel time (HIP events
                on the context's stream around every launch), vs 8 TB/s;
                box_ceiling: what the same box sustains for the same byte mix
                with no classification (tools/ceiling.hip), same pool;
                probe_ceiling / probe_bound: the same box's random-probe rate
                into tables of the pipeline's tbl24 size, and the pipeline's
                LPM probes per second against it (DIR-24-8 workloads);
  secondary     the north-star workload (FW + LPM 100k, 64 B) timed the same
                way in the same run, with its own roofline (fw1k runs);
  cpu_baseline  the oracle's restatement of the reference CPU coprocessor()
                loop (oracle/cop_oracle.c), 1 pinned core, bounded sample.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ghost-dataplane_amd"))

import copdist  # noqa: E402
import copgpu as cg  # noqa: E402

METRIC = "Mpkt/s device-resident coprocessor NF pipeline (64B pkts); HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md)
# counter words ahead of the per-rule ones in the RCCL reduction: the
# COP_COUNTER_SHARDS x 16 counter shards, then as many port-stat shards
SHARD_AND_PORT_WORDS = 2 * 16 * cg.COUNTER_SHARDS
TRAFFIC_DIR = os.path.join(ROOT, "bench_traffic")   # PMC traffic summaries the line quotes (travel with the tree)

S, F, L = cg.STAGE_PARSE, cg.STAGE_FW, cg.STAGE_LPM
# config_id follows BASELINE.json configs[] (1-based); seeds per SURVEY.md §8d
WORKLOADS = {
    "fw1k": dict(cid=2, stages=S | F, fw=1000, routes=0, imix=False, batch=65536, per_launch=1024,
                 desc="firewall ACL 1k rules, 64B pkts, batch 64k (BASELINE configs[1])"),
    "fw_lpm_imix": dict(cid=3, stages=S | F | L, fw=1000, routes=100000, imix=True, batch=65536, per_launch=384,
                        desc="firewall + LPM 100k prefixes, IMIX, batch 64k (BASELINE configs[2])"),
    "fw_lpm": dict(cid=4, stages=S | F | L, fw=1000, routes=100000, imix=False, batch=65536, per_launch=1024,
                   desc="firewall + LPM 100k, 64B pkts, batch 64k per GPU (BASELINE configs[3])"),
    "fw_lpm_1m": dict(cid=5, stages=S | F | L, fw=1000000, routes=1000000, imix=False, batch=262144, per_launch=384,
                      rule_counters=True,
                      desc="1M ACL rules + 1M LPM prefixes, 64B, batch 256k per GPU, per-rule hit "
                           "counters all-reduced over RCCL once per timed region (BASELINE configs[4])"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _ceiling_lib():
    import ctypes

    path = os.path.join(ROOT, "tools", "libceiling.so")
    if not os.path.exists(path):
        log("[bench] tools/libceiling.so not built: no box ceiling")
        return None
    return ctypes.CDLL(path)


def box_ceiling(pkts_addr, n_slots, out_addr):
    """(GB/s, pattern, {pattern: GB/s}) of the 72 B/packet copy mix on this
    box (None if the tool is absent)."""
    import ctypes

    lib = _ceiling_lib()
    if lib is None:
        return None
    fn = lib.ceiling_pattern
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                   ctypes.POINTER(ctypes.c_float)]
    fn.restype = ctypes.c_int
    best, best_name, every = None, None, {}
    # grid-stride copy at 4/8/16 workgroups per CU (and with 4 loads in flight
    # per lane); LDS-DMA rings 2 deep at 2/3 per CU, 4 deep at 1/2, 8 deep at 1
    # (MI355X_MICROARCH.md: float4 copy 6.29 TB/s, nt LDS-DMA streams 6.5-6.8)
    for pattern, mults, name in ((0, (4, 8, 16), "grid-stride"), (4, (2, 4, 8), "grid-stride x4 in flight"),
                                 (1, (2, 3), "lds-dma ring"), (2, (1, 2), "lds-dma ring 4-deep"),
                                 (3, (1,), "lds-dma ring 8-deep")):
        for m in mults:
            ms = ctypes.c_float(0.0)
            if fn(pkts_addr, n_slots, out_addr, pattern, m, 5, ctypes.byref(ms)) == 0 and ms.value > 0:
                every[f"{name} x{m}/CU"] = round(72.0 * n_slots / (ms.value * 1e-3) / 1e9, 1)
                if best is None or ms.value < best:
                    best, best_name = ms.value, f"{name} x{m}/CU"
    if best is None:
        return None
    return 72.0 * n_slots / (best * 1e-3) / 1e9, best_name, every


def probe_ceiling(ctx, tables):
    """Gprobes/s of uniformly random dword loads into `tables` tables of 2^24
    u32 (64 MiB, the pipeline's tbl24 size) on this box, 8 packets per lane
    with all probes in flight (tools/probe_kernels.h), or None."""
    import ctypes

    lib = _ceiling_lib()
    if lib is None:
        return None
    fn = lib.ceiling_probe
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                   ctypes.POINTER(ctypes.c_float)]
    fn.restype = ctypes.c_int
    bufs = [ctx.alloc(64 << 20) for _ in range(2)]
    try:
        for i, b in enumerate(bufs):
            b.fill(0x11 * (i + 1))
        g = ctypes.c_float(0.0)
        rc = fn(bufs[0].addr, bufs[1].addr, 1 << 24, tables, 5, ctypes.byref(g))
        return float(g.value) if rc == 0 else None
    finally:
        for b in bufs:
            b.free()


def spawn_ranks(n: int) -> int:
    """Run this script as n rank processes (one per GPU) and return their
    worst exit status. The parent makes no GPU call: the ranks inherit its
    stdout, where rank 0 prints the JSON line. Every rank is watched at once:
    the first that fails ends the others (they would otherwise sit in a
    gloo rendezvous or barrier until its long timeout)."""
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [None] * n
    bad = None
    while any(rc is None for rc in rcs):
        for r, p_ in enumerate(procs):
            if rcs[r] is None:
                rcs[r] = p_.poll()
                if rcs[r] not in (None, 0) and bad is None:
                    bad = r
        if bad is not None:
            for p_ in procs:
                if p_.poll() is None:
                    p_.terminate()
            for r, p_ in enumerate(procs):
                try:
                    rcs[r] = p_.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p_.kill()
                    rcs[r] = p_.wait()
            break
        time.sleep(0.05)
    failed = [(r, rc) for r, rc in enumerate(rcs) if rc != 0]
    if failed:
        log(f"[bench] ranks failed (rank, exit status): {failed}" + (f"; rank {bad} failed first" if bad is not None
                                                                    else ""))
        return max(abs(rc) for _, rc in failed) or 1
    return 0


def check_devices(args, world, local, ndev):
    """One GPU per rank: refuse --gpus N ranks on fewer GPUs (they would time
    N-way shared GPUs as N GPUs) unless --allow-shared-gpu."""
    if world != args.gpus:
        raise SystemExit(f"[bench] WORLD_SIZE={world} but --gpus {args.gpus}: launch {args.gpus} ranks")
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if local_world > ndev and not args.allow_shared_gpu:
        raise SystemExit(f"[bench] {local_world} ranks on this node but {ndev} GPU(s) visible: each rank needs its "
                         f"own GPU (--allow-shared-gpu to time ranks sharing GPUs anyway)")


def table_probes(fw_tab, rt_tab, sample, imix_offsets, route_form, fw_form="dir"):
    """LPM table probes are not in the algorithmic bytes;
    report them per packet, from a sample batch of the workload (host-side
    restatement of which packets reach each stage). LDS forms issue no
    global-memory probe; DIR-24-8 issues one tbl24 load per packet that
    reaches the stage and a tbl8 load when the entry is extended; the trie
    form 2-4 node loads and a leaf load (L2-resident)."""
    if imix_offsets is not None:
        hdr = np.stack([sample[o:o + 36] for o in imix_offsets[:65536]])
    else:
        hdr = sample.reshape(-1, 64)[:, :36]
    et = (hdr[:, 12].astype(np.uint32) << 8) | hdr[:, 13]
    be = lambda c: ((hdr[:, c].astype(np.uint32) << 24) | (hdr[:, c + 1].astype(np.uint32) << 16)  # noqa: E731
                    | (hdr[:, c + 2].astype(np.uint32) << 8) | hdr[:, c + 3])
    src, dst = be(26), be(30)
    reach = (et == 0x0800) & ((dst & 0xFFFF) > 4)   # stage P: the default routing table's UNKNOWN entries
    n = len(hdr)
    out = {"sample_pkts": int(n), "reach_stage_p": round(float(reach.mean()), 4)}
    for name, tab, key, form in (("fw", fw_tab, src, fw_form), ("route", rt_tab, dst, route_form)):
        if tab is None:
            continue
        if len(tab.intervals()[0]) <= 8192:
            out[name] = {"form": "lds-intervals", "global_probes_per_pkt": 0.0}
            continue
        if form == "trie":
            out[name] = {"form": "trie (LDS top level, L2 nodes)", "global_probes_per_pkt": None}
            continue
        if form == "bkt":
            # one 8-byte index load + one 16-byte pair load per reaching
            # packet, plus the wide-bucket rounds (two 16-byte loads each)
            _, _, info = tab.bkt_probe(key[reach], 1 if name == "fw" else 0, int(os.environ.get("COP_BKT_XBITS", "1")))
            out[name] = {"form": "bkt (bucketed intervals, L2)", "ib": info["ib"],
                         "l2_loads_per_pkt": round((2 * float(reach.sum()) + 2 * info["rounds"]) / n, 4),
                         "wide_lookups_per_pkt": round(info["lifted"] / n, 4),
                         "table_bytes": ((1 << info["ib"]) + 1) * 4 + (info["m"] + 4) * 8}
            continue
        t24, _ = tab.dir24()
        e = t24[key[reach] >> 8]
        ext = ((e & 0x03000000) == 0x03000000).sum()
        out[name] = {"form": "dir24-8", "tbl24_per_pkt": round(float(reach.sum()) / n, 4),
                     "tbl8_per_pkt": round(float(ext) / n, 4)}
    return out


def dir_probes_per_pkt(probes) -> tuple:
    """(random DIR-24-8 probes per packet, tbl24 tables probed)."""
    total, tables = 0.0, 0
    for k in ("fw", "route"):
        d = probes.get(k) or {}
        if d.get("form") == "dir24-8":
            total += d["tbl24_per_pkt"] + d["tbl8_per_pkt"]
            tables += 1
    return total, tables


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def measure(args, name, rank, world, dev, group, gate, primary):
    """Time `args.steps` steps of workload `name` (+ its kernel roofline);
    returns (result dict, context). The caller closes the context. Every
    timed run opens through the start gate (all ranks' windows at once,
    CLOCK_MONOTONIC stamps: copdist.StartGate)."""
    W = WORKLOADS[name]
    B = W["batch"]
    Lb = max(1, (args.per_launch if primary else 0) or W["per_launch"])
    cid = W["cid"]
    t0 = time.time()
    fw_rules = cg.gen_rules(0x5EED1000 + cid, W["fw"], cg.GEN_FW, 20 if W["fw"] <= 1000 else 0)
    routes = cg.gen_rules(0x5EED2000 + cid, W["routes"], cg.GEN_ROUTES, 0) if W["routes"] else None
    if W["fw"] <= 1024:
        fw_tab = cg.LpmTable(fw_rules, 1024, 24, True)                  # lpm_setup's own limits
    else:
        fw_tab = cg.LpmTable(fw_rules, W["fw"], 1 << 20, False)
    rc_on = bool(W.get("rule_counters")) and not args.no_rule_counters
    engine = args.engine
    if engine == "auto":
        # the poll-mode kernel for short runs (no per-launch ramp), one-shot
        # launches of up to 1024 batches for long runs (they stream faster)
        engine = "launch" if args.steps >= 1024 else "pmd"
    stages = args.stages if (args.stages and primary) else W["stages"]
    seg = args.lists == "seg"
    ctx = cg.Context(device=dev, stages=stages, max_batch=B, max_batches=32, n_streams=args.streams,
                     flags=(cg.CFG_RULE_COUNTERS if rc_on else 0) | (cg.CFG_NO_COMPACT if args.no_compact else 0)
                     | {"dir": 0, "trie": cg.CFG_LPM_TRIE, "bkt": cg.CFG_LPM_BKT}[args.route_form]
                     | (cg.CFG_FW_BKT if args.fw_form == "bkt" else 0)
                     | (cg.CFG_SEG_LISTS if seg else 0))
    ctx.set_fw_table(fw_tab)
    coll = None
    if rc_on:
        # RCCL communicator over the GPUs of the job (xGMI); id from rank 0 over gloo
        try:
            uid = group.broadcast_bytes(cg.coll_unique_id() if rank == 0 else None)
            ctx.coll_init(uid, rank, world)
            coll = "ok"
        except Exception as e:  # noqa: BLE001 (reported per rank; the reduce is then skipped)
            coll = f"error: {str(e)[:120]}"
        # the all-reduce is collective: every rank runs it or none does (a
        # rank that failed its init would leave the others in RCCL forever)
        if group.min(1.0 if coll == "ok" else 0.0) < 1.0 and coll == "ok":
            coll = "skipped: another rank's RCCL init failed"
    rt_tab = None
    if routes is not None:
        rt_tab = cg.LpmTable(routes, max(W["routes"], 1), 1 << 20, False)
        ctx.set_route_lpm(rt_tab)
    log(f"[rank {rank}] {name}: tables ready in {time.time() - t0:.1f}s on device {dev}")

    # ---- input pool: distinct batches, > Infinity Cache ----
    pool_bytes = (args.pool_mib << 20) if primary else 0
    t0 = time.time()
    if W["imix"]:
        slab, offs = cg.gen_imix(copdist.shard_seed(0x5EED0000 + cid, rank), B, fw_rules, routes)
        per_batch = slab.nbytes + offs.nbytes
    else:
        per_batch = B * 64
    if not pool_bytes:
        # > 256 MiB Infinity Cache, and at least one full launch of distinct batches
        pool_bytes = max(400 << 20, per_batch * Lb)
    P = max(2, pool_bytes // per_batch)
    d_pkts = ctx.alloc(P * per_batch)
    # outputs: HBM, or (A/B) uncached / fine-grained HBM (--out-mem)
    of = {"device": 0, "uncached": cg.ALLOC_UNCACHED, "fine": cg.ALLOC_FINEGRAINED}[args.out_mem]
    d_res = ctx.alloc(P * B * 8, of)
    d_fwd = ctx.alloc(P * B * 4, of)
    n_seg = (B + cg.SEG_PKTS - 1) // cg.SEG_PKTS
    cnt_per_slot = n_seg if seg else 1   # one count per segment, or per batch
    d_cnt = ctx.alloc(P * cnt_per_slot * 4 + 16, of)
    if W["imix"]:
        # same packet mix in every batch slot, distinct addresses
        for i in range(P):
            d_pkts.upload(slab, i * per_batch)
            d_pkts.upload(offs, i * per_batch + slab.nbytes)
    else:
        chunk = 16
        for i in range(0, P, chunk):
            k = min(chunk, P - i)
            pk = cg.gen_trace(copdist.shard_seed(0x5EED0000 + cid, rank, i), k * B, fw_rules, routes)
            d_pkts.upload(pk, i * per_batch)
    log(f"[rank {rank}] {name}: pool {P} batches x {B} pkts ({P * per_batch / 2**20:.0f} MiB) in "
        f"{time.time() - t0:.1f}s")

    # the pool is a batch ring in HBM: one launch = Lb consecutive slots
    Lb = min(Lb, P)
    if W["imix"]:
        ring = cg.make_ring(d_pkts, P, B, d_res, per_batch, offsets=d_pkts.addr + slab.nbytes,
                            offsets_slot_words=per_batch // 4, fwd_idx=d_fwd, fwd_count=d_cnt)
    else:
        ring = cg.make_ring(d_pkts, P, B, d_res, per_batch, stride=64, fwd_idx=d_fwd, fwd_count=d_cnt)

    pmd = None

    # the pool is written once before the kernel starts and never again:
    # declared (COP_PMD_STATIC_SLOTS), so every tile takes plain loads
    # (--slots reuse: the default, coherent loads once the ring wraps;
    # always: coherent loads on every tile)
    pmd_flags = {"static": cg.PMD_STATIC_SLOTS, "reuse": 0, "always": cg.PMD_SYS_ACQUIRE}[args.slots]

    def pmd_on():
        nonlocal pmd
        if engine == "pmd" and pmd is None:
            pmd = ctx.pmd_start(ring, pmd_flags)

    def pmd_off():
        nonlocal pmd
        if pmd is not None:
            pmd.stop()
            pmd = None

    def run_steps(first, count):
        """Steps first .. first+count-1: batch s sits in ring slot s % P.
        Poll mode: returns the library's own (post, done) CLOCK_MONOTONIC
        stamps of the call (cop_pmd_run_timed)."""
        if pmd is not None:
            # the poll-mode kernel's batch sequence is the step sequence:
            # one call posts them (a quarter ring per post, so the ring never
            # drains) and waits for the last
            return pmd.run_timed(count)
        s = first
        while s < first + count:
            k = min(Lb, first + count - s)
            ctx.submit_ring(ring, s % P, k)
            s += k
        return None

    def sync_all():
        if pmd is None:
            ctx.sync()
        # (poll mode: run_steps waited for every posted batch already)

    # ---- warmup, then exactly K timed steps, `repeats` times; the value is
    # the median run (median of 5 runs) ----
    pmd_on()
    run_steps(0, args.warmup)
    runs, own_runs, reduce_runs, reduce_ms, windows, harness = [], [], [], [], [], []
    for r in range(max(1, args.repeats)):
        pmd_on()
        sync_all()
        group.barrier()
        sync_all()
        t0 = gate.open()   # every rank's window opens here at once
        stamps = run_steps(args.warmup + r * args.steps, args.steps)
        sync_all()
        t1 = copdist.monotonic_ns()
        harness.append((t1 - t0) * 1e-9)
        if stamps is not None and args.window == "library":
            # the window of the library call itself: first post -> last
            # batch seen complete, stamped inside cop_pmd_run_timed (the
            # Python call overhead around it stays out; runs_ms_harness
            # keeps the gate-to-return window beside it)
            t0, t1 = stamps
        if rc_on and coll == "ok":
            # one reporting interval, after the window and timed on its own:
            # read-and-zero the counters + per-rule hits and sum them over
            # all GPUs (RCCL; the poll-mode kernel is paused around it). The
            # reference reads and zeroes its counters every PRINT_DELAY = 2 s
            # (switch.h:23, switch.c:517-521): far fewer reduces than one per
            # 20-step window
            r0 = time.perf_counter()
            tot, _ = ctx.coll_reduce_counters(reset=True, with_rules=False)
            reduce_ms.append((time.perf_counter() - r0) * 1e3)
            reduce_runs.append(int(tot["rx"]))
        group.barrier()
        own_runs.append((t1 - t0) * 1e-9)
        windows.append((t0, t1))
        runs.append(group.max((t1 - t0) * 1e-9))
    elapsed = float(np.median(runs))
    total_pkts = world * args.steps * B
    value = total_pkts / elapsed / 1e6
    own_rate = args.steps * B / float(np.median(own_runs)) / 1e6
    wstats = copdist.window_stats(group.gather_obj(windows), world, args.steps * B)
    log(f"[rank {rank}] {name}: timed {args.steps} steps x {len(runs)} runs ({engine}), median "
        f"{elapsed * 1e3:.3f} ms -> {value:.1f} Mpkt/s (all ranks); runs {[round(x * 1e3, 3) for x in runs]} ms; "
        f"windows overlap {wstats['windows_overlap']}, union {wstats['value_union']:.1f} Mpkt/s")
    res = {"W": W, "name": name, "B": B, "Lb": Lb, "P": P, "engine": engine, "value": value, "elapsed": elapsed,
           "harness_runs": [group.max(x) for x in harness],
           "runs": runs, "own_rate": own_rate, "windows": wstats, "reduce_ms": reduce_ms, "rc_on": rc_on, "coll": coll,
           "fw_rules": fw_rules, "routes": routes,
           "fw_tab": fw_tab, "rt_tab": rt_tab, "cnt_per_slot": cnt_per_slot, "d_pkts": d_pkts, "d_res": d_res,
           # every buffer the ring points at stays referenced as long as the
           # ring is used (a DeviceBuffer frees its memory when collected)
           "bufs": (d_pkts, d_res, d_fwd, d_cnt), "ring": ring, "per_batch": per_batch}
    if W["imix"]:
        res["slab"], res["offs"] = slab, offs

    # ---- the poll-mode kernel's steady state and single-batch latency ----
    if engine == "pmd" and primary and not args.quick:
        pmd_on()
        n_long = min(P, 1024)
        longs = []
        for _ in range(3):
            t0 = time.perf_counter()
            pmd.run(n_long)
            longs.append(time.perf_counter() - t0)
        lat = []
        for _ in range(50):
            t0 = time.perf_counter()
            pmd.run(1)
            lat.append((time.perf_counter() - t0) * 1e6)
        # a producer that posts one batch per call and keeps up to `depth`
        # in flight (waits only for the oldest): the rate a deployment handing
        # over single 64k batches gets
        depth = min(16, P)
        n_one = min(P * 2, 512)
        t0 = time.perf_counter()
        for _ in range(n_one):
            if pmd.posted >= depth:
                pmd.wait(pmd.posted - depth + 1)
            pmd.post(1)
        pmd.wait()
        t_one = time.perf_counter() - t0
        info = pmd.info()
        t_long = float(np.median(longs))
        # the same posts with dynamic tiles (COP_PMD_DYNAMIC_TILES, segmented
        # lists): a kernel of its own, the 1024-batch steady state and the
        # driver's 20-step post (reported beside the static order's)
        dyn = None
        if seg:
            pmd_off()
            pmd = ctx.pmd_start(ring, pmd_flags | cg.PMD_DYNAMIC_TILES)
            pmd.run(n_long)
            d_longs, d_short = [], []
            for _ in range(3):
                t0 = time.perf_counter()
                pmd.run(n_long)
                d_longs.append(time.perf_counter() - t0)
            for _ in range(11):
                # as the line's runs: a barrier between posts (back to back,
                # the next post met workers still counting the last one)
                group.barrier()
                t0 = time.perf_counter()
                pmd.run(args.steps)
                d_short.append(time.perf_counter() - t0)
            di = pmd.info()
            dl = float(np.median(d_longs))
            dyn = {"workers": di["workers"], "packets_per_tile": di["packets_per_tile"],
                   "steady_mpkt_s": round(n_long * B / dl / 1e6, 3), "steady_ms": round(dl * 1e3, 4),
                   f"mpkt_s_{args.steps}_steps": round(args.steps * B / float(np.median(d_short)) / 1e6, 3),
                   "note": "not the line's value: host-timed posts of this kernel, a barrier between them, no gate"}
        res["pmd_info"] = {"workers": info["workers"], "workers_per_cu": info["workers_per_cu"],
                           "packets_per_tile": info["packets_per_tile"], "launches": info["launches"],
                           "steady_batches": n_long, "steady_mpkt_s": round(n_long * B / t_long / 1e6, 3),
                           "steady_ms": round(t_long * 1e3, 4),
                           "single_batch_post_to_done_us_median": round(float(np.median(lat)), 2),
                           "one_batch_posts": {"batches": n_one, "in_flight": depth,
                                               "mpkt_s": round(n_one * B / t_one / 1e6, 3)}}
        if dyn:
            res["pmd_info"]["dynamic_tiles"] = dyn
    pmd_off()

    if rc_on and coll == "ok":
        # the reduction alone (counters are zero now: same bytes, same cost);
        # the interval sums are checked and reported, never asserted (one
        # failing rank must not kill the whole N-GPU line)
        group.barrier()
        r0 = time.perf_counter()
        ctx.coll_reduce_counters(reset=False, with_rules=False)
        r_ms = (time.perf_counter() - r0) * 1e3
        n_rules = len(ctx.rule_counters())
        want = [world * (args.warmup + args.steps) * B] + [world * args.steps * B] * (len(reduce_runs) - 1)
        per_iv = [round(group.max(x), 3) for x in res["reduce_ms"]]
        med_red = float(np.median(per_iv)) if per_iv else 0.0
        res["reduce_info"] = {"rccl_allreduce_u64_words": SHARD_AND_PORT_WORDS + n_rules, "ranks": world,
                              "ms": round(group.max(r_ms), 3),
                              "ms_per_interval": per_iv,
                              "timing": "each interval's reduce runs after its timed window, timed on its own "
                                        "(max over ranks); value excludes it",
                              "value_with_reduce_per_window": round(
                                  world * args.steps * B / (res["elapsed"] + med_red * 1e-3) / 1e6, 3),
                              "cadence": "reference: print_stats reads and zeroes every PRINT_DELAY = 2 s "
                                         "(switch.h:23, switch.c:517-521); one reduce per 2 s costs "
                                         f"{med_red / 2000.0 * 100:.4f} % of the interval",
                              "pkts_reduced_per_interval": reduce_runs,
                              "expected_per_interval": want, "ok": reduce_runs == want}
        if reduce_runs != want:
            log(f"[rank {rank}] RCCL interval sums {reduce_runs} differ from the packets run {want}")
        log(f"[rank {rank}] rccl counter all-reduce of {SHARD_AND_PORT_WORDS + n_rules} u64: {r_ms:.3f} ms")

    # ---- kernel duration per launch (HIP events on the context stream) ----
    run_steps(0, Lb)   # untimed: loads the one-shot kernel's code object (first launch)
    ctx.sync()
    ctx.counters(reset=True)
    ctx.launch_timing(True)
    nl = max(8, min(200, args.steps // Lb)) if primary else 8
    run_steps(0, nl * Lb)
    ctx.sync()
    mean_ms, n_launch = ctx.launch_timing_read(reset=True)
    ctx.launch_timing(False)
    cnt = ctx.counters()
    res.update(mean_ms=mean_ms, n_launch=n_launch, nl=nl, cnt=cnt)
    fwd_frac = cnt["forward"] / max(1, cnt["rx"])
    # algorithmic bytes per packet: the 64 B header line (+4 B offset for
    # IMIX), the 8 B result record, 4 B per forwarded packet for the
    # ordered forward list, and its counts (4 B per 256-packet segment, or
    # per batch)
    bytes_per_pkt = (76 if W["imix"] else 72) + 4 * fwd_frac + 4.0 * cnt_per_slot / B
    alg_bytes = bytes_per_pkt * B * Lb
    achieved = alg_bytes / (mean_ms * 1e-3) / 1e9 if mean_ms > 0 else 0.0
    res.update(bytes_per_pkt=bytes_per_pkt, alg_bytes=alg_bytes, achieved=achieved, total_pkts=total_pkts)
    try:   # a report only: never fails the line
        if W["imix"]:
            probes = table_probes(fw_tab, rt_tab, slab, offs, args.route_form, args.fw_form)
        else:
            sample = cg.gen_trace(copdist.shard_seed(0x5EED0000 + cid, rank, 0), B, fw_rules, routes)
            probes = table_probes(fw_tab, rt_tab, sample, None, args.route_form, args.fw_form)
    except Exception as e:  # noqa: BLE001
        probes = {"error": repr(e)}
    res["probes"] = probes
    ppp, tables = dir_probes_per_pkt(probes) if "error" not in probes else (0.0, 0)
    if tables and not args.quick:
        g = probe_ceiling(ctx, tables)
        if g:
            kernel_pkt_s = B * Lb / (mean_ms * 1e-3)
            res["probe"] = {"per_pkt": round(ppp, 4), "tables": tables,
                            "kernel_gprobes_s": round(ppp * kernel_pkt_s / 1e9, 2),
                            "ceiling_gprobes_s": round(g, 2),
                            "probe_bound": round(ppp * kernel_pkt_s / 1e9 / g, 4),
                            "ceiling_what": f"same box: uniformly random dword loads into {tables} table(s) of "
                                            f"2^24 u32 (the tbl24 size), 8 or 16 packets x {tables} probe(s) per lane, 8 or 16 workgroups per CU, the best of the four shapes, in "
                                            f"flight (tools/probe_kernels.h)"}
    traffic = None
    tpath = os.path.join(TRAFFIC_DIR, f"traffic_{name}_L{Lb}_{args.lists}.json")
    if os.path.exists(tpath):
        try:
            traffic = json.load(open(tpath)).get("hbm_bytes_per_launch")
        except Exception:  # noqa: BLE001
            traffic = None
    res["traffic"] = traffic
    # the poll-mode kernel's PMC traffic per posted batch (tools/pmc_pmd.py:
    # one kernel lifetime serving exactly K posted batches of this workload)
    res["traffic_pmd"] = None
    tp = os.path.join(TRAFFIC_DIR, f"traffic_pmd_{name}_{args.lists}.json")
    if os.path.exists(tp):
        try:
            tj = json.load(open(tp))
            res["traffic_pmd"] = {"per_batch": tj["hbm_bytes_per_batch"], "batches": tj.get("batches"),
                                  "kernel": tj.get("kernel"),
                                  "source": f"bench_traffic/traffic_pmd_{name}_{args.lists}.json"}
        except Exception:  # noqa: BLE001
            pass
    return res, ctx


def roofline_launch_block(res, world, group, args):
    """The one-shot kernel's roofline: algorithmic bytes per launch of Lb
    batches / the mean kernel duration (HIP events on the lane's stream around
    every launch; rocprofv3 --kernel-trace --stats of the same command must
    agree), PMC traffic per launch (tools/pmc_traffic.py)."""
    achieved, alg_bytes = res["achieved"], res["alg_bytes"]
    ach_min, ach_max, ach_sum = group.min(achieved), group.max(achieved), group.sum(achieved)
    traffic = res["traffic"]
    out = {
        "engine": "launch",
        "bound": "hbm",
        "achieved": round(achieved, 2),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "algorithmic_bytes_per_pkt": round(res["bytes_per_pkt"], 3),
        "algorithmic_bytes_per_launch": round(alg_bytes),
        "traffic_per_algorithmic": (round(traffic / alg_bytes, 4) if traffic else None),
        "traffic_source": (f"bench_traffic/traffic_{res['name']}_L{res['Lb']}_{args.lists}.json (rocprofv3 PMC, "
                           f"tools/pmc_traffic.py)" if traffic else None),
        "kernel_ms_per_launch": round(res["mean_ms"], 6),
        "launches_timed": int(res["n_launch"]),
        "batches_per_launch": res["Lb"],
        "all_gpus": {"n": world, "achieved_sum": round(ach_sum, 2), "peak_sum": HBM_PEAK_GBS * world,
                     "frac": round(ach_sum / (HBM_PEAK_GBS * world), 4),
                     "per_gpu_min": round(ach_min, 2), "per_gpu_max": round(ach_max, 2)},
    }
    if "probe" in res:
        out["probe_bound"] = res["probe"]["probe_bound"]
    return out


def roofline_block(res, world, group, args):
    """The roofline of the engine that produced `value`. For the poll-mode
    kernel (one launch serves every posted batch, so there is no per-launch
    duration): the algorithmic bytes of the K timed steps on all GPUs over the
    timed window, i.e. frac == frac_timed, with the kernel's PMC traffic per
    posted batch scaled to the same K steps. For one-shot launches: the
    launch block, plus frac_timed."""
    bpp = res["bytes_per_pkt"]
    frac_timed = round(bpp * res["total_pkts"] / res["elapsed"] / 1e9 / (HBM_PEAK_GBS * world), 4)
    if res["engine"] != "pmd":
        out = roofline_launch_block(res, world, group, args)
        out["frac_timed"] = frac_timed
    else:
        steps_bytes = bpp * args.steps * res["B"]              # per GPU, per timed window
        achieved = steps_bytes / res["elapsed"] / 1e9          # max-over-ranks window
        tp = res.get("traffic_pmd")
        traffic = tp["per_batch"] * args.steps if tp else None
        out = {
            "engine": "pmd",
            "bound": "hbm",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "frac_timed": frac_timed,
            "unit_of_work": f"one timed window: {args.steps} posted batches x {res['B']} packets per GPU",
            "traffic": (round(traffic) if traffic else None),
            "algorithmic_bytes_per_pkt": round(bpp, 3),
            "algorithmic_bytes": round(steps_bytes),
            "traffic_per_algorithmic": (round(traffic / steps_bytes, 4) if traffic else None),
            "traffic_per_batch": (round(tp["per_batch"]) if tp else None),
            "traffic_source": (f"{tp['source']} (rocprofv3 PMC FETCH_SIZE / WRITE_SIZE over one kernel lifetime "
                               f"serving exactly {tp['batches']} posted batches, tools/pmc_pmd.py; the per-batch "
                               f"bytes x {args.steps} steps)" if tp else None),
            "kernel": (tp["kernel"] if tp else None),
            "ms_per_window": round(res["elapsed"] * 1e3, 6),
            "timing": "host CLOCK_MONOTONIC around post -> every batch complete (the poll-mode kernel's one "
                      "launch serves every post: no per-launch kernel time exists; rocprofv3 sees one lifetime "
                      "dispatch)",
        }
    out["table_probes"] = res["probes"]
    if "probe" in res:
        pr = dict(res["probe"])
        if res["engine"] == "pmd":
            # the poll-mode rate over the timed window against the same box's
            # random-probe ceiling (the one-shot kernel's is roofline_launch's)
            g = pr["per_pkt"] * args.steps * res["B"] / res["elapsed"] / 1e9
            pr["timed_gprobes_s"] = round(g, 2)
            pr["probe_bound_timed"] = round(g / pr["ceiling_gprobes_s"], 4)
            out["probe_bound"] = pr["probe_bound_timed"]
        else:
            out["probe_bound"] = pr["probe_bound"]
        out["probe_ceiling"] = pr
    return out


def job_cpu_share() -> tuple:
    """(threads, note): the job's CPU share. The affinity mask of a GPU box
    lists every core of the host, but the job's share is $OMP_NUM_THREADS
    (16 on the pool's one-GPU boxes)."""
    affinity = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    n = max(1, min(affinity, share if share > 0 else affinity))
    note = (f"the job's CPU share: OMP_NUM_THREADS={share} of {affinity} cores in the affinity mask" if share > 0
            else f"every core of the affinity mask ({affinity})")
    return n, note


def e2e_leg(args, dev) -> dict:
    """North star: packets start and end in host memory. The end-to-end rate
    of cop_process_host_stream over an mbuf-like host pool (NB_MBUF = 131072
    buffers 2176 bytes apart, data at 128 bytes of headroom, init.h:38-44),
    visited `passes` times: the host threads gather each batch's 12-byte header
    records (COP_HDR12_STRIDE) into pinned staging (and copy the previous
    batch's 8-byte records out), hipMemcpyAsync H2D, the pipeline (stage P +
    firewall, fw1k), the records written into mapped pinned memory;
    lanes (HIP streams, not threads) overlap batches. Host threads = the
    job's CPU share, the caller included (HIP's own runtime threads aside):
    the count the CPU baseline's multicore leg runs. Checked against the device-resident
    pipeline's own records for the same packets (no oracle here)."""
    NB, STRIDE, HEAD = 131072, 2176, 128
    threads, note = job_cpu_share()
    fw = cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)
    pk = cg.gen_trace(copdist.shard_seed(0x5EED0002, 0, 0), NB, fw)
    pool = np.zeros(NB * STRIDE, dtype=np.uint8)
    pool.reshape(NB, STRIDE)[:, HEAD:HEAD + 64] = pk.reshape(NB, 64)
    passes = 64     # 32 batches of 256k per run: the lanes' fill and drain amortised
    n = passes * NB
    ptrs = (pool.ctypes.data + HEAD + (np.arange(n, dtype=np.uint64) % NB) * STRIDE).astype(np.uint64)
    out = np.zeros(n, dtype=cg.RESULT_DT)
    res = {"pool": f"{NB} mbufs x {STRIDE} B (headroom {HEAD}), {passes} passes = {n} packets per run",
           "stages": "parse + firewall (fw1k)", "cores_note": note, "rows": []}
    want = None
    best = None
    rows = [(4, threads, 131072, 2), (4, threads, 262144, 2), (4, threads, 65536, 2), (2, threads, 131072, 2),
            (4, threads, 131072, 0), (4, threads, 131072, 1), (4, 1, 131072, 2)]
    zc0 = os.environ.get("COP_STREAM_ZC")
    for lanes, thr, batch, zc in rows:
        # zc ($COP_STREAM_ZC): 2 (the default) the copy engine moves the
        # staged records H2D and the kernel writes the results into mapped
        # pinned memory; 1 the kernel reads the staging too; 0 both copied
        os.environ["COP_STREAM_ZC"] = str(zc)
        ctx = cg.Context(device=dev, stages=cg.STAGE_PARSE | cg.STAGE_FW, max_batch=262144, n_streams=lanes)
        try:
            ctx.set_fw_table(cg.LpmTable(fw, 1024, 24, True))
            if want is None:
                # the device-resident kernel's records for the pool's packets
                d_p = ctx.alloc(pk.nbytes)
                d_p.upload(pk)
                d_r = ctx.alloc(NB * 8)
                ctx.submit([cg.make_batch(d_p, NB, d_r)])
                ctx.sync()
                want = d_r.download(cg.RESULT_DT, NB)
            ctx.set_host_threads(thr)
            ctx.process_host_stream(ptrs, batch, out=out)     # warm (pinned staging, pool pages)
            ok = bool(np.array_equal(out[:NB].view(np.uint8), want.view(np.uint8)) and
                      np.array_equal(out[-NB:].view(np.uint8), want.view(np.uint8)))
            times = []
            for _ in range(7):
                t0 = time.perf_counter()
                ctx.process_host_stream(ptrs, batch, out=out)
                times.append(time.perf_counter() - t0)
            t = float(np.median(times))
            row = {"lanes": lanes, "host_threads": thr, "batch": batch,
                   "zero_copy": {0: "none", 1: "staging + records", 2: "records"}[zc],
                   "mpkt_s": round(n / t / 1e6, 3),
                   "header_record_bytes": 12, "h2d_gb_s": round(n * 12 / t / 1e9, 2),
                   "d2h_gb_s": round(n * 8 / t / 1e9, 2),
                   "runs_ms": [round(x * 1e3, 3) for x in times], "matches_device_records": ok}
            res["rows"].append(row)
            log(f"[rank 0] e2e {row}")
            if thr == threads and ok and (best is None or row["mpkt_s"] > best["mpkt_s"]):
                best = row
        finally:
            ctx.close()
    if zc0 is None:
        os.environ.pop("COP_STREAM_ZC", None)
    else:
        os.environ["COP_STREAM_ZC"] = zc0
    if best:
        res.update(mpkt_s=best["mpkt_s"], threads=threads, lanes=best["lanes"], batch=best["batch"],
                   zero_copy=best["zero_copy"])
    one = [r for r in res["rows"] if r["host_threads"] == 1]
    if one:
        res["one_thread_mpkt_s"] = one[0]["mpkt_s"]
    return res


def cpu_legs(args, W, fw_rules) -> dict:
    """cpu_baseline (1 pinned core) and cpu_baseline_multicore (the job's CPU
    share): the oracle's restatement of the reference coprocessor() loop
    (oracle/cop_oracle.c) over a bounded sample, args.cpu_budget seconds."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc   # CPU baseline leg only
    out = {}
    ofw = orc.OracleLpm(max(1024, W["fw"]), 24 if W["fw"] <= 1000 else 1 << 20)
    ofw.setup(fw_rules["ip"], fw_rules["depth"], fw_rules["next_hop"], stop_at_error=W["fw"] <= 1000)
    ns = 131072
    trace = cg.gen_trace(0x5EED0001, ns, fw_rules, None)   # configs[0] seed: CPU reference case
    # pin to the last core this process may use (core 0 also serves this
    # process's main thread and the driver's interrupts)
    core = max(os.sched_getaffinity(0))
    rate, pk, secs = orc.coprocessor_bench(trace, ns, ofw, args.cpu_budget, 1, core)
    model = cpu_model()
    out["cpu_baseline"] = {
        "value": round(rate, 3),
        "unit": "Mpkt/s",
        "cores": 1,
        "kind": "port",
        "cpu_model": model,
        "sample": (f"{pk} packets through the restated coprocessor() loop (burst 32, 16384-slot "
                   f"SPSC ring, 2176 B mbufs, DIR-24-8 firewall, {W['fw']} rules), "
                   f"{secs:.1f} s on 1 pinned core (cpu {core}, {model})"),
    }
    log(f"[rank 0] cpu baseline {rate:.1f} Mpkt/s on 1 core ({pk} pkts)")
    # one coprocessor thread per host core of this
    # job's CPU share (job_cpu_share): the leg uses that many, and says so
    ncores, cores_note = job_cpu_share()
    if ncores > 1:
        rate_m, pk_m, secs_m = orc.coprocessor_bench(trace, ns, ofw, args.cpu_budget / 2, ncores, -1)
        out["cpu_baseline_multicore"] = {
            "value": round(rate_m, 3), "unit": "Mpkt/s", "cores": ncores, "kind": "port", "cpu_model": model,
            "cores_note": cores_note,
            "sample": (f"{pk_m} packets, {ncores} threads each running the restated coprocessor() loop "
                       f"on its own rings and mbuf pool, {secs_m:.1f} s"),
        }
        log(f"[rank 0] cpu baseline {rate_m:.1f} Mpkt/s on {ncores} cores")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--allow-shared-gpu", action="store_true",
                    help="let more ranks than visible GPUs run (they share GPUs; the line says so)")
    ap.add_argument("--dry-run", action="store_true",
                    help="test the launch and rank protocol only: no GPU, fake timings (CPU tests)")
    ap.add_argument("--dry-run-devices", type=int, default=8, help="GPUs a --dry-run pretends to see")
    ap.add_argument("--dry-run-fail-rank", type=int, default=-1, help="--dry-run: this rank exits 3 at start")
    ap.add_argument("--steps", type=int, default=16384)
    ap.add_argument("--warmup", type=int, default=2048)
    ap.add_argument("--workload", default="fw1k", choices=sorted(WORKLOADS))
    ap.add_argument("--secondary", default="auto",
                    help="also time these workloads in the same run, comma-separated, or none (auto, when the "
                         "primary is fw1k: fw_lpm, the north-star FW + LPM pipeline (configs[3]); fw_lpm_imix "
                         "(configs[2]); fw_lpm_1m, 1M + 1M tables with per-rule counters all-reduced over RCCL "
                         "across every rank (configs[4]))")
    ap.add_argument("--slots", default="static", choices=("static", "reuse", "always"),
                    help="poll-mode slot declaration: static = the pool is written once before the start "
                         "(COP_PMD_STATIC_SLOTS, plain loads); reuse = the default of cop_pmd_start "
                         "(system-coherent sc0 sc1 loads once the ring wraps); always = coherent loads on every "
                         "tile (COP_PMD_SYS_ACQUIRE)")
    ap.add_argument("--fw-form", default="dir", choices=("dir", "bkt"),
                    help="firewall tables too large for LDS (1M rules): DIR-24-8 image, or the bucketed intervals "
                         "keyed by rule id (COP_CFG_FW_BKT)")
    ap.add_argument("--out-mem", default="device", choices=("device", "uncached", "fine"),
                    help="A/B: the ring's records, lists and counts in HBM (default), uncached HBM or fine-grained "
                         "HBM (cop_dev_alloc_ex)")
    ap.add_argument("--deadline", type=float, default=1500.0,
                    help="seconds after which a rank that has not finished exits with status 124 (a hung rank "
                         "must not hold the driver's node)")
    ap.add_argument("--per-launch", type=int, default=0,
                    help="batches per kernel launch (ring submit, at most 1024; 0: the workload's default). The "
                         "~23 us per-launch ramp and tail cost 6 %% at 384 batches, 2.5 %% at 1024")
    ap.add_argument("--streams", type=int, default=1, help="launch lanes (concurrent streams)")
    ap.add_argument("--engine", default="auto", choices=("auto", "pmd", "launch"),
                    help="pmd: the poll-mode kernel serves the batch ring (steps are posted to it); launch: one "
                         "kernel launch per --per-launch steps; auto: pmd for short runs (< 1024 steps: no "
                         "per-launch ramp), launch for long runs (large launches stream faster)")
    ap.add_argument("--pool-mib", type=int, default=0,
                    help="distinct input bytes per GPU (0: max(400 MiB, one launch of batches))")
    ap.add_argument("--repeats", type=int, default=5, help="timed runs of K steps; the value is their median")
    ap.add_argument("--window", default="library", choices=("library", "harness"),
                    help="poll-mode runs: time each run over the library call itself (cop_pmd_run_timed: first "
                         "post -> last batch complete) or over the Python harness's gate-to-return window; both "
                         "are reported (runs_ms, runs_ms_harness)")
    ap.add_argument("--cpu-budget", type=float, default=8.0, help="seconds of CPU baseline work")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip rank 0's end-to-end host-memory leg (mbuf pool -> pinned staging -> H2D -> pipeline "
                         "-> D2H)")
    ap.add_argument("--no-numa-bind", action="store_true",
                    help="do not move the process onto the CPUs of the GPU's NUMA node")
    ap.add_argument("--quick", action="store_true",
                    help="A/B runs: the timed steps and the kernel roofline only (no poll-mode extras, single-batch "
                         "latency, ceilings, RCCL check, secondary workload or CPU baseline)")
    ap.add_argument("--no-rule-counters", action="store_true", help="ablation: config 5 without per-rule counters")
    ap.add_argument("--no-rccl-check", action="store_true",
                    help="skip the untimed RCCL all-reduce of the ranks' counters at the end")
    ap.add_argument("--stages", type=int, default=0, help="ablation: override the workload's stage mask")
    ap.add_argument("--no-compact", action="store_true", help="ablation: no ordered forward lists")
    ap.add_argument("--lists", default="seg", choices=("seg", "dense"),
                    help="ordered forward lists: seg = 256-packet segments (COP_CFG_SEG_LISTS: per-segment "
                         "lists + counts, no cross-tile prefix), dense = one list per batch (decoupled look-back)")
    ap.add_argument("--route-form", default="dir", choices=("dir", "trie", "bkt"),
                    help="route tables too large for LDS: DIR-24-8 image (HBM / Infinity Cache) or the multibit "
                         "trie (12-bit LDS top level + L2-resident 6-bit nodes) or the bucketed intervals "
                         "(index + (start, value) pairs in L2: two loads per lookup)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    rank, world, local = copdist.env()
    secondary = args.secondary
    if secondary == "auto":
        secondary = "fw_lpm,fw_lpm_imix,fw_lpm_1m" if args.workload == "fw1k" and not args.quick else "none"
    secondaries = [x for x in secondary.split(",") if x and x != "none" and x != args.workload]
    bad = [x for x in secondaries if x not in WORKLOADS]
    if bad:
        raise SystemExit(f"[bench] unknown --secondary workload(s) {bad}: choose from {sorted(WORKLOADS)}")
    if args.quick:
        args.no_cpu = args.no_rccl_check = True
    if args.deadline > 0:
        watchdog(args.deadline, rank)

    if args.dry_run:
        return dry_run(args, rank, world, local, WORKLOADS[args.workload], secondaries)
    cg.lib()   # load the HIP runtime the product links (before torch)
    ndev = cg.device_count()
    check_devices(args, world, local, ndev)
    dev = copdist.device_for(local, ndev)
    no_bind = args.no_numa_bind or os.environ.get("COP_NO_NUMA_BIND") == "1"
    numa = copdist.bind_near_device(cg.device_pci_bus_id(dev)) if not no_bind else {"skipped": True}
    log(f"[rank {rank}] host side near device {dev}: {numa}")
    group = copdist.Group(rank, world, "gloo")
    gate = copdist.StartGate(group)

    res, ctx = measure(args, args.workload, rank, world, dev, group, gate, primary=True)
    W, B, P, Lb = res["W"], res["B"], res["P"], res["Lb"]
    ranks_info = group.gather_obj({"rank": rank, "device": dev, "mpkt_s": round(res["own_rate"], 3), "numa": numa,
                                   **({"rccl_init": res["coll"]} if res["rc_on"] else {})})

    # ---- single-batch latency: one batch per launch, nothing
    # else in flight; kernel time from HIP events, submit->sync on the host ----
    n_lat = 0 if args.quick else 50
    host_us = [0.0]
    ctx.launch_timing(True)
    for i in range(n_lat):
        h0 = time.perf_counter()
        ctx.submit_ring(res["ring"], i % P, 1)
        ctx.sync()
        host_us.append((time.perf_counter() - h0) * 1e6)
    lat_ms, _ = ctx.launch_timing_read(reset=True)
    ctx.launch_timing(False)
    single_batch = None if args.quick else {"batch": B, "launches": n_lat, "kernel_us_mean": round(lat_ms * 1e3, 2),
                    "host_submit_to_sync_us_median": round(float(np.median(host_us)), 2)}

    # ---- the ranks' counters summed by RCCL over xGMI (print_stats' totals of
    # every coprocessor, switch.c:33-90), checked against the packets each rank
    # ran since the reset above; untimed, and a failure is reported, not fatal
    allreduce_check = None
    if not res["rc_on"] and not args.no_rccl_check:
        try:
            ctx.sync()
            uid = group.broadcast_bytes(cg.coll_unique_id() if rank == 0 else None)
            ctx.coll_init(uid, rank, world)
            group.barrier()
            r0 = time.perf_counter()
            tot, _ = ctx.coll_reduce_counters(reset=False, with_rules=False)
            r_ms = (time.perf_counter() - r0) * 1e3
            want = world * (res["nl"] * Lb + n_lat) * B
            allreduce_check = {"ranks": world, "u64_words": SHARD_AND_PORT_WORDS, "ms": round(group.max(r_ms), 3),
                               "rx_sum": int(tot["rx"]), "rx_expected": want, "ok": int(tot["rx"]) == want}
        except Exception as e:   # noqa: BLE001 (reported in the line)
            allreduce_check = {"ranks": world, "error": str(e)[:200]}
        log(f"[rank {rank}] rccl counter check: {allreduce_check}")

    # the same box's streaming ceiling for this byte mix (tools/ceiling.hip):
    # read every 64 B slot of the pool, write an 8 B record, nothing else
    ceiling = None
    if not W["imix"] and not args.quick:
        ceiling = box_ceiling(res["d_pkts"].addr, P * B, res["d_res"].addr)

    # the roofline of the engine behind `value` (config.engine), and the
    # one-shot kernel's beside it (its HIP-event launch time is what rocprofv3
    # --kernel-trace --stats of this command reports)
    roof = roofline_block(res, world, group, args)
    roof_launch = roof if res["engine"] != "pmd" else roofline_launch_block(res, world, group, args)
    if ceiling is not None:
        roof_launch["box_ceiling"] = {
            "what": "same pool, same process: read each 64 B slot + write an 8 B record, no classification "
                    "(tools/ceiling.hip: the best of grid-stride copies and per-wave LDS-DMA rings)",
            "best_pattern": ceiling[1], "achieved": round(ceiling[0], 2), "unit": "GB/s",
            "frac_of_peak": round(ceiling[0] / HBM_PEAK_GBS, 4),
            "pipeline_frac_of_ceiling": round(res["achieved"] / ceiling[0], 4),
            "patterns": ceiling[2]}

    out = {
        "metric": METRIC,
        "value": round(res["value"], 3),
        "unit": "Mpkt/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(res["elapsed"] * 1e3 / args.steps, 6),
        "runs_ms": [round(x * 1e3, 4) for x in res["runs"]],
        # the window each value run is timed over (config.window), and the
        # gate-to-return window of the Python harness around the same call
        "runs_ms_harness": [round(x * 1e3, 4) for x in res["harness_runs"]],
        # value = every rank's packets / the max over ranks of each rank's own
        # window; beside it, how far the windows overlapped (the start gate
        # opens them together) and the rate over their union
        "windows_overlap": res["windows"]["windows_overlap"],
        "value_union": round(res["windows"]["value_union"], 3),
        "windows": res["windows"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (splitmix64 64B Eth/IPv4/UDP frames and rule sets, SURVEY.md §8d seeds)",
        "config": {
            "workload": args.workload,
            "description": W["desc"],
            "batch": B,
            "batches_per_launch": Lb,
            "streams": args.streams,
            "fw_rules": W["fw"],
            "route_prefixes": W["routes"],
            "route_form": args.route_form if W["routes"] else None,
            "fw_form": args.fw_form if W["fw"] > 8192 else "lds-intervals",
            "slots": args.slots if res["engine"] == "pmd" else None,
            "pkt_layout": "imix slab + u32 offsets" if W["imix"] else "64B slots",
            "stages": args.stages or W["stages"],
            "parallelism": f"independent per-GPU contexts x{world} (no data-path collective)",
            "pool_batches": int(P),
            "rule_counters": res["rc_on"],
            "engine": res["engine"],
            "window": ("library: CLOCK_MONOTONIC inside cop_pmd_run_timed, first post -> last batch complete"
                       if res["engine"] == "pmd" and args.window == "library" else
                       "harness: CLOCK_MONOTONIC from the start gate's release to the return of the run"),
            "fwd_lists": ("none (ablation)" if args.no_compact else
                          "segmented: per 256-packet segment an ordered list + count (COP_CFG_SEG_LISTS)"
                          if args.lists == "seg" else "dense: one ordered list per batch (decoupled look-back)"),
            "ranks": ranks_info,
        },
        "roofline": roof,
        "cpu_baseline": None,
    }
    if roof_launch is not roof:
        out["roofline_launch"] = roof_launch
    if single_batch:
        out["single_batch_latency"] = single_batch
    if "pmd_info" in res:
        # the poll-mode kernel: a 1024-batch post (HBM-resident, one post, no
        # launch) timed on the host, as a fraction of the peak
        pi = res["pmd_info"]
        pi["steady_frac"] = round(pi["steady_mpkt_s"] * 1e6 * res["bytes_per_pkt"] / 1e9 / HBM_PEAK_GBS, 4)
        if "dynamic_tiles" in pi:
            dt = pi["dynamic_tiles"]
            dt["steady_frac"] = round(dt["steady_mpkt_s"] * 1e6 * res["bytes_per_pkt"] / 1e9 / HBM_PEAK_GBS, 4)
        if res.get("traffic_pmd"):
            tp = res["traffic_pmd"]
            pi["traffic_per_batch"] = round(tp["per_batch"])
            pi["traffic_per_algorithmic"] = round(tp["per_batch"] / (res["bytes_per_pkt"] * B), 4)
            pi["traffic_source"] = tp["source"]
        out["pmd"] = pi
    if "reduce_info" in res:
        out["counter_reduce"] = res["reduce_info"]
    if allreduce_check:
        out["counter_allreduce_check"] = allreduce_check
    ctx.close()

    # ---- the other BASELINE workloads in the same run: the north-star FW +
    # LPM 100k (configs[3]), IMIX (configs[2]) and 1M + 1M with per-rule
    # counters reduced over RCCL across every rank (configs[4]) ----
    for sname in secondaries:
        try:
            sres, sctx = measure(args, sname, rank, world, dev, group, gate, primary=False)
            sroof = roofline_block(sres, world, group, args)
            sroof_launch = roofline_launch_block(sres, world, group, args) if sres["engine"] == "pmd" else None
            blk = {
                "description": sres["W"]["desc"], "value": round(sres["value"], 3), "unit": "Mpkt/s",
                "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(sres["elapsed"] * 1e3 / args.steps, 6),
                "runs_ms": [round(x * 1e3, 4) for x in sres["runs"]], "engine": sres["engine"],
                "runs_ms_harness": [round(x * 1e3, 4) for x in sres["harness_runs"]],
                "windows_overlap": sres["windows"]["windows_overlap"],
                "value_union": round(sres["windows"]["value_union"], 3),
                "batch": sres["B"], "fw_rules": sres["W"]["fw"], "route_prefixes": sres["W"]["routes"],
                "pkt_layout": "imix slab + u32 offsets" if sres["W"]["imix"] else "64B slots",
                "route_form": args.route_form, "fw_form": args.fw_form if sres["W"]["fw"] > 8192 else "lds-intervals",
                "rule_counters": sres["rc_on"], "roofline": sroof}
            if sroof_launch is not None:
                blk["roofline_launch"] = sroof_launch
            if sres["rc_on"]:
                blk["rccl_init"] = group.gather_obj(sres["coll"])
            if "reduce_info" in sres:
                blk["counter_reduce"] = sres["reduce_info"]
            out.setdefault("secondary", {})[sname] = blk
            sctx.close()
        except Exception as e:  # noqa: BLE001 (the primary line stands)
            out.setdefault("secondary", {})[sname] = {"error": str(e)[:300]}
            log(f"[rank {rank}] secondary {sname} failed: {e}")

    # the CPU baseline: on rank 0 after the GPU timing, at
    # every N (north_star: "next to the reference DPDK CPU coprocessor timed
    # on the same box's host cores in the same run")
    if rank == 0 and not args.no_cpu:
        e2e = None
        if not args.no_e2e:
            try:
                e2e = e2e_leg(args, dev)
            except Exception as e:  # noqa: BLE001 (a report: never fails the line)
                e2e = {"error": str(e)[:300]}
        out.update(cpu_legs(args, W, res["fw_rules"]))
        if e2e is not None:
            mc = out.get("cpu_baseline_multicore") or {}
            if "mpkt_s" in e2e and mc.get("cores") == e2e.get("threads"):
                e2e["cpu_same_threads"] = mc["value"]
                e2e["ratio_vs_cpu_same_threads"] = round(e2e["mpkt_s"] / mc["value"], 3)
            if "one_thread_mpkt_s" in e2e and out.get("cpu_baseline"):
                e2e["ratio_one_thread_vs_cpu_one_core"] = round(e2e["one_thread_mpkt_s"] /
                                                                out["cpu_baseline"]["value"], 3)
            out["e2e"] = e2e
    group.barrier()   # the other ranks wait for rank 0's CPU legs

    if rank == 0:
        print(json.dumps(out), flush=True)
    gate.close()
    group.close()


def watchdog(seconds: float, rank: int):
    """End this rank with status 124 if it is still running after `seconds`
    (a daemon timer: a rank stuck in a collective whose peer died must not
    hold the node until the driver's own limit)."""
    import threading

    def fire():
        log(f"[rank {rank}] deadline of {seconds:.0f} s passed: exiting (124)")
        os._exit(124)

    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()


def dry_run(args, rank, world, local, W, secondaries):
    """The launch/rank protocol with the GPU leg stubbed: device checks,
    gloo rendezvous, the start gate and its window stamps, the RCCL unique-id
    broadcast and the counter reduction of rule-counter workloads (gloo sum
    standing in for the all-reduce, its mismatch reported, not asserted),
    fake timings, max over ranks, the per-rank gather, the secondary
    workloads and rank 0's one JSON line (CPU tests of --gpus N). Inside
    each window a rank sleeps its fake time: the windows' overlap is real."""
    if rank == args.dry_run_fail_rank:
        log(f"[rank {rank}] dry-run: failing on purpose")
        sys.exit(3)
    check_devices(args, world, local, args.dry_run_devices)
    dev = copdist.device_for(local, args.dry_run_devices)
    group = copdist.Group(rank, world, "gloo")
    gate = copdist.StartGate(group)

    def fake(name):
        Wn = WORKLOADS[name]
        B = Wn["batch"]
        rc_on = bool(Wn.get("rule_counters")) and not args.no_rule_counters
        coll, reduce_info = None, None
        if rc_on:
            uid = group.broadcast_bytes(bytes(range(128)) if rank == 0 else None)
            coll = "ok" if uid == bytes(range(128)) else "error: unique id differs"
        runs, own, reduced, windows = [], [], [], []
        for r in range(max(1, args.repeats)):
            group.barrier()
            t = 80e-3 * (1.0 + 0.01 * rank)   # rank r "takes" 80 (1 + r/100) ms per run
            t0 = gate.open()
            time.sleep(t)
            t1 = copdist.monotonic_ns()
            if rc_on:
                pk = (args.warmup if r == 0 else 0) + args.steps
                reduced.append(int(group.sum_u64(np.array([pk * B], np.uint64))[0]))
            own.append(t)
            windows.append((t0, t1))
            group.barrier()
            runs.append(group.max(t))
        if rc_on:
            want = [world * (args.warmup + args.steps) * B] + [world * args.steps * B] * (len(reduced) - 1)
            reduce_info = {"ranks": world, "pkts_reduced_per_interval": reduced, "expected_per_interval": want,
                           "ok": reduced == want}
        elapsed = float(np.median(runs))
        return {"B": B, "rc_on": rc_on, "coll": coll, "reduce_info": reduce_info, "own": own,
                "value": world * args.steps * B / elapsed / 1e6,
                "windows": copdist.window_stats(group.gather_obj(windows), world, args.steps * B)}

    res = fake(args.workload)
    info = group.gather_obj({"rank": rank, "device": dev,
                             "mpkt_s": round(args.steps * res["B"] / float(np.median(res["own"])) / 1e6, 3),
                             **({"rccl_init": res["coll"]} if res["rc_on"] else {})})
    sec = {}
    for sname in secondaries:
        sr = fake(sname)
        blk = {"value": round(sr["value"], 3), "windows_overlap": sr["windows"]["windows_overlap"],
               "value_union": round(sr["windows"]["value_union"], 3), "batch": sr["B"],
               "rule_counters": sr["rc_on"]}
        if sr["rc_on"]:
            blk["rccl_init"] = group.gather_obj(sr["coll"])
            blk["counter_reduce"] = sr["reduce_info"]
        sec[sname] = blk
    if rank == 0:
        line = {"metric": METRIC, "value": round(res["value"], 3), "unit": "Mpkt/s",
                "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "dry_run": True,
                "windows_overlap": res["windows"]["windows_overlap"],
                "value_union": round(res["windows"]["value_union"], 3), "windows": res["windows"],
                "config": {"workload": args.workload, "ranks": info}}
        if res["reduce_info"]:
            line["counter_reduce"] = res["reduce_info"]
        if sec:
            line["secondary"] = sec
        if not args.no_cpu:
            # the real CPU legs (oracle), on rank 0 at every N, as in a GPU run
            cid = W["cid"]
            fw_rules = cg.gen_rules(0x5EED1000 + cid, W["fw"], cg.GEN_FW, 20 if W["fw"] <= 1000 else 0)
            line.update(cpu_legs(args, W, fw_rules))
        print(json.dumps(line), flush=True)
    group.barrier()
    gate.close()
    group.close()


if __name__ == "__main__":
    main()
