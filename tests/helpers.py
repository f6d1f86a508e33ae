"""Shared helpers for parity tests: run a trace through the GPU pipeline
(through the C ABI) and through the oracle, and compare bit for bit."""
import numpy as np

import copgpu as cg
import oracle as orc


def oracle_tables(fw_rules=None, routes=None, fw_cfg=(1024, 24, True), rt_cfg=(1 << 20, 1 << 16, False)):
    fw = orc.OracleLpm(fw_cfg[0], fw_cfg[1])
    if fw_rules is not None and len(fw_rules):
        fw.setup(fw_rules["ip"], fw_rules["depth"], fw_rules["next_hop"], stop_at_error=fw_cfg[2])
    rt = orc.OracleLpm(rt_cfg[0], rt_cfg[1])
    if routes is not None and len(routes):
        rt.setup(routes["ip"], routes["depth"], routes["next_hop"], stop_at_error=rt_cfg[2])
    return fw, rt


def gpu_run(ctx, pkts: np.ndarray, n: int, stride=64, offsets=None, batches=1, compact=True):
    """Upload, split into `batches` consecutive batches in one submit, return
    (results, forward-list, per-batch counts)."""
    dp = ctx.alloc(max(pkts.nbytes, 16))
    dp.upload(pkts)
    dres = ctx.alloc(max(n * 8, 16))
    dfwd = ctx.alloc(max(n * 4, 16))
    dcnt = ctx.alloc(16 * 4 * max(batches, 1))
    doff = None
    if offsets is not None:
        doff = ctx.alloc(max(offsets.nbytes, 16))
        doff.upload(offsets)
    dres.fill(0xAB)
    dcnt.fill(0xFF)
    bounds = np.linspace(0, n, batches + 1).astype(np.int64)
    bl = []
    for b in range(batches):
        lo, hi = int(bounds[b]), int(bounds[b + 1])
        if offsets is not None:
            # IMIX: per-batch offset slice, same slab
            bl.append(cg.make_batch(dp, hi - lo, dres, offsets=doff.addr + lo * 4,
                                    fwd_idx=(dfwd.addr + lo * 4) if compact else None,
                                    fwd_count=(dcnt.addr + b * 4) if compact else None,
                                    results_offset=lo * 8))
        else:
            bl.append(cg.make_batch(dp, hi - lo, dres, stride=stride, pkts_offset=lo * stride,
                                    fwd_idx=(dfwd.addr + lo * 4) if compact else None,
                                    fwd_count=(dcnt.addr + b * 4) if compact else None,
                                    results_offset=lo * 8))
    ctx.submit(bl)
    ctx.sync()
    res = dres.download(cg.RESULT_DT, n)
    counts = dcnt.download(np.uint32, batches)
    fwd_all = dfwd.download(np.uint32, n)
    fwd = []
    for b in range(batches):
        lo = int(bounds[b])
        c = int(counts[b]) if compact else 0
        fwd.append(fwd_all[lo: lo + c] + lo)
    fwd = np.concatenate(fwd) if fwd else np.zeros(0, np.uint32)
    for x in (dp, dres, dfwd, dcnt, doff):
        if x is not None:
            x.free()
    return res, fwd, counts


def assert_parity(res_gpu, fwd_gpu, res_orc, fwd_orc):
    for f in ("verdict", "flags", "port", "route_nh"):
        bad = np.nonzero(res_gpu[f] != res_orc[f])[0]
        assert bad.size == 0, (f"{f} mismatch at {bad[:10]}: gpu={res_gpu[f][bad[:10]]} "
                               f"oracle={res_orc[f][bad[:10]]}")
    assert np.array_equal(fwd_gpu, fwd_orc), f"forward list differs ({len(fwd_gpu)} vs {len(fwd_orc)})"
