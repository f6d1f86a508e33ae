"""GPU pipeline (through the C ABI) against the committed fixtures
(tests/golden/*.npz): g1 is the reference's own rules.json fixture; g2-g6
are oracle regression vectors (produced by oracle/cop_oracle.c, not by the
reference: see make_golden.py)."""
import glob
import os

import numpy as np
import pytest

import copgpu as cg
from helpers import gpu_run

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = sorted(glob.glob(os.path.join(HERE, "golden", "*.npz")))


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
@pytest.mark.parametrize("force_dir", [False, True])
def test_gpu_matches_golden(gpu_ctx_factory, path, force_dir):
    g = dict(np.load(path, allow_pickle=False))
    flags = (cg.CFG_FW_FORCE_DIR24 | cg.CFG_LPM_FORCE_DIR24) if force_dir else 0
    ctx = gpu_ctx_factory(stages=int(g["stages"]), flags=flags, routing_table=g["rt"])
    fw = np.zeros(len(g["fw_ip"]), dtype=cg.PREFIX_DT)
    fw["ip"], fw["depth"], fw["next_hop"] = g["fw_ip"], g["fw_depth"], g["fw_nh"]
    ctx.set_fw_table(cg.LpmTable(fw, int(g["fw_cfg"][0]), int(g["fw_cfg"][1]), bool(g["fw_cfg"][2])))
    if len(g["rt_ip"]):
        rt = np.zeros(len(g["rt_ip"]), dtype=cg.PREFIX_DT)
        rt["ip"], rt["depth"], rt["next_hop"] = g["rt_ip"], g["rt_depth"], g["rt_nh"]
        ctx.set_route_lpm(cg.LpmTable(rt, 1 << 20, 1 << 16, False))
    n = int(g["n"])
    offs = g["offsets"] if len(g["offsets"]) else None
    ctx.counters(reset=True)
    res, fwd, _ = gpu_run(ctx, g["pkts"], n, offsets=offs)
    assert np.array_equal(res.view(np.uint8).reshape(-1, 8), g["res"])
    assert np.array_equal(fwd, g["fwd"])
    c = ctx.counters()
    assert [c[k] for k in g["counter_names"]] == list(g["counters"])
