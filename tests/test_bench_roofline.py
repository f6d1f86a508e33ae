"""bench.py's roofline blocks (CPU, no GPU): `roofline` describes the engine
behind `value` (config.engine). For the poll-mode kernel its `frac` is the
timed window's fraction and its traffic the kernel's PMC bytes per posted
batch scaled to the timed steps; the one-shot kernel's block, whose launch
time rocprofv3 checks, is `roofline_launch`. Inputs are a synthetic
measure() result on one rank (copdist.Group with world 1)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import copdist  # noqa: E402


class Args:
    steps = 20
    lists = "seg"


def fake_res(engine, traffic_pmd=True):
    B, bpp = 65536, 74.75
    res = {"name": "fw1k", "engine": engine, "B": B, "Lb": 1024, "bytes_per_pkt": bpp,
           "total_pkts": 20 * B, "elapsed": 24.3e-6,
           "alg_bytes": bpp * B * 1024, "mean_ms": 0.9, "n_launch": 8,
           "achieved": bpp * B * 1024 / 0.9e-3 / 1e9, "traffic": 5.05e9,
           "probes": {"sample_pkts": B}, "traffic_pmd": None}
    if traffic_pmd:
        res["traffic_pmd"] = {"per_batch": 4.938e6, "batches": 1024, "kernel": "cop_pmd<1, 0, 2, 4, false>",
                              "source": "bench_traffic/traffic_pmd_fw1k_seg.json"}
    return res


def test_pmd_roofline_is_the_timed_window():
    g = copdist.Group(0, 1)
    res = fake_res("pmd")
    r = bench.roofline_block(res, 1, g, Args)
    assert r["engine"] == "pmd"
    want = 74.75 * 20 * 65536 / 24.3e-6 / 1e9
    assert r["achieved"] == pytest.approx(want, rel=1e-3)
    assert r["frac"] == r["frac_timed"] == pytest.approx(want / bench.HBM_PEAK_GBS, abs=1e-4)
    # PMC bytes per posted batch x the timed steps, against the same steps' algorithmic bytes
    assert r["traffic"] == pytest.approx(4.938e6 * 20, rel=1e-6)
    assert r["traffic_per_algorithmic"] == pytest.approx(4.938e6 / (74.75 * 65536), abs=1e-4)
    assert r["kernel"].startswith("cop_pmd<")
    launch = bench.roofline_launch_block(res, 1, g, Args)
    assert launch["engine"] == "launch"
    assert launch["frac"] == pytest.approx(res["achieved"] / bench.HBM_PEAK_GBS, abs=1e-4)
    assert launch["traffic_per_algorithmic"] == pytest.approx(5.05e9 / res["alg_bytes"], abs=1e-4)


def test_launch_engine_roofline_keeps_frac_timed():
    g = copdist.Group(0, 1)
    res = fake_res("launch", traffic_pmd=False)
    r = bench.roofline_block(res, 1, g, Args)
    assert r["engine"] == "launch"
    assert r["frac"] == pytest.approx(res["achieved"] / bench.HBM_PEAK_GBS, abs=1e-4)
    assert r["frac_timed"] == pytest.approx(74.75 * 20 * 65536 / 24.3e-6 / 1e9 / bench.HBM_PEAK_GBS, abs=1e-4)


def test_pmd_roofline_without_pmc_says_so():
    g = copdist.Group(0, 1)
    r = bench.roofline_block(fake_res("pmd", traffic_pmd=False), 1, g, Args)
    assert r["traffic"] is None and r["traffic_per_algorithmic"] is None and r["traffic_source"] is None


def test_every_benched_workload_has_pmc_files():
    """The line's `traffic` is never null for the four workloads the
    driver's command times: both engines' PMC summaries are committed."""
    for name, W in bench.WORKLOADS.items():
        assert os.path.exists(os.path.join(bench.TRAFFIC_DIR, f"traffic_pmd_{name}_seg.json")), name
        assert os.path.exists(os.path.join(bench.TRAFFIC_DIR, f"traffic_{name}_L{W['per_launch']}_seg.json")), name
