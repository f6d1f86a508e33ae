"""Synthetic workload generator: determinism, frame format
at the offsets the reference reads, traffic mix, IMIX layout."""
import numpy as np

import copgpu as cg


def test_deterministic():
    a = cg.gen_rules(1, 500, cg.GEN_FW, 20)
    b = cg.gen_rules(1, 500, cg.GEN_FW, 20)
    assert np.array_equal(a, b)
    t1 = cg.gen_trace(7, 1000, a)
    t2 = cg.gen_trace(7, 1000, a)
    assert np.array_equal(t1, t2)
    assert not np.array_equal(t1, cg.gen_trace(8, 1000, a))


def test_fw_rule_mix():
    r = cg.gen_rules(0x5EED1002, 20000, cg.GEN_FW, 20)
    d = r["depth"]
    assert abs((d == 24).mean() - 0.60) < 0.02
    assert abs(((d >= 16) & (d <= 23)).mean() - 0.20) < 0.02
    assert abs(((d >= 8) & (d <= 15)).mean() - 0.10) < 0.02
    long_ = d > 24
    assert abs(long_.mean() - 0.10) < 0.02
    assert len(np.unique(r["ip"][long_] >> 8)) <= 20      # fits number_tbl8s = 24
    assert abs((r["next_hop"] == 0).mean() - 0.5) < 0.02
    assert r["next_hop"].max() <= 255


def test_route_mix():
    r = cg.gen_rules(0x5EED2003, 20000, cg.GEN_ROUTES, 0)
    d = r["depth"]
    assert abs((d == 24).mean() - 0.55) < 0.02
    assert r["next_hop"].min() >= 1 and r["next_hop"].max() < (1 << 24)


def test_frame_format_and_mix():
    fw = cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)
    n = 50000
    t = cg.gen_trace(0x5EED0002, n, fw).reshape(n, 64)
    et = (t[:, 12].astype(np.uint32) << 8) | t[:, 13]
    assert abs((et == 0x86DD).mean() - 0.02) < 0.005
    assert set(np.unique(et)) == {0x0800, 0x86DD}
    assert np.all(t[:, 14] == 0x45)
    # IPv4 header checksum over bytes 14..33 sums to 0xFFFF
    words = (t[:, 14:34:2].astype(np.uint32) << 8) | t[:, 15:34:2]
    s = words.sum(axis=1)
    while (s >> 16).any():
        s = (s & 0xFFFF) + (s >> 16)
    assert np.all(s == 0xFFFF)
    dst = (t[:, 30].astype(np.uint32) << 24) | (t[:, 31].astype(np.uint32) << 16) | (t[:, 32].astype(np.uint32) << 8) | t[:, 33]
    vport = (dst >> 8) == ((192 << 16) | (167 << 8) | 10)
    assert abs(vport.mean() - 0.60) < 0.01
    assert abs(((dst & 0xFFFF) <= 4).mean() - 0.05) < 0.01


def test_imix_layout():
    slab, offs = cg.gen_imix(3, 12000)
    assert np.all(offs % 64 == 0)
    sizes = np.diff(np.append(offs, offs[-1] + 64))
    tl = np.array([(int(slab[o + 16]) << 8) | int(slab[o + 17]) for o in offs]) + 14   # IPv4 total length + 14
    assert set(np.unique(tl)) == {64, 594, 1518}
    frac = [(tl == s).mean() for s in (64, 594, 1518)]
    assert abs(frac[0] - 7 / 12) < 0.02 and abs(frac[1] - 4 / 12) < 0.02
    assert np.all(sizes[:-1] >= tl[:-1])
