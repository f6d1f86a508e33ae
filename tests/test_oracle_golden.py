"""Oracle checks (CPU): the oracle against the committed golden fixtures,
against the reference's own fixture, and against an independent
brute-force LPM. Parity status: the reference has no golden vectors of its
own; the pinned part is reference_rules.json."""
import glob
import os

import numpy as np
import pytest

import oracle as orc

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = sorted(glob.glob(os.path.join(HERE, "golden", "*.npz")))


def load(path):
    return dict(np.load(path, allow_pickle=False))


def oracle_from_fixture(g):
    fw = orc.OracleLpm(int(g["fw_cfg"][0]), int(g["fw_cfg"][1]))
    if len(g["fw_ip"]):
        fw.setup(g["fw_ip"], g["fw_depth"], g["fw_nh"], stop_at_error=bool(g["fw_cfg"][2]))
    rt = orc.OracleLpm(1 << 20, 1 << 16)
    if len(g["rt_ip"]):
        rt.setup(g["rt_ip"], g["rt_depth"], g["rt_nh"], stop_at_error=False)
    return fw, rt


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_oracle_reproduces_golden(path):
    g = load(path)
    fw, rt = oracle_from_fixture(g)
    offs = g["offsets"] if len(g["offsets"]) else None
    res, fwd, cnt = orc.process(g["pkts"], int(g["n"]), offsets=offs, rt=g["rt"], stages=int(g["stages"]),
                                fw=fw, route=rt)
    assert np.array_equal(res.view(np.uint8).reshape(-1, 8), g["res"])
    assert np.array_equal(fwd, g["fwd"])
    assert [cnt[k] for k in g["counter_names"]] == list(g["counters"])


def test_reference_fixture_pins_accept_all():
    """engine/nfs/firewall/rules.json holds two rules, both action 0: the
    firewall forwards every IPv4 packet that reaches it (firewall.c:201-210
    maps next hop 0 to FW_FORWARD; a miss also yields next hop 0)."""
    g = load(os.path.join(HERE, "golden", "g1_reference_rules.npz"))
    v = g["res"][:, 0]
    reached = (v != 2) & (v != 4)
    assert reached.sum() > 1000
    assert np.all(v[reached] == 0)
    rules = orc.load_rules_json(os.path.join(HERE, "golden", "reference_rules.json"))
    assert rules == [((192 << 24) | (167 << 16) | (10 << 8), 24, 0), ((10 << 24) | (11 << 16) | (1 << 8) | 16, 32, 0)]


def test_fw_verdict_mapping():
    """firewall.c:196-210: the ret<0 DROP is overwritten by switch(rule):
    miss -> nh 0 -> FORWARD; hit with nh 0 -> FORWARD; hit nh != 0 -> DROP."""
    lpm = orc.OracleLpm(16, 4)
    assert lpm.add(0x0A000000, 8, 0) == 0
    assert lpm.add(0x0B000000, 8, 7) == 0
    pk = np.zeros(3 * 64, dtype=np.uint8)
    for i, src in enumerate([0x0A010203, 0x0B010203, 0x0C010203]):
        p = pk[i * 64:(i + 1) * 64]
        p[12], p[13], p[14] = 0x08, 0x00, 0x45
        p[26:30] = list(src.to_bytes(4, "big"))
        p[30:34] = [192, 167, 10, 1]
    res, fwd, _ = orc.process(pk, 3, stages=3, fw=lpm)
    assert list(res["verdict"]) == [0, 1, 0]
    assert list(res["flags"] & 2) == [2, 2, 0]
    assert list(fwd) == [0, 2]


def test_get_next_hop_and_route_table():
    rt = orc.route_table_default(5)
    assert list(rt[:5]) == [0xFFFF] * 5
    assert [rt[0x0A01 + i] for i in range(5)] == [0, 1, 2, 3, 4]
    assert rt[0x0A06] == 0 and rt[0xFFFF] == 0          # unknown dst -> vport 0 (init.c:51-53)
    pk = np.zeros(64, dtype=np.uint8)
    pk[12], pk[13] = 0x86, 0xDD
    assert orc.lib().orc_get_next_hop(pk.ctypes.data, rt.ctypes.data) == 0xFFFF
    pk[12], pk[13] = 0x08, 0x00
    pk[30:34] = [192, 167, 10, 3]
    assert orc.lib().orc_get_next_hop(pk.ctypes.data, rt.ctypes.data) == 2
    pk[32:34] = [0, 4]
    assert orc.lib().orc_get_next_hop(pk.ctypes.data, rt.ctypes.data) == 0xFFFF


def _random_rules(rng, n, depth_lo=1, depth_hi=32):
    ip = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    depth = rng.integers(depth_lo, depth_hi + 1, n).astype(np.uint8)
    nh = rng.integers(0, 2**24, n).astype(np.uint32)
    # nest some prefixes inside earlier ones
    for i in range(1, n, 3):
        j = rng.integers(0, i)
        d = depth[j]
        if d < depth[i]:
            m = np.uint32((0xFFFFFFFF << (32 - int(d))) & 0xFFFFFFFF)
            ip[i] = (ip[j] & m) | (ip[i] & ~m)
    return ip, depth, nh


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_incremental_dir24_equals_brute_force(seed):
    rng = np.random.default_rng(seed)
    ip, depth, nh = _random_rules(rng, 400)
    lpm = orc.OracleLpm(1024, 4096)
    first, _ = lpm.setup(ip, depth, nh, stop_at_error=False)
    assert first == -1
    rip, rd, rnh = lpm.rules()
    probes = np.concatenate([rng.integers(0, 2**32, 20000, dtype=np.uint64).astype(np.uint32),
                             rip, rip + 1, rip - 1,
                             (rip | ~np.uint32(0)).astype(np.uint32)])
    a_nh, a_hit = lpm.lookup(probes)
    b_nh, b_hit = orc.brute_lookup(rip, rd, rnh, probes)
    assert np.array_equal(a_nh, b_nh) and np.array_equal(a_hit, b_hit)


def test_rte_lpm_add_semantics():
    lpm = orc.OracleLpm(3, 1)
    assert lpm.add(1, 0, 1) < 0 and lpm.add(1, 33, 1) < 0          # -EINVAL
    assert lpm.add(0x0A0000FF, 8, 5) == 0                           # masked to 10.0.0.0/8
    assert lpm.add(0x0A123456, 8, 6) == 0                           # same rule: last write wins
    assert lpm.n_rules == 1
    assert lpm.lookup(np.array([0x0A999999], np.uint32))[0][0] == 6
    assert lpm.add(0x0B000000, 25, 1) == 0                          # takes the only tbl8 group
    assert lpm.add(0x0C000000, 25, 1) < 0                           # -ENOSPC: no tbl8 group
    assert lpm.n_rules == 2                                         # the failed rule is removed
    assert lpm.add(0x0B000080, 25, 2) == 0                          # same /24: no new group
    assert lpm.add(0x0D000000, 16, 1) < 0                           # -ENOSPC: max_rules 3
    assert lpm.add(0x0A000000, 8, 0x1FFFFFF) == 0                   # nh is 24 bits
    assert lpm.lookup(np.array([0x0A000001], np.uint32))[0][0] == 0xFFFFFF


def test_lpm_setup_stops_at_first_error():
    lpm = orc.OracleLpm(2, 24)
    first, err = lpm.setup(np.array([1 << 24, 2 << 24, 3 << 24, 4 << 24], np.uint32),
                           np.array([8, 8, 8, 8], np.uint8), np.array([1, 2, 3, 4], np.uint32))
    assert first == 2 and err < 0
    assert lpm.n_rules == 2


def test_oracle_python_rules_loader_edge_cases(tmp_path):
    f = tmp_path / "r.json"
    f.write_text('{"a": {"IP": " 1.2.3.4x", "Depth": 280, "ACTION": true},'
                 ' "b": {"ip": "300.1.1.-1", "depth": -1, "action": 2.9, "ip": "9.9.9.9"},'
                 ' "c": {"ip": "4294967297.0.0.1", "depth": "24", "action": null}}')
    r = orc.load_rules_json(str(f))
    assert r[0] == ((1 << 24) | (2 << 16) | (3 << 8) | 4, 280 & 0xFF, 1)
    assert r[1] == ((300 & 0xFF) << 24 | (1 << 16) | (1 << 8) | 0xFF, 0xFF, 2)
    assert r[2] == ((1 << 24) | 1, 0, 0)
