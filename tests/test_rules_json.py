"""rules.json loading: the product's C loader (cop_rules_load_json) against
the oracle's Python restatement of setup_rules/fw_config_parse_file
(firewall.c:57-105, 276-323) on the reference fixture and edge cases."""
import errno
import os

import numpy as np
import pytest

import copgpu as cg
import oracle as orc

HERE = os.path.dirname(os.path.abspath(__file__))


def both(path):
    a = cg.rules_load_json(path)
    b = orc.load_rules_json(path)
    return [(int(r["ip"]), int(r["depth"]), int(r["next_hop"])) for r in a], b


def test_reference_fixture():
    a, b = both(os.path.join(HERE, "golden", "reference_rules.json"))
    assert a == b and len(a) == 2


CASES = {
    "case_keys": '{"r": {"IP": "1.2.3.4", "DePtH": 24, "Action": 3}}',
    "dup_keys_first_wins": '{"r": {"ip": "1.2.3.4", "ip": "5.6.7.8", "depth": 8, "depth": 9, "action": 1}}',
    "uint8_trunc": '{"r": {"ip": "1.2.3.4", "depth": 280, "action": 513}}',
    "valueint_forms": '{"a": {"ip": "1.1.1.1", "depth": true, "action": false},'
                      ' "b": {"ip": "1.1.1.1", "depth": 24.9, "action": -3},'
                      ' "c": {"ip": "1.1.1.1", "depth": "24", "action": null},'
                      ' "d": {"ip": "1.1.1.1", "depth": 1e12, "action": -1e12}}',
    "sscanf_ip": '{"a": {"ip": " 1.2.3.4junk", "depth": 8, "action": 0},'
                 ' "b": {"ip": "256.257.-1.4294967297", "depth": 8, "action": 0},'
                 ' "c": {"ip": "+1.+2.3.4", "depth": 8, "action": 0}}',
    "array_root": '[{"ip": "9.8.7.6", "depth": 16, "action": 4}]',
    "empty": "{}",
    "escapes": '{"r\\u00e9": {"ip": "1.2.3.4", "depth": 8, "action": 1}}',
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_loader_cases(tmp_path, name):
    f = tmp_path / "rules.json"
    f.write_text(CASES[name])
    a, b = both(str(f))
    assert a == b


@pytest.mark.parametrize("text", [
    '{"r": {"ip": "1.2.3", "depth": 8, "action": 1}}',      # sscanf != 4
    '{"r": {"ip": 5, "depth": 8, "action": 1}}',            # ip not a string
    '{"r": {"depth": 8, "action": 1}}',                     # missing key (reference rte_exits)
    '{"r": [1, 2]}',                                        # rule not an object
    '{"r": {"ip": "1.2.3.4", "depth": 8, "action": 1}',     # syntax
])
def test_loader_errors(tmp_path, text):
    f = tmp_path / "rules.json"
    f.write_text(text)
    with pytest.raises(cg.CopError):
        cg.rules_load_json(str(f))
    with pytest.raises(Exception):
        orc.load_rules_json(str(f))


def test_missing_file():
    with pytest.raises(cg.CopError):
        cg.rules_load_json("/nonexistent/rules.json")


def test_write_roundtrip_short_lines(tmp_path):
    rules = cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)
    f = tmp_path / "rules.json"
    cg.rules_write_json(str(f), rules)
    assert max(len(line) for line in f.read_text().splitlines()) < 255   # firewall.c:72 fgets buffer
    a, b = both(str(f))
    assert a == b
    assert a == [(int(r["ip"]), int(r["depth"]), int(r["next_hop"])) for r in rules]
    back = cg.rules_load_json(str(f))
    assert np.array_equal(back["ip"], rules["ip"])


# ---- binary prefix dumps (cop_rules_load_bin / cop_rules_write_bin) ----

def test_bin_round_trip_1m(tmp_path):
    rules = cg.gen_rules(0x5EED1005, 1000000, cg.GEN_FW, 0)
    p = str(tmp_path / "fw1m.bin")
    cg.rules_write_bin(p, rules)
    assert os.path.getsize(p) == 16 + 12 * len(rules)
    back = cg.rules_load_bin(p)
    for f in ("ip", "depth", "next_hop"):
        assert np.array_equal(back[f], rules[f])
    # the same table as from the in-memory rules (file order kept)
    a = cg.LpmTable(rules[:50000], 50000, 1 << 16, False)
    b = cg.LpmTable(back[:50000], 50000, 1 << 16, False)
    assert np.array_equal(a.rules(), b.rules())


def test_bin_matches_json(tmp_path):
    rules = cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)
    pj, pb = str(tmp_path / "r.json"), str(tmp_path / "r.bin")
    cg.rules_write_json(pj, rules)
    cg.rules_write_bin(pb, rules)
    j, b = cg.rules_load_json(pj), cg.rules_load_bin(pb)
    for f in ("ip", "depth", "next_hop"):
        assert np.array_equal(j[f], b[f])


def test_bin_empty_and_errors(tmp_path):
    p = str(tmp_path / "e.bin")
    cg.rules_write_bin(p, np.zeros(0, dtype=cg.PREFIX_DT))
    assert len(cg.rules_load_bin(p)) == 0
    good = str(tmp_path / "g.bin")
    cg.rules_write_bin(good, cg.gen_rules(1, 10, cg.GEN_FW, 0))
    raw = open(good, "rb").read()
    cases = {
        "magic": b"XPRB" + raw[4:],
        "version": raw[:4] + (2).to_bytes(4, "little") + raw[8:],
        "truncated": raw[:-1],
        "trailing": raw + b"\0",
        "count": raw[:8] + (11).to_bytes(8, "little") + raw[16:],
        "short_header": raw[:10],
    }
    for name, data in cases.items():
        q = str(tmp_path / f"{name}.bin")
        open(q, "wb").write(data)
        with pytest.raises(cg.CopError) as ei:
            cg.rules_load_bin(q)
        assert ei.value.code == -errno.EINVAL, name
    with pytest.raises(cg.CopError) as ei:
        cg.rules_load_bin(str(tmp_path / "missing.bin"))
    assert ei.value.code == -errno.ENOENT
