"""rules.json loading: the product's C loader (cop_rules_load_json) against
the oracle's Python restatement of setup_rules/fw_config_parse_file
(firewall.c:57-105, 276-323) on the reference fixture and edge cases."""
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
