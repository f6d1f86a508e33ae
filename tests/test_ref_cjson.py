"""Loader parity pinned to the reference's own parser.

oracle/ref_cjson.py replays setup_rules (firewall.c:276-323) over the
reference's vendored cJSON 1.7.12, compiled from /root/reference into
oracle/_ref/ (`make -C oracle ref`). Both rules.json loaders — the
product's (csrc/rules_json.c, through the C ABI) and the oracle's Python
restatement — must produce exactly the reference's (src_ip, depth, action)
list on every input where the reference is defined; where the reference
calls rte_exit or reads an uninitialised field, both must report an error.
"""
import os

import numpy as np
import pytest

import copgpu as cg
import oracle as orc
import ref_cjson

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.skipif(not ref_cjson.available(),
                                reason="oracle/_ref not built (needs /root/reference: make -C oracle ref)")

R = '{"r": {"ip": "%s", "depth": %s, "action": %s}}'
EDGE = {
    "fixture_like": '{\n\t"rule1": {\n\t\t"ip": "192.168.10.0",\n\t\t"depth": 24,\n\t\t"action": 0\n\t}\n}\n',
    "key_case": '{"a": {"IP": "10.0.0.1", "Depth": 24, "ACTION": 3}, "b": {"iP": "10.0.0.2", "dEpTh": 8, "action": 1}}',
    "float_depth": R % ("10.1.2.3", "24.9", "1.5"),
    "neg_values": R % ("10.1.2.3", "-1", "-255"),
    "big_values": R % ("10.1.2.3", "300", "65537"),
    "exp_values": R % ("10.1.2.3", "1e1", "2.5E+2"),
    "int_overflow": R % ("10.1.2.3", "2147483648", "-2147483649"),
    "huge": R % ("10.1.2.3", "1e300", "-1e300"),
    "bool_null": '{"a": {"ip": "1.2.3.4", "depth": true, "action": false}, "b": {"ip": "1.2.3.5", "depth": null, "action": true}}',
    "string_numbers": R % ("10.1.2.3", '"24"', '"1"'),
    "array_values": R % ("10.1.2.3", "[24]", "{}"),
    "ip_spaces": R % (" 10.0.0.1", "24", "1"),
    "ip_inner_spaces": R % ("10. 0. 0. 1", "24", "1"),
    "ip_trailing": R % ("10.0.0.1junk", "24", "1"),
    "ip_wide_bytes": R % ("300.256.1000.4294967295", "24", "1"),
    "ip_signs": R % ("+1.-2.3.4", "24", "1"),
    "ip_leading_zeros": R % ("010.001.000.009", "24", "1"),
    "ip_escape": '{"r": {"ip": "10.0.0.\\u0031", "depth": 24, "action": 1}}',
    "dup_keys": '{"r": {"ip": "1.1.1.1", "ip": "2.2.2.2", "depth": 8, "depth": 16, "action": 1}}',
    "extra_keys": '{"r": {"note": "x", "ip": "1.1.1.1", "depth": 8, "action": 1, "more": [1, 2]}}',
    "top_array": '[{"ip": "1.1.1.1", "depth": 8, "action": 1}, {"ip": "2.2.2.2", "depth": 16, "action": 0}]',
    "crlf": '{\r\n"r": {\r\n"ip": "1.1.1.1",\r\n"depth": 8,\r\n"action": 1\r\n}\r\n}\r\n',
    "trailing_garbage": R % ("1.1.1.1", "8", "1") + " trailing",
    "empty_object": "{}",
    "nul_inside": R % ("1.1.1.1", "8", "1") + "\0" + '{"junk": ',
    # the reference rte_exits / reads garbage on these
    "syntax_error": '{"r": {"ip": "1.1.1.1", "depth": 8, "action": 1}',
    "missing_action": '{"r": {"ip": "1.1.1.1", "depth": 8}}',
    "rule_not_object": '{"r": 5}',
    "ip_not_string": R.replace('"%s"', '%s') % ("167772161", "24", "1"),
    "ip_three_parts": R % ("1.2.3", "24", "1"),
    "ip_empty": R % ("", "24", "1"),
}


def ref_result(path):
    try:
        return ("ok", ref_cjson.setup_rules(path))
    except (ref_cjson.RefExit, ref_cjson.RefUndefined) as e:
        return ("error", type(e).__name__)


def product_result(path):
    try:
        r = cg.rules_load_json(path)
    except cg.CopError:
        return ("error", None)
    return ("ok", [(int(x["ip"]), int(x["depth"]), int(x["next_hop"])) for x in r])


def oracle_result(path):
    try:
        return ("ok", orc.load_rules_json(path))
    except ValueError:
        return ("error", None)


def check(path):
    ref = ref_result(path)
    for name, got in (("product", product_result(path)), ("oracle", oracle_result(path))):
        assert got[0] == ref[0], (name, path, got, ref)
        if ref[0] == "ok":
            assert got[1] == ref[1], (name, path, got[1][:5], ref[1][:5])
    return ref


def test_reference_cjson_version():
    assert ref_cjson.version() == "1.7.12"


def test_reference_fixture():
    kind, rules = check(os.path.join(ROOT, "tests", "golden", "reference_rules.json"))
    assert kind == "ok" and len(rules) == 2


@pytest.mark.parametrize("name", sorted(EDGE))
def test_edge_files(tmp_path, name):
    p = tmp_path / f"{name}.json"
    p.write_bytes(EDGE[name].encode())
    kind, _ = check(str(p))
    assert (kind == "error") == (name in {"syntax_error", "missing_action", "rule_not_object", "ip_not_string",
                                          "ip_three_parts", "ip_empty"}), kind


@pytest.mark.parametrize("seed,n", [(0x5EED1002, 1000), (0x5EED1005, 20000)])
def test_generated_files(tmp_path, seed, n):
    rules = cg.gen_rules(seed, n, cg.GEN_FW, 20)
    p = str(tmp_path / "rules.json")
    cg.rules_write_json(p, rules)
    kind, got = check(p)
    assert kind == "ok"
    assert [r[0] for r in got] == [int(x) for x in rules["ip"]]
    assert [r[1] for r in got] == [int(x) for x in rules["depth"]]
    assert [r[2] for r in got] == [int(x) & 0xFF for x in rules["next_hop"]]


@pytest.mark.parametrize("base_name", ["fixture", "generated", "edge"])
def test_random_mutations(tmp_path, base_name):
    """Byte-level mutations of valid files: whatever the reference makes of
    each (rules, rte_exit or undefined), the loaders agree."""
    if base_name == "fixture":
        base = open(os.path.join(ROOT, "tests", "golden", "reference_rules.json"), "rb").read()
    elif base_name == "generated":
        p0 = str(tmp_path / "g.json")
        cg.rules_write_json(p0, cg.gen_rules(99, 12, cg.GEN_FW, 4))
        base = open(p0, "rb").read()
    else:
        base = ('\xef\xbb\xbf[{"IP": " 1.2.3.4", "depth": 1.5e1, "Action": -3},'
                ' {"ip": "9.8.7.\\u0036", "depth": true, "action": "x"}]').encode("latin-1")
    rng = np.random.default_rng({"fixture": 7, "generated": 8, "edge": 9}[base_name])
    alphabet = b'{}[]:,". 0123456789-+eE\ntruefalsn\\ipdepthactionuU\x00\x01\x0b\x1f\xef'
    for t in range(1000):
        b = bytearray(base)
        for _ in range(int(rng.integers(1, 4))):
            op = int(rng.integers(0, 3))
            pos = int(rng.integers(0, len(b)))
            if op == 0 and len(b) > 1:
                del b[pos]
            elif op == 1:
                b.insert(pos, alphabet[int(rng.integers(0, len(alphabet)))])
            else:
                b[pos] = alphabet[int(rng.integers(0, len(alphabet)))]
        p = tmp_path / f"m{t}.json"
        p.write_bytes(bytes(b))
        check(str(p))
