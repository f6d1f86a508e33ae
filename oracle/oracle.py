"""Python face of the oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module. It wraps liboracle.so (cop_oracle.c, the C
restatement of the reference path) and restates the rules.json loader of
firewall.c:57-105,276-323 in Python.

Parity status (see cop_oracle.c): pinned only by the reference's own
fixture engine/nfs/firewall/rules.json (tests/golden/); otherwise
"parity unpinned" — a restatement of the reference source cross-checked
against an independent brute-force LPM.
"""
from __future__ import annotations

import ctypes
import json
import os
from ctypes import POINTER, byref, c_double, c_int, c_uint8, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
INT_MAX, INT_MIN = 2**31 - 1, -(2**31)

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built (run make -C oracle)")
        L = ctypes.CDLL(LIB_PATH)
        sig = {
            "orc_route_table_default": (None, [c_void_p, c_uint32]),
            "orc_get_next_hop": (c_uint32, [c_void_p, c_void_p]),
            "orc_lpm_create": (c_void_p, [c_uint32, c_uint32]),
            "orc_lpm_create2": (c_void_p, [c_uint32, c_uint32, c_uint32]),
            "orc_lpm_match_rules": (None, [c_void_p, c_void_p, c_uint64, c_void_p]),
            "orc_lpm_free": (None, [c_void_p]),
            "orc_lpm_add": (c_int, [c_void_p, c_uint32, c_uint32, c_uint32]),
            "orc_lpm_lookup": (c_int, [c_void_p, c_uint32, POINTER(c_uint32)]),
            "orc_lpm_lookup_batch": (None, [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p]),
            "orc_lpm_n_rules": (c_uint32, [c_void_p]),
            "orc_lpm_tbl8_used": (c_uint32, [c_void_p]),
            "orc_lpm_rules": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint32]),
            "orc_lpm_setup": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint32, c_int, POINTER(c_int)]),
            "orc_brute_lookup": (None, [c_void_p, c_void_p, c_void_p, c_uint32, c_void_p, c_uint64, c_void_p,
                                        c_void_p]),
            "orc_process": (c_uint32, [c_void_p, c_void_p, c_uint64, c_uint32, c_void_p, c_uint32, c_uint32,
                                       c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
            "orc_coprocessor_bench": (c_double, [c_void_p, c_uint64, c_void_p, c_double, c_int, c_int,
                                                 POINTER(c_uint64), POINTER(c_double)]),
        }
        for k, (r, a) in sig.items():
            f = getattr(L, k)
            f.restype = r
            f.argtypes = a
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(c_void_p) if a is not None else None


class OracleLpm:
    """Incremental DIR-24-8 restatement of DPDK 17.11 rte_lpm.

    rules_only=True keeps the rule hash and tbl8 accounting but no DIR-24-8
    image (lookups by hash probes, depth 32 down): the 1M-rule form."""

    def __init__(self, max_rules=1024, number_tbl8s=24, rules_only=False):
        self.h = lib().orc_lpm_create2(max_rules, number_tbl8s, 1 if rules_only else 0)
        if not self.h:
            raise MemoryError("orc_lpm_create")

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_lpm_free(self.h)
            self.h = None

    def add(self, ip, depth, nh) -> int:
        return lib().orc_lpm_add(self.h, ip & 0xFFFFFFFF, depth, nh & 0xFFFFFFFF)

    def setup(self, ip, depth, nh, stop_at_error=True):
        """lpm_setup: returns (index of first failed rule or -1, errno)."""
        ip = np.ascontiguousarray(ip, dtype=np.uint32)
        depth = np.ascontiguousarray(depth, dtype=np.uint8)
        nh = np.ascontiguousarray(nh, dtype=np.uint32)
        err = c_int(0)
        first = lib().orc_lpm_setup(self.h, _p(ip), _p(depth), _p(nh), len(ip), 1 if stop_at_error else 0,
                                    byref(err))
        return first, err.value

    def lookup(self, ips: np.ndarray):
        ips = np.ascontiguousarray(ips, dtype=np.uint32)
        nh = np.zeros(len(ips), dtype=np.uint32)
        hit = np.zeros(len(ips), dtype=np.uint8)
        lib().orc_lpm_lookup_batch(self.h, _p(ips), len(ips), _p(nh), _p(hit))
        return nh, hit

    @property
    def n_rules(self):
        return lib().orc_lpm_n_rules(self.h)

    @property
    def tbl8_used(self):
        return lib().orc_lpm_tbl8_used(self.h)

    def rules(self):
        n = self.n_rules
        ip = np.zeros(n, dtype=np.uint32)
        d = np.zeros(n, dtype=np.uint8)
        nh = np.zeros(n, dtype=np.uint32)
        lib().orc_lpm_rules(self.h, _p(ip), _p(d), _p(nh), n)
        order = np.lexsort((d, ip))
        return ip[order], d[order], nh[order]

    def rules_by_id(self):
        """Accepted rules indexed by rule id (first-acceptance order)."""
        n = self.n_rules
        ip = np.zeros(n, dtype=np.uint32)
        d = np.zeros(n, dtype=np.uint8)
        nh = np.zeros(n, dtype=np.uint32)
        lib().orc_lpm_rules(self.h, _p(ip), _p(d), _p(nh), n)
        return ip, d, nh

    def match_rules(self, ips: np.ndarray) -> np.ndarray:
        """Matching rule id per address by hash probes (-1 on a miss)."""
        ips = np.ascontiguousarray(ips, dtype=np.uint32)
        out = np.zeros(len(ips), dtype=np.int32)
        lib().orc_lpm_match_rules(self.h, _p(ips), len(ips), _p(out))
        return out


def brute_lookup(rip, rdepth, rnh, ips):
    rip = np.ascontiguousarray(rip, dtype=np.uint32)
    rdepth = np.ascontiguousarray(rdepth, dtype=np.uint8)
    rnh = np.ascontiguousarray(rnh, dtype=np.uint32)
    ips = np.ascontiguousarray(ips, dtype=np.uint32)
    nh = np.zeros(len(ips), dtype=np.uint32)
    hit = np.zeros(len(ips), dtype=np.uint8)
    lib().orc_brute_lookup(_p(rip), _p(rdepth), _p(rnh), len(rip), _p(ips), len(ips), _p(nh), _p(hit))
    return nh, hit


def route_table_default(n_ports=5):
    rt = np.zeros(65536, dtype=np.uint16)
    lib().orc_route_table_default(_p(rt), n_ports)
    return rt


RESULT_DT = np.dtype([("verdict", "u1"), ("flags", "u1"), ("port", "<u2"), ("route_nh", "<u4")])


def process(pkts: np.ndarray, n: int, *, stride=64, offsets=None, rt=None, n_ports=5, stages=3,
            fw: OracleLpm | None = None, route: OracleLpm | None = None, rule_hits: np.ndarray | None = None):
    """Per-packet contract over one batch -> (results, forward list, counters).
    rule_hits (u64[fw.n_rules], optional) accumulates FW hits per rule id."""
    if rt is None:
        rt = route_table_default(n_ports)
    if rule_hits is not None:
        assert fw is not None and rule_hits.dtype == np.uint64 and len(rule_hits) >= fw.n_rules
    fw = fw or OracleLpm(1, 1)
    route = route or OracleLpm(1, 1)
    res = np.zeros(n, dtype=RESULT_DT)
    fwd = np.zeros(max(n, 1), dtype=np.uint32)
    cnt = np.zeros(16, dtype=np.uint64)
    offs = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint32)
    k = lib().orc_process(_p(pkts), _p(offs), stride, n, _p(rt), n_ports, stages, fw.h, route.h, _p(res),
                          _p(fwd), _p(cnt), _p(rule_hits))
    names = ["pkt_drop", "pkt_accept", "pkt_not_ipv4", "pkt_total", "parse_err", "no_port", "forward",
             "route_hit", "rx"]
    return res, fwd[:k], {nm: int(cnt[i]) for i, nm in enumerate(names)}


def coprocessor_bench(trace64: np.ndarray, n_trace: int, fw: OracleLpm, budget_s: float, nthreads=1,
                      first_cpu=-1):
    """Timed CPU coprocessor() loop -> (Mpkt/s aggregate, packets, seconds)."""
    pk = c_uint64(0)
    secs = c_double(0)
    rate = lib().orc_coprocessor_bench(_p(trace64), n_trace, fw.h, budget_s, nthreads, first_cpu, byref(pk),
                                       byref(secs))
    return rate, pk.value, secs.value


# ---------------------------------------------------------------------------
# rules.json loader restatement (firewall.c:57-105, 276-323, cJSON 1.7.12)

def _sscanf_u(s: str, i: int):
    """One glibc %u conversion: skip whitespace, optional sign, decimal digits."""
    n = len(s)
    while i < n and s[i] in " \t\n\v\f\r":
        i += 1
    neg = False
    if i < n and s[i] in "+-":
        neg = s[i] == "-"
        i += 1
    j = i
    while j < n and s[j].isdigit() and s[j] in "0123456789":
        j += 1
    if j == i:
        return None, i
    v = int(s[i:j])
    if v > 2**64 - 1:
        v = 2**64 - 1          # strtoul saturates
    elif neg:
        v = (-v) % 2**64
    return v & 0xFFFFFFFF, j  # stored through unsigned int


def parse_ip(s: str):
    """sscanf(ip_str, "%u.%u.%u.%u") == 4 ? RTE_IPV4(...) : None."""
    vals, i = [], 0
    for k in range(4):
        if k:
            if i >= len(s) or s[i] != ".":
                return None
            i += 1
        v, i = _sscanf_u(s, i)
        if v is None:
            return None
        vals.append(v)
    return ((vals[0] & 0xFF) << 24) | ((vals[1] & 0xFF) << 16) | ((vals[2] & 0xFF) << 8) | (vals[3] & 0xFF)


def _valueint(v):
    if v is True:
        return 1
    if isinstance(v, bool) or v is None or not isinstance(v, (int, float)):
        return 0
    if v >= INT_MAX:
        return INT_MAX
    if v <= INT_MIN:
        return INT_MIN
    return int(v)


def load_rules_json(path: str):
    """-> list of (ip, depth, action) with the reference's field semantics."""
    with open(path, "rb") as f:
        text = f.read().split(b"\0", 1)[0].decode("utf-8", errors="surrogateescape")
    root = json.loads(text, object_pairs_hook=lambda pairs: ("__obj__", pairs))
    children = root[1] if isinstance(root, tuple) else (root if isinstance(root, list) else [])
    if isinstance(root, tuple):
        children = [v for _, v in children]
    out = []
    for c in children:
        if not (isinstance(c, tuple) and c[0] == "__obj__"):
            raise ValueError("rule is not an object")
        pairs = c[1]

        def get(key):
            for k, v in pairs:
                if k.lower() == key:
                    return v, True
            return None, False
        ip, h1 = get("ip")
        depth, h2 = get("depth")
        action, h3 = get("action")
        if not (h1 and h2 and h3) or not isinstance(ip, str):
            raise ValueError("missing key / non-string ip")
        v = parse_ip(ip)
        if v is None:
            raise ValueError(f"bad ip {ip!r}")
        out.append((v, _valueint(depth) & 0xFF, _valueint(action) & 0xFF))
    return out
