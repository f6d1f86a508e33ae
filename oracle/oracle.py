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
import os
import re
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
            # dpdk_lpm_v1604.c: the literal rules_tbl / rule_info restatement
            "dl_lpm_create": (c_void_p, [c_uint32, c_uint32]),
            "dl_lpm_free": (None, [c_void_p]),
            "dl_lpm_add": (c_int, [c_void_p, c_uint32, c_uint32, c_uint32]),
            "dl_lpm_lookup_batch": (None, [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p]),
            "dl_lpm_setup": (ctypes.c_int64, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_int,
                                              POINTER(ctypes.c_int32), c_void_p]),
            "dl_lpm_n_rules": (c_uint32, [c_void_p]),
            "dl_lpm_tbl8_used": (c_uint32, [c_void_p]),
            "dl_lpm_rule_info": (None, [c_void_p, c_void_p, c_void_p]),
            "dl_lpm_rules": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint32]),
        }
        for k, (r, a) in sig.items():
            f = getattr(L, k)
            f.restype = r
            f.argtypes = a
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(c_void_p) if a is not None else None


class DpdkLpm:
    """The literal restatement of DPDK 17.11 rte_lpm's v1604 add path
    (oracle/dpdk_lpm_v1604.c): rules_tbl grouped by depth with
    rule_info[depth-1] = {used_rules, first_rule}, rule_add_v1604 /
    rule_delete_v1604, tbl8_alloc_v1604, add_depth_small/big_v1604."""

    def __init__(self, max_rules=1024, number_tbl8s=24):
        self.h = lib().dl_lpm_create(max_rules, number_tbl8s)
        if not self.h:
            raise MemoryError("dl_lpm_create")

    def __del__(self):
        if getattr(self, "h", None):
            lib().dl_lpm_free(self.h)
            self.h = None

    def add(self, ip, depth, nh) -> int:
        return lib().dl_lpm_add(self.h, ip & 0xFFFFFFFF, depth, nh & 0xFFFFFFFF)

    def setup(self, ip, depth, nh, stop_at_error=True):
        """lpm_setup's loop: (index of the first failed add or -1, its errno,
        every add's return code; -9999 = never presented)."""
        ip = np.ascontiguousarray(ip, dtype=np.uint32)
        depth = np.ascontiguousarray(depth, dtype=np.uint8)
        nh = np.ascontiguousarray(nh, dtype=np.uint32)
        rc = np.zeros(len(ip), dtype=np.int32)
        err = ctypes.c_int32(0)
        first = lib().dl_lpm_setup(self.h, _p(ip), _p(depth), _p(nh), len(ip), 1 if stop_at_error else 0,
                                   byref(err), _p(rc))
        return int(first), err.value, rc

    def lookup(self, ips: np.ndarray):
        ips = np.ascontiguousarray(ips, dtype=np.uint32)
        nh = np.zeros(len(ips), dtype=np.uint32)
        hit = np.zeros(len(ips), dtype=np.uint8)
        lib().dl_lpm_lookup_batch(self.h, _p(ips), len(ips), _p(nh), _p(hit))
        return nh, hit

    @property
    def n_rules(self):
        return lib().dl_lpm_n_rules(self.h)

    @property
    def tbl8_used(self):
        return lib().dl_lpm_tbl8_used(self.h)

    def rule_info(self):
        used = np.zeros(32, dtype=np.uint32)
        first = np.zeros(32, dtype=np.uint32)
        lib().dl_lpm_rule_info(self.h, _p(used), _p(first))
        return used, first

    def rules(self):
        """(ip, depth, nh) in rules_tbl order: grouped by depth."""
        n = self.n_rules
        ip = np.zeros(n, dtype=np.uint32)
        d = np.zeros(n, dtype=np.uint8)
        nh = np.zeros(n, dtype=np.uint32)
        k = lib().dl_lpm_rules(self.h, _p(ip), _p(d), _p(nh), n)
        assert k == n
        return ip, d, nh


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


# cJSON 1.7.12 parser restatement (engine/thirdparty/cJSON.c): the grammar
# the reference's rules loader actually accepts. Values are tuples:
# ("obj", [(key, value), ...]) / ("arr", [...]) / ("str", bytes) /
# ("num", float) / ("true",) / ("false",) / ("null",).

class _CjsonFail(Exception):
    pass


_NUM_CHARS = b"0123456789+-eE."
_STRTOD = re.compile(rb"[+-]?(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?")


class _CjsonParser:
    def __init__(self, data: bytes):
        self.b = data + b"\0"          # buffer.length = strlen + 1 (cJSON_ParseWithOpts)
        self.n = len(self.b)
        self.i = 0
        self.depth = 0

    def ws(self):                       # buffer_skip_whitespace: every byte <= 32
        while self.i < self.n and self.b[self.i] <= 32:
            self.i += 1
        if self.i == self.n:
            self.i -= 1

    def at(self, k=0):
        return self.b[self.i + k] if self.i + k < self.n else None

    def value(self):                    # parse_value
        b, i = self.b, self.i
        for lit, v in ((b"null", ("null",)), (b"false", ("false",)), (b"true", ("true",))):
            if i + len(lit) <= self.n and b.startswith(lit, i):
                self.i += len(lit)
                return v
        c = self.at()
        if c == 0x22:
            return ("str", self.string())
        if c is not None and (c == 0x2D or 0x30 <= c <= 0x39):
            return self.number()
        if c == 0x5B:
            return self.container(0x5B, 0x5D)
        if c == 0x7B:
            return self.container(0x7B, 0x7D)
        raise _CjsonFail

    def number(self):                   # parse_number: strtod over <= 63 number chars
        j = self.i
        while j < self.n and j - self.i < 63 and self.b[j] in _NUM_CHARS:
            j += 1
        m = _STRTOD.match(self.b[self.i:j])
        if not m:
            raise _CjsonFail
        self.i += m.end()
        return ("num", float(m.group(0)))

    def string(self):                   # parse_string (+ utf16_literal_to_utf8)
        b = self.b
        if b[self.i] != 0x22:
            raise _CjsonFail
        end = self.i + 1
        while end < self.n and b[end] != 0x22:
            if b[end] == 0x5C:
                if end + 1 >= self.n:
                    raise _CjsonFail
                end += 1
            end += 1
        if end >= self.n or b[end] != 0x22:
            raise _CjsonFail
        out = bytearray()
        p = self.i + 1
        esc = {ord("b"): 8, ord("f"): 12, ord("n"): 10, ord("r"): 13, ord("t"): 9, 0x22: 0x22, 0x5C: 0x5C, 0x2F: 0x2F}
        while p < end:
            if b[p] != 0x5C:
                out.append(b[p])
                p += 1
                continue
            c = b[p + 1]
            if c in esc:
                out.append(esc[c])
                p += 2
            elif c == ord("u"):
                if end - p < 6:
                    raise _CjsonFail
                first = _hex4(b[p + 2:p + 6])
                if 0xDC00 <= first <= 0xDFFF:
                    raise _CjsonFail
                if 0xD800 <= first <= 0xDBFF:
                    q = p + 6
                    if end - q < 6 or b[q] != 0x5C or b[q + 1] != ord("u"):
                        raise _CjsonFail
                    second = _hex4(b[q + 2:q + 6])
                    if not 0xDC00 <= second <= 0xDFFF:
                        raise _CjsonFail
                    cp = 0x10000 + (((first & 0x3FF) << 10) | (second & 0x3FF))
                    p += 12
                else:
                    cp = first
                    p += 6
                out += chr(cp).encode("utf-8", errors="surrogatepass")
            else:
                raise _CjsonFail
        self.i = end + 1
        return bytes(out).split(b"\0", 1)[0]    # valuestring is a C string

    def container(self, open_c, close_c):   # parse_array / parse_object
        if self.depth >= 1000:              # CJSON_NESTING_LIMIT
            raise _CjsonFail
        self.depth += 1
        is_obj = open_c == 0x7B
        items = []
        self.i += 1
        self.ws()
        if self.at() == close_c:
            self.i += 1
            self.depth -= 1
            return ("obj" if is_obj else "arr", items)
        self.i -= 1
        while True:
            self.i += 1
            self.ws()
            if is_obj:
                if self.at() != 0x22:
                    raise _CjsonFail
                key = self.string()
                self.ws()
                if self.at() != 0x3A:
                    raise _CjsonFail
                self.i += 1
                self.ws()
                items.append((key, self.value()))
            else:
                items.append(self.value())
            self.ws()
            if self.at() != 0x2C:
                break
        if self.at() != close_c:
            raise _CjsonFail
        self.i += 1
        self.depth -= 1
        return ("obj" if is_obj else "arr", items)


def _hex4(h: bytes) -> int:             # parse_hex4: 0 on any invalid digit
    try:
        return int(h.decode("ascii"), 16) if len(h) == 4 and all(c in b"0123456789abcdefABCDEF" for c in h) else 0
    except ValueError:
        return 0


def cjson_parse(data: bytes):
    """cJSON_Parse: BOM, whitespace, one value; trailing bytes ignored. None on failure."""
    p = _CjsonParser(data)
    if p.n > 4 and p.b.startswith(b"\xEF\xBB\xBF"):
        p.i = 3
    p.ws()
    try:
        return p.value()
    except (_CjsonFail, IndexError):
        return None


def _valueint(v):
    """cJSON valueint: saturated (int) of a number, 1 for true, else 0."""
    if v[0] == "num":
        x = v[1]
        if x >= INT_MAX:
            return INT_MAX
        if x <= INT_MIN:
            return INT_MIN
        return int(x)
    return 1 if v[0] == "true" else 0


def _get_object_item(item, key: bytes):
    """cJSON_GetObjectItem: first child whose name matches case-insensitively
    (ASCII tolower); array elements have no name and never match."""
    if item[0] != "obj":
        return None
    for k, v in item[1]:
        if k.lower() == key:
            return v
    return None


def load_rules_json(path: str):
    """setup_rules (firewall.c:276-323) over the cJSON restatement ->
    list of (ip, depth, action); ValueError where the reference calls
    rte_exit or leaves src_ip uninitialised (fw_pkt_parse_ip failure)."""
    with open(path, "rb") as f:
        data = f.read().split(b"\0", 1)[0]       # json_str is a C string
    root = cjson_parse(data)
    if root is None:
        raise ValueError("could not be parsed")
    children = [v for _, v in root[1]] if root[0] == "obj" else (root[1] if root[0] == "arr" else [])
    out = []
    for c in children:
        ip, depth, action = (_get_object_item(c, k) for k in (b"ip", b"depth", b"action"))
        if ip is None or depth is None or action is None:
            raise ValueError("IP/Depth/Action not found")
        v = parse_ip(ip[1].decode("utf-8", errors="surrogateescape")) if ip[0] == "str" else None
        if v is None:
            raise ValueError(f"bad ip {ip!r}")
        out.append((v, _valueint(depth) & 0xFF, _valueint(action) & 0xFF))
    return out
