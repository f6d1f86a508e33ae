"""ctypes binding of libcopgpu.so (the C ABI in include/cop_gpu.h).

This is the Python face of the drop-in boundary: tests and bench.py call
the HIP pipeline only through these C entry points. There is no CPU
fallback: if libcopgpu.so is missing, importing this module raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, Structure, byref, c_char_p, c_double, c_int, c_int32,
                    c_size_t, c_uint8, c_uint16, c_uint32, c_uint64, c_void_p)

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libcopgpu.so")

# ---------------------------------------------------------------------------
# constants (include/cop_gpu.h)
STAGE_PARSE, STAGE_FW, STAGE_LPM = 0x1, 0x2, 0x4
FORWARD, DROP_FW, DROP_PARSE, DROP_NOT_IPV4, DROP_NO_PORT = 0, 1, 2, 3, 4
FLAG_ROUTE_HIT, FLAG_FW_HIT = 0x1, 0x2
COUNTER_SHARDS = 256   # COP_COUNTER_SHARDS
LPM_STOP_AT_FIRST_ERROR = 0x1
CFG_FW_FORCE_DIR24, CFG_LPM_FORCE_DIR24, CFG_NO_COMPACT, CFG_RULE_COUNTERS = 0x1, 0x2, 0x4, 0x8
CFG_DEMUX_PORTS, CFG_PORT_STATS, CFG_LPM_TRIE, CFG_SEG_LISTS = 0x10, 0x20, 0x40, 0x80
CFG_LPM_BKT = 0x100
CFG_FW_BKT = 0x200
SEG_PKTS = 256   # COP_SEG_PKTS: packets per forward-list segment (CFG_SEG_LISTS)
MAX_DEMUX_PORTS = 8
GEN_FW, GEN_ROUTES = 0, 1
UNKNOWN_PORT = 0xFFFF
HDR16_STRIDE = 16   # packed header records: frame bytes 12..15 + 24..35 per packet
HDR12_STRIDE = 12   # compact records (one-shot batches): frame bytes 12..15 + 26..33 per packet

PREFIX_DT = np.dtype([("ip", "<u4"), ("next_hop", "<u4"), ("depth", "u1"), ("_pad", "u1", (3,))])
RESULT_DT = np.dtype([("verdict", "u1"), ("flags", "u1"), ("port", "<u2"), ("route_nh", "<u4")])
COUNTER_NAMES = ["pkt_drop", "pkt_accept", "pkt_not_ipv4", "pkt_total", "parse_err", "no_port",
                 "forward", "route_hit", "rx"]


class CopError(RuntimeError):
    def __init__(self, code, msg=""):
        super().__init__(f"cop error {code}: {msg}")
        self.code = code


class LpmConfig(Structure):
    _fields_ = [("max_rules", c_uint32), ("number_tbl8s", c_uint32), ("flags", c_uint32)]


class LpmReport(Structure):
    _fields_ = [("n_in", c_uint32), ("n_added", c_uint32), ("n_distinct", c_uint32),
                ("n_updated", c_uint32), ("n_failed", c_uint32), ("n_skipped", c_uint32),
                ("first_error", c_int32), ("first_error_idx", c_uint32), ("tbl8_used", c_uint32),
                ("n_intervals", c_uint32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Config(Structure):
    _fields_ = [("device", c_int), ("stages", c_uint32), ("n_ports", c_uint32),
                ("max_batch", c_uint32), ("max_batches", c_uint32), ("flags", c_uint32),
                ("n_streams", c_uint32), ("routing_table", POINTER(c_uint16))]


class Batch(Structure):
    _fields_ = [("pkts", c_void_p), ("offsets", c_void_p), ("n", c_uint32), ("stride", c_uint32),
                ("data_off", c_uint32), ("_pad", c_uint32), ("results", c_void_p),
                ("fwd_idx", c_void_p), ("fwd_count", c_void_p)]


class BatchRing(Structure):
    _fields_ = [("pkts", c_void_p), ("offsets", c_void_p), ("results", c_void_p), ("fwd_idx", c_void_p),
                ("fwd_count", c_void_p), ("pkts_slot_bytes", c_uint64), ("offsets_slot_words", c_uint64),
                ("results_slot", c_uint64), ("fwd_slot", c_uint64), ("n_slots", c_uint32), ("n", c_uint32),
                ("stride", c_uint32), ("data_off", c_uint32)]


class TraceOpts(Structure):
    _fields_ = [("n_ports", c_uint32), ("pct_non_ipv4", c_uint32), ("pct_bad_version", c_uint32),
                ("pct_unknown_dst", c_uint32), ("pct_vport_dst", c_uint32),
                ("pct_src_in_rule", c_uint32)]


class PmdInfo(Structure):
    _fields_ = [("workers", c_uint32), ("workers_per_cu", c_uint32), ("tiles_per_batch", c_uint32),
                ("packets_per_tile", c_uint32), ("launches", c_uint32), ("state", c_uint32),
                ("posted", c_uint64), ("completed", c_uint64), ("slot_loads", c_uint32), ("kernel", c_uint32)]


class NfStats(Structure):
    _fields_ = [("rx_packets", c_uint64), ("rx_dropped", c_uint64), ("tx_packets", c_uint64),
                ("tx_dropped", c_uint64)]


class PortStats(Structure):
    _fields_ = [("rx_packets", c_uint64), ("rx_dropped", c_uint64), ("tx_packets", c_uint64),
                ("tx_dropped", c_uint64), ("nf_dropped", c_uint64)]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


# every function declared in include/cop_gpu.h: name -> (restype, argtypes)
SIGNATURES = {
    "cop_lpm_build": (c_int, [c_void_p, c_uint32, POINTER(LpmConfig), POINTER(c_void_p), POINTER(LpmReport)]),
    "cop_lpm_free": (None, [c_void_p]),
    "cop_lpm_export_dir24": (c_int, [c_void_p, c_void_p, c_void_p, c_uint32]),
    "cop_lpm_export_intervals": (c_int, [c_void_p, c_void_p, c_void_p, c_uint32]),
    "cop_lpm_export_rules": (c_int, [c_void_p, c_void_p, c_uint32]),
    "cop_lpm_lookup_rules": (c_int, [c_void_p, c_void_p, c_uint32, c_void_p]),
    "cop_rules_load_json": (c_int, [c_char_p, POINTER(c_void_p), POINTER(c_uint32)]),
    "cop_rules_free": (None, [c_void_p]),
    "cop_rules_write_json": (c_int, [c_char_p, c_void_p, c_uint32]),
    "cop_rules_load_bin": (c_int, [c_char_p, POINTER(c_void_p), POINTER(c_uint32)]),
    "cop_rules_write_bin": (c_int, [c_char_p, c_void_p, c_uint32]),
    "cop_route_table_default": (None, [c_void_p, c_uint32]),
    "cop_config_default": (None, [POINTER(Config)]),
    "cop_create": (c_int, [POINTER(Config), POINTER(c_void_p)]),
    "cop_destroy": (None, [c_void_p]),
    "cop_last_error": (c_char_p, [c_void_p]),
    "cop_device_count": (c_int, []),
    "cop_device_pci_bus_id": (c_int, [c_int, ctypes.c_char_p, c_int]),
    "cop_set_fw_table": (c_int, [c_void_p, c_void_p]),
    "cop_set_route_lpm": (c_int, [c_void_p, c_void_p]),
    "cop_set_routing_table": (c_int, [c_void_p, c_void_p]),
    "cop_load_fw_rules_file": (c_int, [c_void_p, c_char_p, POINTER(LpmConfig), POINTER(LpmReport)]),
    "cop_submit": (c_int, [c_void_p, POINTER(Batch), c_uint32]),
    "cop_submit_ring": (c_int, [c_void_p, POINTER(BatchRing), c_uint32, c_uint32]),
    "cop_sync": (c_int, [c_void_p]),
    "cop_pmd_start": (c_int, [c_void_p, POINTER(BatchRing), POINTER(c_void_p)]),
    "cop_pmd_post": (c_int, [c_void_p, c_uint32]),
    "cop_pmd_wait": (c_int, [c_void_p, c_uint64]),
    "cop_pmd_posted": (c_uint64, [c_void_p]),
    "cop_pmd_run": (c_int, [c_void_p, c_uint64]),
    "cop_pmd_run_timed": (c_int, [c_void_p, c_uint64, POINTER(c_uint64), POINTER(c_uint64)]),
    "cop_pmd_info": (c_int, [c_void_p, POINTER(PmdInfo)]),
    "cop_pmd_stop": (c_int, [c_void_p]),
    "cop_pmd_start_rings": (c_int, [c_void_p, POINTER(BatchRing), c_uint32, c_uint32, POINTER(c_void_p)]),
    "cop_pmd_post_ring": (c_int, [c_void_p, c_uint32, c_uint32]),
    "cop_pmd_post_batch": (c_int, [c_void_p, c_uint32, c_uint32]),
    "cop_pmd_wait_ring": (c_int, [c_void_p, c_uint32, c_uint64]),
    "cop_pmd_posted_ring": (c_uint64, [c_void_p, c_uint32]),
    "cop_pmd_completed_ring": (c_uint64, [c_void_p, c_uint32]),
    "cop_poll": (c_int, [c_void_p]),
    "cop_process_host": (c_int, [c_void_p, POINTER(c_void_p), c_uint32, c_void_p, c_void_p, c_void_p]),
    "cop_process_host_stream": (c_int, [c_void_p, c_void_p, c_uint64, c_uint32, c_void_p]),
    "cop_set_host_threads": (c_int, [c_void_p, c_uint32]),
    "cop_pack_headers": (None, [c_void_p, c_uint32, c_void_p]),
    "cop_pack_headers12": (None, [c_void_p, c_uint32, c_void_p]),
    "cop_counters_read": (c_int, [c_void_p, c_void_p, c_int]),
    "cop_counters_device_ptr": (c_void_p, [c_void_p]),
    "cop_rule_counters_read": (c_int, [c_void_p, c_void_p, c_uint32, c_int]),
    "cop_port_stats_read": (c_int, [c_void_p, POINTER(PortStats), c_uint32, c_int]),
    "cop_counters_snapshot": (c_int, [c_void_p, c_void_p, POINTER(PortStats), c_uint32, c_int]),
    "cop_rule_counters_device_ptr": (c_int, [c_void_p, POINTER(c_void_p), POINTER(c_uint32)]),
    "cop_coll_unique_id": (c_int, [c_void_p]),
    "cop_coll_init": (c_int, [c_void_p, c_void_p, c_int, c_int]),
    "cop_coll_reduce_counters": (c_int, [c_void_p, c_void_p, c_void_p, c_uint32, c_int]),
    "cop_dev_alloc": (c_int, [c_void_p, c_size_t, POINTER(c_void_p)]),
    "cop_dev_alloc_ex": (c_int, [c_void_p, c_size_t, c_uint32, POINTER(c_void_p)]),
    "cop_dev_free": (c_int, [c_void_p, c_void_p]),
    "cop_host_alloc_pinned": (c_int, [c_void_p, c_size_t, POINTER(c_void_p)]),
    "cop_host_alloc_mapped": (c_int, [c_void_p, c_size_t, POINTER(c_void_p), POINTER(c_void_p)]),
    "cop_host_free_pinned": (c_int, [c_void_p, c_void_p]),
    "cop_memcpy_h2d": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t]),
    "cop_memcpy_d2h": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t]),
    "cop_memcpy_d2d": (c_int, [c_void_p, c_void_p, c_void_p, c_size_t]),
    "cop_memset_d": (c_int, [c_void_p, c_void_p, c_int, c_size_t]),
    "cop_timer_start": (c_int, [c_void_p]),
    "cop_timer_stop": (c_int, [c_void_p, POINTER(c_double)]),
    "cop_launch_timing": (c_int, [c_void_p, c_int]),
    "cop_launch_timing_read": (c_int, [c_void_p, POINTER(c_double), POINTER(c_uint64), c_int]),
    "cop_ring_create": (c_void_p, [c_uint32]),
    "cop_ring_free": (None, [c_void_p]),
    "cop_ring_enqueue_bulk": (c_uint32, [c_void_p, c_void_p, c_uint32, POINTER(c_uint32)]),
    "cop_ring_dequeue_burst": (c_uint32, [c_void_p, c_void_p, c_uint32, POINTER(c_uint32)]),
    "cop_ring_count": (c_uint32, [c_void_p]),
    "cop_set_mbuf_layout": (None, [c_uint32, c_uint32]),
    "cop_set_rule_file": (None, [c_char_p]),
    "coprocessor_setup": (c_int, []),
    "cop_set_dropin_stages": (c_int, [c_uint32]),
    "cop_dropin_stages": (c_uint32, []),
    "cop_coprocessor_setup_stages": (c_int, [c_uint32]),
    "cop_coprocessor_setup_fw": (c_int, []),
    "cop_coprocessor_setup_no_nf": (c_int, []),
    "coprocessor_teardown": (c_int, []),
    "process_packet": (c_int, [c_void_p]),
    "process_burst": (c_int, [c_void_p, c_uint32, c_void_p]),
    "cop_coprocessor_poll": (c_int, [c_void_p, c_void_p, c_void_p, c_uint32, c_void_p, c_void_p, POINTER(NfStats)]),
    "cop_coprocessor_poll_async": (c_int, [c_void_p, c_void_p, c_void_p, c_uint32, c_void_p, c_void_p,
                                           POINTER(NfStats)]),
    "cop_coprocessor_flush": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, POINTER(NfStats)]),
    "cop_pmd_host_create": (c_int, [c_void_p, c_uint32, c_uint32, c_uint32, POINTER(c_void_p)]),
    "cop_coprocessor_poll_pmd": (c_int, [c_void_p, c_uint32, c_void_p, c_void_p, c_uint32, c_void_p, c_void_p,
                                         POINTER(NfStats)]),
    "cop_coprocessor_flush_pmd": (c_int, [c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, POINTER(NfStats)]),
    "cop_pmd_host_destroy": (c_int, [c_void_p]),
    "cop_host_batch_submit": (c_int, [c_void_p, c_uint32, c_void_p, c_uint32]),
    "cop_host_batch_wait": (c_int, [c_void_p, c_uint32, POINTER(c_void_p), POINTER(c_uint32)]),
    "coprocessor_ctx": (c_void_p, []),
    "cop_gen_rules": (c_int, [c_uint64, c_uint32, c_int, c_uint32, c_void_p]),
    "cop_trace_opts_default": (None, [POINTER(TraceOpts)]),
    "cop_gen_trace": (c_int, [c_uint64, c_uint32, POINTER(TraceOpts), c_void_p, c_uint32, c_void_p,
                              c_uint32, c_void_p, c_uint32]),
    "cop_gen_imix": (c_int, [c_uint64, c_uint32, POINTER(TraceOpts), c_void_p, c_uint32, c_void_p,
                             c_uint32, c_void_p, POINTER(c_uint64), c_void_p]),
}

_lib = None


def lib():
    """Load libcopgpu.so (raises ImportError when it has not been built)."""
    global _lib
    if _lib is None:
        # $COP_LIB: an alternative in-tree build of the same ABI (A/B runs)
        path = os.environ.get("COP_LIB") or LIB_PATH
        if not os.path.exists(path):
            raise ImportError(f"{path} not built (run make -C ghost-dataplane_amd)")
        L = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("COP_LIB") and not hasattr(L, name):
                continue   # an older A/B build: calls it lacks fail when used
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(c_void_p) if a is not None else None


def _check(rc, ctx=None, what=""):
    if rc < 0:
        msg = what
        if ctx is not None and ctx.handle:
            msg += ": " + lib().cop_last_error(ctx.handle).decode(errors="replace")
        raise CopError(rc, msg)
    return rc


# ---------------------------------------------------------------------------
# host helpers

def pack_headers(ptrs: np.ndarray) -> np.ndarray:
    """cop_pack_headers over host packet addresses (u64 array): n x 16 bytes."""
    ptrs = np.ascontiguousarray(ptrs, dtype=np.uint64)
    out = np.zeros(len(ptrs) * HDR16_STRIDE, np.uint8)
    lib().cop_pack_headers(ptrs.ctypes.data, len(ptrs), out.ctypes.data)
    return out


def pack_headers_np(frames: np.ndarray, n: int, stride: int = 64) -> np.ndarray:
    """The same records from a contiguous frame array, in numpy (tests)."""
    f = np.asarray(frames, np.uint8)[: n * stride].reshape(n, stride)
    return np.ascontiguousarray(np.concatenate([f[:, 12:16], f[:, 24:36]], axis=1)).reshape(-1)


def pack_headers12(ptrs: np.ndarray) -> np.ndarray:
    """cop_pack_headers12 over host packet addresses (u64 array): n x 12 bytes."""
    ptrs = np.ascontiguousarray(ptrs, dtype=np.uint64)
    out = np.zeros(len(ptrs) * HDR12_STRIDE, np.uint8)
    lib().cop_pack_headers12(ptrs.ctypes.data, len(ptrs), out.ctypes.data)
    return out


def prefixes(ip, depth, next_hop) -> np.ndarray:
    ip = np.asarray(ip, dtype=np.uint64)
    a = np.zeros(len(ip), dtype=PREFIX_DT)
    a["ip"] = ip.astype(np.uint32)
    a["depth"] = np.asarray(depth, dtype=np.int64).astype(np.uint8)
    a["next_hop"] = np.asarray(next_hop, dtype=np.uint64).astype(np.uint32)
    return a


def gen_rules(seed: int, n: int, kind: int = GEN_FW, n_long_parents: int = 20) -> np.ndarray:
    out = np.zeros(n, dtype=PREFIX_DT)
    _check(lib().cop_gen_rules(seed, n, kind, n_long_parents, _ptr(out)), what="gen_rules")
    return out


def trace_opts(**kw) -> TraceOpts:
    o = TraceOpts()
    lib().cop_trace_opts_default(byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def gen_trace(seed: int, n: int, fw=None, routes=None, stride: int = 64, opts: TraceOpts | None = None,
              out: np.ndarray | None = None) -> np.ndarray:
    if out is None:
        out = np.zeros(n * stride, dtype=np.uint8)
    fw = fw if fw is not None else np.zeros(0, dtype=PREFIX_DT)
    routes = routes if routes is not None else np.zeros(0, dtype=PREFIX_DT)
    _check(lib().cop_gen_trace(seed, n, byref(opts) if opts else None, _ptr(fw), len(fw), _ptr(routes),
                               len(routes), _ptr(out), stride), what="gen_trace")
    return out


def gen_imix(seed: int, n: int, fw=None, routes=None, opts: TraceOpts | None = None):
    fw = fw if fw is not None else np.zeros(0, dtype=PREFIX_DT)
    routes = routes if routes is not None else np.zeros(0, dtype=PREFIX_DT)
    size = c_uint64(0)
    o = byref(opts) if opts else None
    _check(lib().cop_gen_imix(seed, n, o, _ptr(fw), len(fw), _ptr(routes), len(routes), None, byref(size), None))
    slab = np.zeros(size.value + 64, dtype=np.uint8)
    offs = np.zeros(n, dtype=np.uint32)
    _check(lib().cop_gen_imix(seed, n, o, _ptr(fw), len(fw), _ptr(routes), len(routes), _ptr(slab),
                              byref(size), _ptr(offs)))
    return slab, offs


def route_table_default(n_ports: int = 5) -> np.ndarray:
    rt = np.zeros(65536, dtype=np.uint16)
    lib().cop_route_table_default(_ptr(rt), n_ports)
    return rt


def rules_load_json(path: str) -> np.ndarray:
    p = c_void_p()
    n = c_uint32()
    _check(lib().cop_rules_load_json(path.encode(), byref(p), byref(n)), what=f"load {path}")
    try:
        buf = (ctypes.c_uint8 * (n.value * PREFIX_DT.itemsize)).from_address(p.value) if n.value else b""
        return np.frombuffer(bytes(buf), dtype=PREFIX_DT).copy()
    finally:
        lib().cop_rules_free(p)


def rules_write_json(path: str, rules: np.ndarray):
    rules = np.ascontiguousarray(rules, dtype=PREFIX_DT)
    _check(lib().cop_rules_write_json(path.encode(), _ptr(rules), len(rules)), what=f"write {path}")


def rules_load_bin(path: str) -> np.ndarray:
    """Binary prefix dump (cop_rules_load_bin) -> PREFIX_DT array."""
    p = c_void_p()
    n = c_uint32()
    _check(lib().cop_rules_load_bin(path.encode(), byref(p), byref(n)), what=f"load {path}")
    try:
        buf = (ctypes.c_uint8 * (n.value * PREFIX_DT.itemsize)).from_address(p.value) if n.value else b""
        return np.frombuffer(bytes(buf), dtype=PREFIX_DT).copy()
    finally:
        lib().cop_rules_free(p)


def rules_write_bin(path: str, rules: np.ndarray):
    rules = np.ascontiguousarray(rules, dtype=PREFIX_DT)
    _check(lib().cop_rules_write_bin(path.encode(), _ptr(rules), len(rules)), what=f"write {path}")


class LpmTable:
    """Host-built LPM table with DPDK rte_lpm_add semantics."""

    def __init__(self, rules: np.ndarray, max_rules=1024, number_tbl8s=24, stop_at_first_error=True):
        rules = np.ascontiguousarray(rules, dtype=PREFIX_DT)
        cfg = LpmConfig(max_rules, number_tbl8s, LPM_STOP_AT_FIRST_ERROR if stop_at_first_error else 0)
        self.handle = c_void_p()
        self.report = LpmReport()
        _check(lib().cop_lpm_build(_ptr(rules), len(rules), byref(cfg), byref(self.handle),
                                   byref(self.report)), what="cop_lpm_build")

    def __del__(self):
        if getattr(self, "handle", None) and self.handle.value:
            lib().cop_lpm_free(self.handle)
            self.handle = c_void_p()

    def rules(self) -> np.ndarray:
        n = _check(lib().cop_lpm_export_rules(self.handle, None, 0))
        out = np.zeros(n, dtype=PREFIX_DT)
        _check(lib().cop_lpm_export_rules(self.handle, _ptr(out), n))
        return out

    def lookup_rules(self, ips: np.ndarray) -> np.ndarray:
        """Matching rule id per address (-1 on a miss), host-side."""
        ips = np.ascontiguousarray(ips, dtype=np.uint32)
        out = np.zeros(len(ips), dtype=np.int32)
        _check(lib().cop_lpm_lookup_rules(self.handle, _ptr(ips), len(ips), _ptr(out)))
        return out

    def intervals(self):
        m = _check(lib().cop_lpm_export_intervals(self.handle, None, None, 1 << 31))
        s = np.zeros(m, dtype=np.uint32)
        v = np.zeros(m, dtype=np.uint32)
        _check(lib().cop_lpm_export_intervals(self.handle, _ptr(s), _ptr(v), m))
        return s, v

    def trie_probe(self, ips: np.ndarray, form: int = 0):
        """The multibit-trie form (lpm_trie.c) of this table's device image
        (form 0: next hop, 1: rule id), walked on the host: (trie values,
        interval-search values, nodes, leaves) for each address."""
        ips = np.ascontiguousarray(ips, dtype=np.uint32)
        out = np.zeros(len(ips), dtype=np.uint32)
        ref = np.zeros(len(ips), dtype=np.uint32)
        nn, nl = ctypes.c_uint32(), ctypes.c_uint32()
        f = lib().cop_lpm_trie_probe
        f.restype = c_int
        f.argtypes = [c_void_p, c_int, c_void_p, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p]
        _check(f(self.handle, form, _ptr(ips), len(ips), _ptr(out), _ptr(ref), byref(nn), byref(nl)),
               what="cop_lpm_trie_probe")
        return out, ref, nn.value, nl.value

    def bkt_probe(self, ips: np.ndarray, form: int = 0, xbits: int = 1):
        """The bucketed interval form (lpm_bkt.c) of this table's device
        image (form 0: next hop, 1: rule id), looked up on the host the way
        the kernel does: (values, interval-search values, info dict)."""
        ips = np.ascontiguousarray(ips, dtype=np.uint32)
        out = np.zeros(len(ips), dtype=np.uint32)
        ref = np.zeros(len(ips), dtype=np.uint32)
        info = np.zeros(6, dtype=np.uint32)
        f = lib().cop_lpm_bkt_probe
        f.restype = c_int
        f.argtypes = [c_void_p, c_int, c_uint32, c_void_p, c_uint32, c_void_p, c_void_p, c_void_p]
        _check(f(self.handle, form, xbits, _ptr(ips), len(ips), _ptr(out), _ptr(ref), _ptr(info)), what="cop_lpm_bkt_probe")
        return out, ref, dict(zip(("m", "ib", "lv", "widest", "lifted", "rounds"), (int(x) for x in info)))

    def dir24(self):
        t24 = np.zeros(1 << 24, dtype=np.uint32)
        cap = 256 * max(1, self.report.n_distinct)
        t8 = np.zeros(cap, dtype=np.uint32)
        n_ext = _check(lib().cop_lpm_export_dir24(self.handle, _ptr(t24), _ptr(t8), cap))
        return t24, t8[: n_ext * 256]


ALLOC_UNCACHED, ALLOC_FINEGRAINED = 1, 2


class DeviceBuffer:
    def __init__(self, ctx: "Context", nbytes: int, flags: int = 0):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        self.ptr = c_void_p()
        if flags:
            _check(lib().cop_dev_alloc_ex(ctx.handle, self.nbytes, flags, byref(self.ptr)), ctx, "dev_alloc_ex")
        else:
            _check(lib().cop_dev_alloc(ctx.handle, self.nbytes, byref(self.ptr)), ctx, "dev_alloc")

    @property
    def addr(self) -> int:
        return self.ptr.value

    def upload(self, a: np.ndarray, offset: int = 0):
        a = np.ascontiguousarray(a)
        assert offset + a.nbytes <= self.nbytes
        _check(lib().cop_memcpy_h2d(self.ctx.handle, c_void_p(self.addr + offset), _ptr(a), a.nbytes),
               self.ctx, "h2d")

    def download(self, dtype, count: int, offset: int = 0) -> np.ndarray:
        out = np.zeros(count, dtype=dtype)
        assert offset + out.nbytes <= self.nbytes
        if out.nbytes:
            _check(lib().cop_memcpy_d2h(self.ctx.handle, _ptr(out), c_void_p(self.addr + offset), out.nbytes),
                   self.ctx, "d2h")
        return out

    def fill(self, value: int = 0):
        _check(lib().cop_memset_d(self.ctx.handle, self.ptr, value, self.nbytes), self.ctx, "memset")

    def free(self):
        if self.ptr.value:
            lib().cop_dev_free(self.ctx.handle, self.ptr)
            self.ptr = c_void_p()

    def __del__(self):
        try:
            if self.ptr.value and self.ctx.handle:
                self.free()
        except Exception:
            pass


COLL_ID_BYTES = 128


def coll_unique_id() -> bytes:
    """RCCL unique id (rank 0 creates it; the caller distributes it)."""
    buf = (c_uint8 * COLL_ID_BYTES)()
    _check(lib().cop_coll_unique_id(buf), what="cop_coll_unique_id")
    return bytes(buf)


def device_count() -> int:
    return lib().cop_device_count()


def device_pci_bus_id(device: int) -> str:
    buf = ctypes.create_string_buffer(64)
    _check(lib().cop_device_pci_bus_id(device, buf, 64), what="cop_device_pci_bus_id")
    return buf.value.decode().lower()


class Context:
    """One GPU context (cop_ctx): device, stream, NF tables."""

    def __init__(self, device=0, stages=STAGE_PARSE | STAGE_FW, n_ports=5, max_batch=262144,
                 max_batches=32, flags=0, routing_table: np.ndarray | None = None, n_streams=None):
        cfg = Config()
        lib().cop_config_default(byref(cfg))
        cfg.device, cfg.stages, cfg.n_ports = device, stages, n_ports
        cfg.max_batch, cfg.max_batches, cfg.flags = max_batch, max_batches, flags
        if n_streams is not None:
            cfg.n_streams = n_streams
        self._rt = None
        if routing_table is not None:
            self._rt = np.ascontiguousarray(routing_table, dtype=np.uint16)
            cfg.routing_table = self._rt.ctypes.data_as(POINTER(c_uint16))
        self.handle = c_void_p()
        rc = lib().cop_create(byref(cfg), byref(self.handle))
        if rc < 0:
            raise CopError(rc, "cop_create failed (no GPU?)")
        self.cfg = cfg

    def close(self):
        if self.handle and self.handle.value:
            for m in getattr(self, "_pmds", []):
                m.stop()
            lib().cop_destroy(self.handle)
            self.handle = c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_fw_table(self, t: LpmTable):
        _check(lib().cop_set_fw_table(self.handle, t.handle), self, "set_fw_table")

    def set_route_lpm(self, t: LpmTable):
        _check(lib().cop_set_route_lpm(self.handle, t.handle), self, "set_route_lpm")

    ROUTE_FORMS = {1: "lds", 2: "dir", 3: "trie", 4: "bkt"}

    def route_form(self) -> str:
        """The route stage's table form a launch uses now (lds: LDS
        intervals, dir: DIR-24-8, trie, bkt: bucketed intervals in L2)."""
        f = lib().cop_debug_route_form
        f.restype = c_int
        f.argtypes = [c_void_p]
        return self.ROUTE_FORMS[_check(f(self.handle), self, "route_form")]

    def set_routing_table(self, rt: np.ndarray):
        rt = np.ascontiguousarray(rt, dtype=np.uint16)
        assert rt.size == 65536
        _check(lib().cop_set_routing_table(self.handle, _ptr(rt)), self, "set_routing_table")

    def load_fw_rules_file(self, path, max_rules=1024, number_tbl8s=24, stop_at_first_error=True):
        cfg = LpmConfig(max_rules, number_tbl8s, LPM_STOP_AT_FIRST_ERROR if stop_at_first_error else 0)
        rep = LpmReport()
        _check(lib().cop_load_fw_rules_file(self.handle, path.encode(), byref(cfg), byref(rep)), self,
               "load_fw_rules_file")
        return rep

    def alloc(self, nbytes, flags: int = 0) -> DeviceBuffer:
        """HBM (flags: ALLOC_UNCACHED / ALLOC_FINEGRAINED, cop_dev_alloc_ex)."""
        return DeviceBuffer(self, nbytes, flags)

    def pmd_start(self, ring, flags: int = 0) -> "Pmd":
        """Start the poll-mode (persistent) kernel serving `ring` (or a list
        of rings: one kernel serving each; PMD_VARIABLE_N in flags)."""
        return Pmd(self, ring, flags)

    def submit(self, batches):
        arr = (Batch * len(batches))(*batches)
        _check(lib().cop_submit(self.handle, arr, len(batches)), self, "submit")

    def submit_ring(self, ring: BatchRing, first_slot: int, count: int):
        _check(lib().cop_submit_ring(self.handle, byref(ring), first_slot, count), self, "submit_ring")

    def sync(self):
        _check(lib().cop_sync(self.handle), self, "sync")

    def counters(self, reset=False) -> dict:
        c = np.zeros(16, dtype=np.uint64)
        _check(lib().cop_counters_read(self.handle, _ptr(c), 1 if reset else 0), self, "counters")
        return {k: int(c[i]) for i, k in enumerate(COUNTER_NAMES)}

    def counters_device_ptr(self) -> int:
        return lib().cop_counters_device_ptr(self.handle)

    def port_stats(self, reset=False) -> list:
        """Per-port coprocessor_stats (CFG_PORT_STATS), synchronous."""
        arr = (PortStats * MAX_DEMUX_PORTS)()
        n = _check(lib().cop_port_stats_read(self.handle, arr, MAX_DEMUX_PORTS, 1 if reset else 0), self,
                   "port_stats")
        return [arr[i].as_dict() for i in range(n)]

    def snapshot(self, reset=False, ports=0):
        """Live counters (+ per-port stats) without waiting for submitted work."""
        c = np.zeros(16, dtype=np.uint64)
        arr = (PortStats * MAX_DEMUX_PORTS)()
        _check(lib().cop_counters_snapshot(self.handle, _ptr(c), arr, ports, 1 if reset else 0), self, "snapshot")
        return {k: int(c[i]) for i, k in enumerate(COUNTER_NAMES)}, [arr[i].as_dict() for i in range(ports)]

    def rule_counters(self, reset=False) -> np.ndarray:
        """Per-rule FW hit counters (CFG_RULE_COUNTERS), indexed by rule id."""
        n = _check(lib().cop_rule_counters_read(self.handle, None, 0, 0), self, "rule_counters")
        out = np.zeros(n, dtype=np.uint64)
        _check(lib().cop_rule_counters_read(self.handle, _ptr(out), n, 1 if reset else 0), self, "rule_counters")
        return out

    def coll_init(self, uid: bytes, rank: int, nranks: int):
        buf = (c_uint8 * COLL_ID_BYTES).from_buffer_copy(uid)
        _check(lib().cop_coll_init(self.handle, buf, rank, nranks), self, "coll_init")

    def coll_reduce_counters(self, reset=False, with_rules=True):
        """RCCL all-reduce of counters (+ per-rule counters) over the ranks."""
        c = np.zeros(16, dtype=np.uint64)
        n = 0
        if with_rules and (self.cfg.flags & CFG_RULE_COUNTERS):
            n = _check(lib().cop_rule_counters_read(self.handle, None, 0, 0), self, "rule_counters")
        hits = np.zeros(max(n, 1), dtype=np.uint64)
        _check(lib().cop_coll_reduce_counters(self.handle, _ptr(c), _ptr(hits), n, 1 if reset else 0), self,
               "coll_reduce_counters")
        return {k: int(c[i]) for i, k in enumerate(COUNTER_NAMES)}, hits[:n]

    def process_host(self, pkts: np.ndarray, n: int, stride: int = 64):
        """End-to-end: host packet memory -> pinned gather -> H2D -> kernel -> D2H."""
        base = pkts.ctypes.data
        ptrs = (c_void_p * n)(*[base + i * stride for i in range(n)])
        res = np.zeros(n, dtype=RESULT_DT)
        fwd = np.zeros(max(n, 1), dtype=np.uint32)
        cnt = c_uint32(0)
        _check(lib().cop_process_host(self.handle, ptrs, n, _ptr(res), _ptr(fwd), byref(cnt)), self,
               "process_host")
        return res, fwd[: cnt.value]

    def set_host_threads(self, n: int):
        _check(lib().cop_set_host_threads(self.handle, n), self, "set_host_threads")

    def process_host_stream(self, ptrs: np.ndarray, batch: int, out: np.ndarray | None = None) -> np.ndarray:
        """Streaming end-to-end path over host packet addresses (u64 array).
        out: a RESULT_DT array of len(ptrs) to fill (timed loops reuse one)."""
        ptrs = np.ascontiguousarray(ptrs, dtype=np.uint64)
        if out is not None:
            assert out.dtype == RESULT_DT and len(out) == len(ptrs) and out.flags.c_contiguous
            res = out
        else:
            res = np.zeros(len(ptrs), dtype=RESULT_DT)
        _check(lib().cop_process_host_stream(self.handle, _ptr(ptrs), len(ptrs), batch, _ptr(res)), self,
               "process_host_stream")
        return res

    def timer_start(self):
        _check(lib().cop_timer_start(self.handle), self, "timer_start")

    def timer_stop(self) -> float:
        ms = c_double(0)
        _check(lib().cop_timer_stop(self.handle, byref(ms)), self, "timer_stop")
        return ms.value

    def launch_timing(self, enable=True):
        _check(lib().cop_launch_timing(self.handle, 1 if enable else 0), self, "launch_timing")

    def launch_timing_read(self, reset=True):
        ms = c_double(0)
        n = c_uint64(0)
        _check(lib().cop_launch_timing_read(self.handle, byref(ms), byref(n), 1 if reset else 0), self,
               "launch_timing_read")
        return ms.value, n.value


PMD_VARIABLE_N = 1
PMD_SYS_ACQUIRE = 2     # acquire on every tile
PMD_STATIC_SLOTS = 4    # slots written once before the start: plain loads (default: coherent loads once the ring wraps)
PMD_DYNAMIC_TILES = 8   # tiles claimed from tickets, the next tile's loads issued early (segmented lists)


class Pmd:
    """A poll-mode kernel serving one batch ring (cop_pmd_*): post(count)
    hands the next `count` slots to the running kernel (batch sequence
    numbers continue across posts; batch b sits in slot b % n_slots),
    wait(seq) blocks until batches < seq have completed. With a list of
    rings (cop_pmd_start_rings), one kernel serves them all: ring r is
    posted and waited with post_ring / post_batch / wait_ring."""

    def __init__(self, ctx: "Context", ring, flags: int = 0):
        self.ctx = ctx
        self.handle = c_void_p()
        if isinstance(ring, (list, tuple)):
            arr = (BatchRing * len(ring))(*ring)
            self.ring = arr   # keep the descriptors alive
            self.n_rings = len(ring)
            _check(lib().cop_pmd_start_rings(ctx.handle, arr, len(ring), flags, byref(self.handle)), ctx,
                   "pmd_start_rings")
        else:
            self.ring = ring   # keep the descriptor alive
            self.n_rings = 1
            if flags:
                arr = (BatchRing * 1)(ring)
                self.ring = arr
                _check(lib().cop_pmd_start_rings(ctx.handle, arr, 1, flags, byref(self.handle)), ctx,
                       "pmd_start_rings")
            else:
                _check(lib().cop_pmd_start(ctx.handle, byref(ring), byref(self.handle)), ctx, "pmd_start")
        if not hasattr(ctx, "_pmds"):
            ctx._pmds = []
        ctx._pmds.append(self)
        # bound once: these sit inside timed regions (a lookup per call costs
        # a measurable part of a 30 us post)
        L = lib()
        self._post, self._wait, self._run = L.cop_pmd_post, L.cop_pmd_wait, L.cop_pmd_run
        self._run_timed = L.cop_pmd_run_timed
        self._t = (c_uint64(0), c_uint64(0))
        self._tp = (byref(self._t[0]), byref(self._t[1]))
        self._n_posted = 0   # every post goes through this object

    def post(self, count: int):
        _check(self._post(self.handle, count), self.ctx, "pmd_post")
        self._n_posted += count

    def wait(self, seq: int | None = None):
        rc = self._wait(self.handle, self._n_posted if seq is None else seq)
        if rc < 0:
            _check(rc, self.ctx, "pmd_wait")

    def run(self, count: int):
        """Post `count` batches and wait for all of them (one C call)."""
        rc = self._run(self.handle, count)
        if rc < 0:
            _check(rc, self.ctx, "pmd_run")
        self._n_posted += count

    def run_timed(self, count: int):
        """run(count), returning (t_post_ns, t_done_ns): CLOCK_MONOTONIC taken
        inside the library just before the first post and just after the
        last completion (cop_pmd_run_timed)."""
        rc = self._run_timed(self.handle, count, *self._tp)
        if rc < 0:
            _check(rc, self.ctx, "pmd_run_timed")
        self._n_posted += count
        return self._t[0].value, self._t[1].value

    @property
    def posted(self) -> int:
        return int(lib().cop_pmd_posted(self.handle))

    def post_ring(self, ring: int, count: int):
        _check(lib().cop_pmd_post_ring(self.handle, ring, count), self.ctx, "pmd_post_ring")

    def post_batch(self, ring: int, n: int):
        """One batch of n packets (PMD_VARIABLE_N) to `ring`."""
        _check(lib().cop_pmd_post_batch(self.handle, ring, n), self.ctx, "pmd_post_batch")

    def wait_ring(self, ring: int, seq: int | None = None):
        if seq is None:
            seq = int(lib().cop_pmd_posted_ring(self.handle, ring))
        _check(lib().cop_pmd_wait_ring(self.handle, ring, seq), self.ctx, "pmd_wait_ring")

    def posted_ring(self, ring: int) -> int:
        return int(lib().cop_pmd_posted_ring(self.handle, ring))

    def completed_ring(self, ring: int) -> int:
        return int(lib().cop_pmd_completed_ring(self.handle, ring))

    def info(self) -> dict:
        i = PmdInfo()
        _check(lib().cop_pmd_info(self.handle, byref(i)), self.ctx, "pmd_info")
        d = {k: getattr(i, k) for k, _ in PmdInfo._fields_}
        k = d["kernel"]
        # the instantiation's template arguments, as rocprofv3 names the kernel
        d["kernel_name"] = (f"cop_pmd<{k & 15}, {(k >> 4) & 15}, {(k >> 8) & 15}, {d['packets_per_tile'] // 256}, "
                            f"{'true' if (k >> 12) & 1 else 'false'}>")
        return d

    def stop(self):
        if self.handle and self.handle.value:
            h, self.handle = self.handle, c_void_p()
            if self in getattr(self.ctx, "_pmds", []):
                self.ctx._pmds.remove(self)
            _check(lib().cop_pmd_stop(h), self.ctx, "pmd_stop")

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.stop()


def make_ring(pkts, n_slots: int, n: int, results, pkts_slot_bytes: int, results_slot: int = 0,
              fwd_idx=None, fwd_slot: int = 0, fwd_count=None, stride: int = 64, offsets=None,
              offsets_slot_words: int = 0, data_off: int = 0) -> BatchRing:
    def addr(x):
        if x is None:
            return None
        return x.addr if isinstance(x, DeviceBuffer) else int(x)
    r = BatchRing()
    r.pkts, r.offsets, r.results = addr(pkts), addr(offsets), addr(results)
    r.fwd_idx, r.fwd_count = addr(fwd_idx), addr(fwd_count)
    r.pkts_slot_bytes, r.offsets_slot_words = pkts_slot_bytes, offsets_slot_words
    r.results_slot = results_slot or n
    r.fwd_slot = fwd_slot or n
    r.n_slots, r.n, r.stride, r.data_off = n_slots, n, stride, data_off
    # the ring holds device addresses only: keep the buffers it was made from
    # alive as long as the ring (a collected DeviceBuffer frees its memory,
    # and a kernel writing through the stale address would fault the GPU)
    r._keep = tuple(x for x in (pkts, offsets, results, fwd_idx, fwd_count) if isinstance(x, DeviceBuffer))
    return r


def make_batch(pkts: DeviceBuffer | int, n: int, results: DeviceBuffer | int, stride: int = 64,
               offsets: DeviceBuffer | int | None = None, fwd_idx=None, fwd_count=None,
               data_off: int = 0, pkts_offset: int = 0, results_offset: int = 0) -> Batch:
    def addr(x, off=0):
        if x is None:
            return None
        return (x.addr if isinstance(x, DeviceBuffer) else int(x)) + off
    b = Batch()
    b.pkts = addr(pkts, pkts_offset)
    b.offsets = addr(offsets)
    b.n = n
    b.stride = stride
    b.data_off = data_off
    b.results = addr(results, results_offset)
    b.fwd_idx = addr(fwd_idx)
    b.fwd_count = addr(fwd_count)
    b._keep = tuple(x for x in (pkts, offsets, results, fwd_idx, fwd_count) if isinstance(x, DeviceBuffer))
    return b
