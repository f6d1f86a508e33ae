"""TEST INFRASTRUCTURE ONLY: the reference's own rules.json parser.

The reference parses its rule file with its vendored cJSON 1.7.12
(engine/thirdparty/cJSON.c). That file is plain C with no DPDK dependency,
so `make -C oracle ref` compiles it where it lies under /root/reference into
oracle/_ref/libcjson_ref.so (nothing is copied into the repo). This module
replays setup_rules (firewall.c:276-323) over that real parser:
  fw_config_parse_file  (firewall.c:57-105): the file as one C string
  cJSON_Parse, root->child, ->next                      (firewall.c:292-318)
  cJSON_GetObjectItem "ip" / "depth" / "action"         (:305-307, rte_exit on NULL)
  fw_pkt_parse_ip(valuestring)                          (:314; restated: firewall.c
                                                         needs DPDK headers, see
                                                         oracle.parse_ip)
  depth/action = valueint stored in uint8_t fields      (:315-316, firewall.h:49-53)
It pins the loader restatements (oracle.py, csrc/rules_json.c) to the
reference's parser on the inputs tests/test_ref_cjson.py feeds them.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, Structure, c_char_p, c_double, c_int, c_void_p

from oracle import parse_ip

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_ref", "libcjson_ref.so")


class _CJSON(Structure):
    pass


# struct cJSON, cJSON.h:94-114 (1.7.12)
_CJSON._fields_ = [("next", POINTER(_CJSON)), ("prev", POINTER(_CJSON)), ("child", POINTER(_CJSON)),
                   ("type", c_int), ("valuestring", c_char_p), ("valueint", c_int),
                   ("valuedouble", c_double), ("string", c_char_p)]


class RefExit(Exception):
    """The reference calls rte_exit (parse failure, missing key)."""


class RefUndefined(Exception):
    """The reference reads an uninitialised field (fw_pkt_parse_ip failed)."""


_lib = None


def available() -> bool:
    return os.path.exists(LIB_PATH)


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(LIB_PATH)
        L.cJSON_Parse.restype = POINTER(_CJSON)
        L.cJSON_Parse.argtypes = [c_char_p]
        L.cJSON_GetObjectItem.restype = POINTER(_CJSON)
        L.cJSON_GetObjectItem.argtypes = [POINTER(_CJSON), c_char_p]
        L.cJSON_Delete.restype = None
        L.cJSON_Delete.argtypes = [POINTER(_CJSON)]
        L.cJSON_Version.restype = c_char_p
        _lib = L
    return _lib


def version() -> str:
    return lib().cJSON_Version().decode()


def setup_rules(path: str):
    """-> [(src_ip, depth, action)] exactly as the reference would build them."""
    L = lib()
    with open(path, "rb") as f:
        data = f.read()
    root = L.cJSON_Parse(data)          # C string: stops at the first NUL, like json_str
    if not root:
        raise RefExit("could not be parsed")
    try:
        out = []
        item = root.contents.child
        while item:
            ip = L.cJSON_GetObjectItem(item, b"ip")
            depth = L.cJSON_GetObjectItem(item, b"depth")
            action = L.cJSON_GetObjectItem(item, b"action")
            if not ip or not depth or not action:
                raise RefExit("IP/Depth/Action not found")
            s = ip.contents.valuestring
            v = parse_ip(s.decode("utf-8", errors="surrogateescape")) if s is not None else None
            if v is None:
                raise RefUndefined("fw_pkt_parse_ip failed: src_ip left uninitialised")
            out.append((v, depth.contents.valueint & 0xFF, action.contents.valueint & 0xFF))
            item = item.contents.next
        return out
    finally:
        L.cJSON_Delete(root)
