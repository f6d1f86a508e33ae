"""The C boundary from C: tests/c/switch_dropin.c plays switch.c's calls
(coprocessor_setup, process_packet, a burst, and the rx_q -> GPU -> tx_q
ring loop of coprocessor(), switch.c:443-474) against libcopgpu.so using
only include/cop_gpu.h. The CPU test compiles and links it as C99 with
-Werror (no HIP headers, no torch); the GPU test runs it and compares every
return value and the tx_q order with the oracle."""
import os
import subprocess

import numpy as np
import pytest

import copgpu as cg
import oracle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ghost-dataplane_amd")
SRC = os.path.join(ROOT, "tests", "c", "switch_dropin.c")


def build(tmp_path):
    exe = str(tmp_path / "switch_dropin")
    r = subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", "-Werror", "-DENABLE_FW_NF",
                        "-I", os.path.join(ROOT, "include"), SRC, "-o", exe, "-L", PKG, "-lcopgpu",
                        f"-Wl,-rpath,{PKG}"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def test_c_dropin_compiles_and_links(tmp_path):
    exe = build(tmp_path)
    # the binary needs only libcopgpu (+ libc/HIP runtime behind it), no torch
    ldd = subprocess.run(["ldd", exe], capture_output=True, text=True).stdout
    assert "libcopgpu.so" in ldd and "torch" not in ldd


@pytest.mark.gpu
def test_c_dropin_matches_oracle(tmp_path):
    exe = build(tmp_path)
    rules = cg.gen_rules(0x5EED1002, 1000, cg.GEN_FW, 20)
    rf = str(tmp_path / "rules.json")
    cg.rules_write_json(rf, rules)
    n = 100000
    out = str(tmp_path / "out.bin")
    r = subprocess.run([exe, rf, str(n), out], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    raw = np.fromfile(out, dtype=np.uint8)
    n1 = min(n, 512)
    ret1 = raw[:4 * n1].view(np.int32)
    ret2 = raw[4 * n1: 4 * (n1 + n)].view(np.int32)
    nf = int(raw[4 * (n1 + n): 4 * (n1 + n) + 4].view(np.uint32)[0])
    fwd = raw[4 * (n1 + n) + 4:].view(np.uint32)
    assert len(fwd) == nf
    # oracle: the same trace (seed and generator as the C program), the
    # reference limits (1024 rules / 24 tbl8 groups, stop at first error)
    loaded = cg.rules_load_json(rf)
    pk = cg.gen_trace(0x5EED0C00, n, loaded)
    o = orc.OracleLpm(1024, 24)
    o.setup(loaded["ip"], loaded["depth"], loaded["next_hop"])
    # the drop-in runs the FW chain only (COP_DROPIN_STAGES, coprocessor.c:59-62)
    ro, fo, _ = orc.process(pk, n, stages=cg.STAGE_FW, fw=o)
    rp, _, _ = orc.process(pk, n, stages=cg.STAGE_PARSE | cg.STAGE_FW, fw=o)
    assert np.sum((rp["verdict"] == cg.DROP_PARSE) & (ro["verdict"] == 0)) > 0
    want = np.where(ro["verdict"] == 0, 0, -1).astype(np.int32)
    assert np.array_equal(ret1, want[:n1])
    assert np.array_equal(ret2, want)
    assert np.array_equal(fwd, fo)
    assert 0 < nf < n
