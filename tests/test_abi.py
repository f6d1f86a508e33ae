"""The C-ABI boundary: libcopgpu.so loads and exports every function that
include/cop_gpu.h declares; the header is plain C (no HIP/CUDA/torch
types); without a GPU the context API fails cleanly (-ENODEV)."""
import ctypes
import os
import re
import subprocess

import copgpu as cg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "cop_gpu.h")


def declared_functions():
    text = open(HDR).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    text = re.sub(r"typedef[^;]*;", "", text)
    names = set()
    for m in re.finditer(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\(([^()]*)\)\s*;", text):
        names.add(m.group(1))
    return names


def test_header_declares_the_reference_api():
    names = declared_functions()
    for f in ("coprocessor_setup", "coprocessor_teardown", "process_packet", "cop_submit", "cop_sync",
              "cop_ring_enqueue_bulk", "cop_ring_dequeue_burst", "cop_lpm_build", "cop_rules_load_json",
              "cop_coprocessor_poll"):
        assert f in names, f


def test_every_declared_symbol_is_exported():
    out = subprocess.run(["nm", "-D", "--defined-only", cg.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = declared_functions() - exported
    assert not missing, missing
    lib = cg.lib()
    for name in declared_functions():
        assert getattr(lib, name) is not None
    assert declared_functions() <= set(cg.SIGNATURES), declared_functions() - set(cg.SIGNATURES)


def test_header_is_plain_c():
    text = re.sub(r"/\*.*?\*/", "", open(HDR).read(), flags=re.S)
    for bad in ("hip_runtime", "cuda", "torch", "hipStream_t", "__global__", "#ifdef __HIP"):
        assert bad not in text
    # compiles as C99 on its own, with and without the reference stage macros
    for extra in ([], ["-DENABLE_FW_NF"], ["-DDISABLE_NF"]):
        r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-fsyntax-only", "-x", "c", "-I",
                            os.path.join(ROOT, "include"), "-"] + extra,
                           input='#include "cop_gpu.h"\nint main(void){return COP_DEFAULT_STAGES;}\n',
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr


def test_struct_layouts():
    assert ctypes.sizeof(cg.Batch) == 56
    assert cg.PREFIX_DT.itemsize == 12
    assert cg.RESULT_DT.itemsize == 8


def test_struct_layouts_match_c(tmp_path):
    """Every struct the binding mirrors has the C compiler's size and field
    offsets (compiled from include/cop_gpu.h)."""
    mirrors = {"cop_batch": cg.Batch, "cop_batch_ring": cg.BatchRing, "cop_config": cg.Config,
               "cop_lpm_config": cg.LpmConfig, "cop_lpm_report": cg.LpmReport, "cop_trace_opts": cg.TraceOpts,
               "cop_nf_stats": cg.NfStats, "cop_port_stats": cg.PortStats}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "cop_gpu.h"', "int main(void){"]
    for cname, py in mirrors.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines.append('printf("cop_counters size %zu\\n", sizeof(cop_counters));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    r = subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    got = {tuple(l.split()[:2]): int(l.split()[2]) for l in out if l.strip()}
    for cname, py in mirrors.items():
        assert got[(cname, "size")] == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert got[(cname, f)] == getattr(py, f).offset, (cname, f)
    assert got[("cop_counters", "size")] == 16 * 8


def test_no_gpu_fails_cleanly():
    if cg.device_count() > 0:
        return   # covered by the gpu tests
    import pytest
    with pytest.raises(cg.CopError) as e:
        cg.Context()
    assert e.value.code == -19   # -ENODEV
    assert cg.lib().coprocessor_setup() != 0
    assert cg.lib().process_packet(None) == -1
