"""The drop-in's NF chain follows the reference's stage macros
(coprocessor.h:19-21): ENABLE_FW_NF (always defined by the reference's
coprocessor.h:21) -> the firewall stage; DISABLE_NF -> no NF stage (switch.c
never calls the coprocessor, switch.c:411,426,524; a call anyway forwards
every packet, as process_packet does without ENABLE_FW_NF, coprocessor.c:59-64).
The macros live in the caller's build: cop_gpu.h turns coprocessor_setup()
into cop_coprocessor_setup_stages(COP_DROPIN_STAGES). CPU only: the
preprocessor and the run-time setter (no GPU call)."""
import os
import subprocess

import pytest

import copgpu as cg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")

SRC = r'''
#include "cop_gpu.h"
#include <stdio.h>
int main(void) { printf("%u\n", (unsigned)COP_DROPIN_STAGES); return 0; }
int use(void) { return coprocessor_setup(); }
'''


def expand(tmp_path, *defs):
    c = tmp_path / "m.c"
    c.write_text(SRC)
    exe = tmp_path / "m"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-c", "-o", str(tmp_path / "m.o"), f"-I{INC}",
                    *[f"-D{d}" for d in defs], str(c)], check=True)
    pre = subprocess.run(["gcc", "-E", "-P", f"-I{INC}", *[f"-D{d}" for d in defs], str(c)], check=True,
                         capture_output=True, text=True).stdout
    subprocess.run(["gcc", "-std=c99", "-o", str(exe), f"-I{INC}", *[f"-D{d}" for d in defs], "-DCOP_NO_DROPIN_MACROS",
                    "-x", "c", "-"], input=SRC.replace("int use(void) { return coprocessor_setup(); }", ""),
                   text=True, check=True)
    val = int(subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout)
    return val, pre


@pytest.mark.parametrize("defs,want", [((), 2), (("ENABLE_FW_NF=1",), 2), (("DISABLE_NF",), 0),
                                       (("COP_DROPIN_NO_NF",), 0)])
def test_macros_select_the_dropin_chain(tmp_path, defs, want):
    val, pre = expand(tmp_path, *defs)
    assert val == want
    assert "cop_coprocessor_setup_stages(" in pre.split("int use(void)")[1]


def test_runtime_setter():
    L = cg.lib()
    try:
        assert L.cop_dropin_stages() == cg.STAGE_FW          # the reference's default chain
        assert L.cop_set_dropin_stages(0) == 0
        assert L.cop_dropin_stages() == 0
        assert L.cop_set_dropin_stages(cg.STAGE_PARSE) < 0   # parse/route belong to the fast path
        assert L.cop_set_dropin_stages(cg.STAGE_LPM | cg.STAGE_FW) < 0
    finally:
        L.cop_set_dropin_stages(cg.STAGE_FW)
