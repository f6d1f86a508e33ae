"""The drop-in's NF chain follows the reference's stage macros
(coprocessor.h:19-21): ENABLE_FW_NF (always defined by the reference's
coprocessor.h:21) -> the firewall stage; DISABLE_NF -> no NF stage (switch.c
never calls the coprocessor, switch.c:411,426,524; a call anyway forwards
every packet, as process_packet does without ENABLE_FW_NF, coprocessor.c:59-64).
The macros live in the caller's build: cop_gpu.h aliases coprocessor_setup
to the chain's setup function (cop_coprocessor_setup_fw / _no_nf), an
object-like macro, so the reference's own `int coprocessor_setup(void);`
(coprocessor.h:30) still compiles after it. CPU only: the
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

# the reference's coprocessor.h:23-30 declarations after the header, and a
# function pointer to the setup (a function-like macro broke both)
REF_DECLS = r'''
#include "cop_gpu.h"
int coprocessor_setup(void);
int coprocessor_teardown(void);
int process_packet(struct rte_mbuf *pkt);
int (*setup_fn)(void) = &coprocessor_setup;
int use(void) { return coprocessor_setup() + setup_fn(); }
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
    fn = "cop_coprocessor_setup_no_nf(" if want == 0 else "cop_coprocessor_setup_fw("
    assert fn in pre.split("int use(void)")[1]


@pytest.mark.parametrize("defs", [(), ("ENABLE_FW_NF=1",), ("DISABLE_NF",)])
def test_reference_declarations_after_header(tmp_path, defs):
    c = tmp_path / "d.c"
    c.write_text(REF_DECLS)
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-c", "-o", str(tmp_path / "d.o"),
                        f"-I{INC}", *[f"-D{d}" for d in defs], str(c)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_chain_setters_exported():
    L = cg.lib()
    assert L.cop_coprocessor_setup_fw is not None and L.cop_coprocessor_setup_no_nf is not None


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
