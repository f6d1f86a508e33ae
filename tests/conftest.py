import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ghost-dataplane_amd")
ORACLE = os.path.join(ROOT, "oracle")
for p in (PKG, ORACLE, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP path)")


def _ensure_built():
    # Build in-tree if a library is missing (here: cross-compile for gfx950;
    # on the GPU box the prebuilt .so files from the snapshot are used).
    if not os.path.exists(os.path.join(PKG, "libcopgpu.so")):
        subprocess.run(["make", "-C", PKG, "-j8"], check=True)
    if not os.path.exists(os.path.join(ORACLE, "liboracle.so")):
        subprocess.run(["make", "-C", ORACLE], check=True)
    if os.path.isdir("/root/reference") and not os.path.exists(os.path.join(ORACLE, "_ref", "libcjson_ref.so")):
        subprocess.run(["make", "-C", ORACLE, "ref"], check=True)


_ensure_built()


@pytest.fixture
def gpu_ctx_factory():
    import copgpu as cg

    if cg.device_count() < 1:
        pytest.fail("GPU test on a machine without a visible GPU")
    made = []

    def make(**kw):
        c = cg.Context(**kw)
        made.append(c)
        return c

    yield make
    for c in made:
        c.close()
