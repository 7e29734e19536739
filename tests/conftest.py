import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "uu-infogr-raytracer_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device; runs the HIP path")


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.lib()
    return pyoracle


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def rtlib():
    """The product library (libraytracer_hip.so); built on demand with the in-tree Makefile."""
    from raytracer_hip import abi
    if not os.path.exists(abi.LIB_PATH):
        import subprocess
        subprocess.run(["make", "-s", "-C", os.path.join(PKG, "csrc")], check=True)
    return abi.load_library()


@pytest.fixture(scope="session")
def gpu_ctx(rtlib):
    """A single-GPU context (GPU tests only).  Fails loudly without a device."""
    from raytracer_hip import Context
    ctx = Context(1)
    yield ctx
    ctx.close()
