import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ppo.c_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libppo's HIP kernels)")


@pytest.fixture(scope="session")
def oracle():
    import oracle_ffi

    oracle_ffi.build()
    oracle_ffi.load()
    return oracle_ffi


@pytest.fixture(scope="session")
def lib_built():
    """libppo.so loaded (built if absent) — CPU tests only inspect it, never compute."""
    if not os.path.exists(os.path.join(PKG, "lib", "libppo.so")):
        subprocess.run(["make", "-j8", "-C", PKG], check=True)
    import ppo_ffi

    return ppo_ffi.load()


@pytest.fixture(scope="session")
def lib(lib_built):
    """libppo on a GPU: any failure to find the device is an error, never a skip."""
    n = lib_built.ppo_device_count()
    if n < 1:
        raise RuntimeError("no HIP device visible: GPU tests need an MI355X")
    assert lib_built.ppo_set_device(0) == 0
    return lib_built
