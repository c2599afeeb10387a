"""Shared fixtures. `-m gpu` tests need an MI355X; everything else runs on CPU.

The product package lives in `icl-mixed-precision-gmres_amd/` (not a Python
identifier) and is loaded through its file path; the CPU oracle (`oracle/`)
is the parity checker and is only ever imported from tests.
"""
import importlib.util
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))


def load_package():
    if "mpgmres_amd" in sys.modules:
        return sys.modules["mpgmres_amd"]
    pkg_dir = REPO / "icl-mixed-precision-gmres_amd"
    spec = importlib.util.spec_from_file_location("mpgmres_amd", pkg_dir / "__init__.py",
                                                  submodule_search_locations=[str(pkg_dir)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["mpgmres_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct MI355X (gfx950) and the built HIP libraries")
    config.addinivalue_line("markers", "slow: long-running case")


@pytest.fixture(scope="session")
def mpg():
    return load_package()


@pytest.fixture(scope="session")
def oracle():
    from oracle import binding

    binding.lib()
    return binding


@pytest.fixture(scope="session")
def hip(mpg):
    """Kernel-level C-ABI + one context on device 0."""
    from tests.devbuf import Hip

    h = Hip(mpg.hip_lib())
    yield h
    h.close()
