import importlib.util
import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
PKG_DIR = ROOT / "ue22cs343bb1-openmp-assignment_amd"
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libdash on the device)")


def load_dash():
    """The product's Python mirror (ue22cs343bb1-openmp-assignment_amd/dash.py)."""
    name = "dash_amd"
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, PKG_DIR / "dash.py")
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def dash():
    mod = load_dash()
    if not mod.LIB_PATH.exists():
        mod.build()
    return mod


@pytest.fixture(scope="session")
def oracle():
    import oracle_ctypes
    oracle_ctypes.lib()
    return oracle_ctypes
