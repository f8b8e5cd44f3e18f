"""Test configuration: registers the `gpu` marker and makes the package
`path-tracer_amd/` importable as `path_tracer_amd`."""
from __future__ import annotations

import importlib.util
import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG_DIR = ROOT / "path-tracer_amd"


def load_package():
    if "path_tracer_amd" in sys.modules:
        return sys.modules["path_tracer_amd"]
    spec = importlib.util.spec_from_file_location("path_tracer_amd", PKG_DIR / "__init__.py",
                                                  submodule_search_locations=[str(PKG_DIR)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["path_tracer_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


# Spectrum table cache shared by every test process (built on first use).
os.environ.setdefault("PT_SPECTRUM_TABLE", str(ROOT / "build" / "sRGBSpectrumTable.dat"))
sys.path.insert(0, str(Path(__file__).resolve().parent))
load_package()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def pt():
    return load_package()
