"""Shared test setup: registers the `gpu` marker, exposes the package as `ecm2_amd`
(its directory name contains hyphens) and the oracle as `oracle`."""
import importlib.util
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _load_pkg():
    if "ecm2_amd" in sys.modules:
        return sys.modules["ecm2_amd"]
    pkg_dir = os.path.join(ROOT, "cardiac-ablation-ecm2_amd")
    spec = importlib.util.spec_from_file_location("ecm2_amd", os.path.join(pkg_dir, "__init__.py"),
                                                  submodule_search_locations=[pkg_dir])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["ecm2_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


_load_pkg()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
