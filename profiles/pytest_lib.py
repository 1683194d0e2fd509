#!/usr/bin/env python3
"""Run pytest against another build of the library (parity of an A/B build before it is timed):
python3 profiles/pytest_lib.py <path/to/libecm2pa.so> [pytest args...]

The package is registered as `ecm2_amd` exactly as tests/conftest.py and bench.py do, and the given
library is loaded first, so every test's load_library() returns it."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import pytest  # noqa: E402

if __name__ == "__main__":
    lib = sys.argv[1]
    E = bench.load_pkg()
    E.load_library(lib)
    sys.exit(pytest.main(sys.argv[2:]))
