#!/usr/bin/env python3
"""Run bench.py against another build of the library (same-box A/B of a kernel change):
python3 profiles/ab_lib.py <path/to/libecm2pa.so> [bench.py args...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

if __name__ == "__main__":
    lib = sys.argv[1]
    E = bench.load_pkg()
    E.load_library(lib)  # cached: bench's own load_library() returns this one
    sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
    bench.main()
