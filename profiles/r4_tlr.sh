#!/bin/bash
# Round 4: the TRILINEAR lattice kernel with the plane-only map coefficients (c1, c2, c4) re-read per
# plane instead of held through the rows (ECM2_TLB_RELOAD=1: 254-256 VGPRs, no spills, against 11-14
# spilled values) -- parity on the trilinear tests with the variant library, then a same-box A/B on the
# trilinear C4 mesh and the drop-in configuration.  (Adopted: the reload is unconditional since 1d6d7f2 and
# the ECM2_TLB_RELOAD switch is gone; the variant library was built at 64edb79 + -DECM2_TLB_RELOAD=1.)
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r4tlr
mkdir -p "$O"
export TMPDIR=/tmp
# (the variant library loaded first: the package caches it, so the tests run on it)
timeout -k 10 300 python -u -c "import sys, importlib; sys.path.insert(0, '.'); sys.path.insert(0, 'tests'); import torch; \
import helpers; E = helpers.load_pkg(); E.load_library('cardiac-ablation-ecm2_amd/lib/libecm2pa_tlr.so'); \
import pytest; sys.exit(pytest.main(['-x', '-q', '--timeout', '200', '--timeout-method', 'thread', '-m', 'gpu', \
'tests/test_gpu_parity.py', 'tests/test_gpu_configs.py', '-k', 'trilinear or jacobian or drop_in']))" > "$O/tests.txt" 2>&1 || { tail -30 "$O/tests.txt"; exit 1; }
tail -1 "$O/tests.txt"
bash profiles/ab_libs.sh tlr_tri "libecm2pa.so libecm2pa_tlr.so" --workload c4 --mesh trilinear --steps 30 --warmup 5 --variants 0 || exit $?
bash profiles/ab_libs.sh tlr_dropin "libecm2pa.so libecm2pa_tlr.so" --workload c4 --numbering entity --mesh trilinear --geometry-input jacobians --steps 30 --warmup 5 --variants 0 || exit $?
