#!/bin/bash
# GPU suite at the tree, then a same-box A/B on C5 (p = 4 brick kernel): b = HEAD before vs
# c = the final stage driven by the per-(D, BZ) lattice-point table (no per-point holder derivation)
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r3bpt
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit $rc
bash profiles/ab_libs.sh bpt_c5 "libecm2pa_b.so libecm2pa_c.so" --workload c5 --steps 50 --warmup 5 || exit $?
