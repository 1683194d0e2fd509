#!/bin/bash
# Plan classes at 24^3 (diagnostic), GPU suite at the tree, then same-box A/B: c = HEAD vs e = 2D
# summation runs that join slot-affine 1D runs as explicit-dof runs
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r3join
mkdir -p "$O"
timeout -k 10 200 python3 -u profiles/r3_plan_dump.py 24 > "$O/plan_dump.txt" 2>&1 || exit $?
grep -E "^plan|plan info" "$O/plan_dump.txt"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit $rc
bash profiles/ab_libs.sh join_c4e "libecm2pa_c.so libecm2pa_e.so" --workload c4 --steps 50 --warmup 5 --variants 0 --numbering entity || exit $?
bash profiles/ab_libs.sh join_c4 "libecm2pa_c.so libecm2pa_e.so" --workload c4 --steps 50 --warmup 5 --variants 0 || exit $?
bash profiles/ab_libs.sh join_c3 "libecm2pa_c.so libecm2pa_e.so" --workload c3 --steps 30 --warmup 5 || exit $?
