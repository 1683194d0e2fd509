#!/bin/bash
# GPU suite at the tree (summation pass with 2 plan blocks per workgroup), then same-box A/Bs of
# the pass with 1 / 2 / 4 plan blocks per workgroup (every block's partial loads issued before
# any sum: more bytes in flight per thread) on C5, C4 (both numberings) and C3
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r3bpw
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit $rc
L="libecm2pa_bpw1.so libecm2pa_bpw2.so libecm2pa_bpw4.so"
bash profiles/ab_libs.sh bpw_c5 "$L" --workload c5 --steps 50 --warmup 5 || exit $?
bash profiles/ab_libs.sh bpw_c4 "$L" --workload c4 --steps 50 --warmup 5 --variants 0 || exit $?
bash profiles/ab_libs.sh bpw_c4e "$L" --workload c4 --steps 50 --warmup 5 --variants 0 --numbering entity || exit $?
bash profiles/ab_libs.sh bpw_c3 "$L" --workload c3 --steps 30 --warmup 5 || exit $?
