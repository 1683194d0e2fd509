#!/bin/bash
# cooperative lattice gather for regular p<=2 blocks: suite, then same-box A/B (before = per-lane gather)
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -2 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit $rc
bash profiles/ab_lib_r2.sh latg_c4 --workload c4 --steps 50 --warmup 5 || exit $?
bash profiles/ab_member_r2.sh latg 8 4 || exit $?
bash profiles/ab_lib_r2.sh latg_c2 --workload c2 --steps 50 --warmup 5 || exit $?
