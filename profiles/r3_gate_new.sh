#!/bin/bash
# round 3: the new GPU tests (attribute markers, RCCL rows of a non-empty schedule), then the suite
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r3new
mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
   -k "marker or rccl_rows" > "$O/pytest_new.log" 2>&1
rc=$?
tail -3 "$O/pytest_new.log"; grep -E "FAILED|ERROR" "$O/pytest_new.log" | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
exit $rc
