#!/bin/bash
# whole GPU suite (serial schedule now the default), then the emulated ranks of both schedules
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit $rc
echo "-- serial (direct)"; TAG=_serial bash profiles/member_emul.sh 2 4 8 || exit $?
echo "-- overlap (graph)"; TAG=_overlap EXTRA="--schedule overlap" bash profiles/member_emul.sh 2 4 8 || exit $?
TAG=_serial bash profiles/member_trace.sh 8 0 8 7 4 1 2 1 || exit $?
