#!/bin/bash
# (Needs the split-schedule experiment code, measured and removed: profiles/r2_ab_split.txt; kept as the record of the run.)
# split variant of the serial schedule: distributed GPU tests, then emulated ranks serial vs split (direct)
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests/test_distributed.py tests/test_gpu_configs.py -m gpu -x -v --timeout 200 --timeout-method thread > "$O/pytest_split.log" 2>&1
rc=$?
tail -2 "$O/pytest_split.log"; grep -E "FAILED|ERROR" "$O/pytest_split.log" | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
echo "-- serial"; TAG=_serial bash profiles/member_emul.sh 2 4 8 || exit $?
echo "-- split"; TAG=_split EXTRA="--schedule split" bash profiles/member_emul.sh 2 4 8 || exit $?
done
TAG=_split EXTRA="--schedule split" bash profiles/member_trace.sh 8 3 || exit $?
