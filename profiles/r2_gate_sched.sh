#!/bin/bash
# Serial vs overlapped distributed-Mult schedule: the distributed GPU tests under the serial
# schedule, then the emulated per-rank C4 Mult (member_emul.sh) under both, then a serial trace.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
ECM2_PAR_SCHEDULE=serial timeout -k 10 400 python3 -u -m pytest tests/test_distributed.py tests/test_gpu_configs.py -m gpu -x -v --timeout 200 --timeout-method thread > "$O/pytest_serial.log" 2>&1
rc=$?
tail -3 "$O/pytest_serial.log"; grep -E "FAILED|Error" "$O/pytest_serial.log" | head
[ $rc -eq 0 ] || exit $rc
echo "-- serial"; ECM2_PAR_SCHEDULE=serial TAG=_serial bash profiles/member_emul.sh 2 4 8 || exit $?
echo "-- overlap"; TAG=_overlap bash profiles/member_emul.sh 2 4 8 || exit $?
ECM2_PAR_SCHEDULE=serial TAG=_serial bash profiles/member_trace.sh 8 3 2 0 || exit $?
