#!/bin/bash
# serial schedule with the interior-anchored brick order: parity, emulated ranks (direct), trace
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
ECM2_PAR_SCHEDULE=serial timeout -k 10 400 python3 -u -m pytest tests/test_distributed.py tests/test_gpu_configs.py -m gpu -x -v --timeout 200 --timeout-method thread > "$O/pytest_serial.log" 2>&1
rc=$?
tail -2 "$O/pytest_serial.log"; grep -E "FAILED|Error" "$O/pytest_serial.log" | head
[ $rc -eq 0 ] || exit $rc
ECM2_PAR_SCHEDULE=serial TAG=_serial_direct EXTRA="--member-graph 0" bash profiles/member_emul.sh 2 4 8 || exit $?
ECM2_PAR_SCHEDULE=serial TAG=_serial_direct EXTRA="--member-graph 0" bash profiles/member_trace.sh 8 3 || exit $?
