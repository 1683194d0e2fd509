#!/bin/bash
# serial schedule: graph replay vs direct launches per member Mult (emulated C4 ranks)
set -uo pipefail
echo "-- serial, direct launches"; ECM2_PAR_SCHEDULE=serial TAG=_serial_direct EXTRA="--member-graph 0" bash profiles/member_emul.sh 2 4 8 || exit $?
echo "-- serial, graph"; ECM2_PAR_SCHEDULE=serial TAG=_serial_graph bash profiles/member_emul.sh 8 || exit $?
ECM2_PAR_SCHEDULE=serial TAG=_serial_direct EXTRA="--member-graph 0" bash profiles/member_trace.sh 8 3 || exit $?
