#!/bin/bash
# Distributed-Mult schedules on the emulated C4 ranks (profiles/r2_member_emul.txt): serial with direct
# launches (the default), serial with a HIP graph per Mult, overlapped with a graph (round 1's default),
# each at N = 2, 4, 8 on one box, then the serial kernel timeline of member 3 at N = 8.
# (Blocks 2-4 of r2_member_emul.txt were measured with intermediate builds whose environment switch
# this script's flags replace: --schedule, --member-graph.)
set -uo pipefail
echo "-- serial, direct"; TAG=_serial bash profiles/member_emul.sh ${@:-2 4 8} || exit $?
echo "-- serial, graph"; TAG=_serial_graph EXTRA="--member-graph 1" bash profiles/member_emul.sh ${@:-2 4 8} || exit $?
echo "-- overlap, graph"; TAG=_overlap EXTRA="--schedule overlap" bash profiles/member_emul.sh ${@:-2 4 8} || exit $?
TAG=_serial bash profiles/member_trace.sh 8 3 || exit $?
