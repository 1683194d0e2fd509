#!/bin/bash
# member-emulation gate: its parity test, then the emulated per-rank C4 Mult at N = 2, 4, 8
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "member_rows or loopback_group_matches_serial" > "$O/pytest_member.log" 2>&1
rc=$?
tail -3 "$O/pytest_member.log"; grep -E "FAILED|Error" "$O/pytest_member.log" | head
[ $rc -eq 0 ] || exit $rc
bash profiles/member_emul.sh ${@:-2 4 8} | tee "$O/member_emul.txt"
