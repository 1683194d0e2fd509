#!/bin/bash
# round 3 (session 2): GPU suite at HEAD, then the default bench line
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r3head
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py > "$O/bench.json" 2> "$O/bench.err"
rc=$?
cat "$O/bench.json"
exit $rc
