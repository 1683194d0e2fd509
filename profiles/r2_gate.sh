#!/bin/bash
# Round-2 GPU gate: the whole -m gpu suite, then the default bench line (C4) and C5.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -5 "$O/pytest_gpu.log"
grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > "$O/bench_c4.json" 2> "$O/bench_c4.err" || exit $?
cat "$O/bench_c4.json"
[ "${1:-}" = "ab" ] && bash profiles/ab_brick_r2.sh
exit $rc
