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
timeout -k 10 400 python3 bench.py --workload c5 --steps 30 --warmup 5 --full-layout 0 --no-cpu-baseline > "$O/bench_c5.json" 2> "$O/bench_c5.err" || exit $?
cat "$O/bench_c5.json"
if [ "${1:-}" = "ab" ]; then bash profiles/ab_brick_r2.sh || exit $?; fi
if [ "${1:-}" = "sq" ]; then bash profiles/sq_pass.sh c5 --workload c5 --steps 10 --warmup 2 --full-layout 0 || exit $?; fi
exit $rc
