#!/bin/bash
# Round-2 closing gate: the whole -m gpu suite, the default bench line (C4), C5, and the loopback
# N = 8 group line (all members on one GPU, serialised: a plumbing check of the partitioned path).
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > "$O/bench_c4.json" 2> "$O/bench_c4.err" || exit $?
tail -1 "$O/bench_c4.json"
timeout -k 10 400 python3 bench.py --workload c5 --steps 30 --warmup 5 --full-layout 0 --no-cpu-baseline > "$O/bench_c5.json" 2> "$O/bench_c5.err" || exit $?
tail -1 "$O/bench_c5.json"
timeout -k 10 400 python3 bench.py --loopback 8 --steps 20 --warmup 3 --no-cpu-baseline > "$O/bench_c4_lb8.json" 2> "$O/bench_c4_lb8.err" || exit $?
tail -1 "$O/bench_c4_lb8.json"
