#!/bin/bash
# closing check at HEAD: whole GPU suite, smoke(), the default bench line (C4) and C5
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/head
mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -2 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit $?
tail -1 "$O/smoke.log"
timeout -k 10 400 python3 bench.py > "$O/bench_c4.json" 2> "$O/bench_c4.err" || exit $?
tail -1 "$O/bench_c4.json" | cut -c1-400
timeout -k 10 400 python3 bench.py --workload c5 --steps 30 --warmup 5 --full-layout 0 > "$O/bench_c5.json" 2> "$O/bench_c5.err" || exit $?
tail -1 "$O/bench_c5.json" | cut -c1-400
