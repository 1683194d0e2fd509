#!/bin/bash
# bench.py contract tests, then the default line (pin still used at the default size)
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests/test_bench.py -m gpu -v --timeout 300 --timeout-method thread > "$O/pytest_bench.log" 2>&1
rc=$?
tail -4 "$O/pytest_bench.log"; grep -E "FAILED|ERROR|Error" "$O/pytest_bench.log" | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --full-layout 0 > "$O/bench_default.json" 2> "$O/bench_default.err" || exit $?
python3 -c "import json; b=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1]); print(b['value'], b['roofline']['traffic'], b['roofline']['achieved_basis'])"
