#!/bin/bash
# Full GPU suite, then kernel traces of C4 and C5 (summation pass time per Mult).
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/sumcheck
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit $rc
for w in c4 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace_$w" -o run --output-format csv \
    -- python3 bench.py --workload $w --steps 50 --warmup 5 --no-cpu-baseline --full-layout 0 > "$O/bench_$w.json" 2> "$O/bench_$w.err" || exit $?
  find "$O/trace_$w" -name "*kernel_stats.csv" -exec grep -E "k_apply|k_sum" {} \; | cut -c1-60,200-
  python3 -c "import json; d=json.loads(open('$O/bench_$w.json').read().strip().splitlines()[-1]); print('$w', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
done
