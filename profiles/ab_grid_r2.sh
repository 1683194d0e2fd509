#!/bin/bash
# NOTE: the grid mode and its ECM2_GRID_OFF switch were deleted after this run (profiles/r2_ab_grid.txt).
# Round-2 A/B of grid-computed unit origins (no table load before the first loads) at C5 / C4.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/ab_grid
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -2 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit $rc
for w in ${WORKLOADS:-c5}; do
for rep in 1 2; do
  for v in off on; do
    if [ $v = off ]; then export ECM2_GRID_OFF=1; else unset ECM2_GRID_OFF; fi
    timeout -k 10 300 python3 bench.py --workload $w --steps 50 --warmup 5 --no-cpu-baseline --full-layout 0 > "$O/bench_${w}_${v}_$rep.json" 2> "$O/bench_${w}_${v}_$rep.err" || exit $?
    python3 -c "import json; d=json.loads(open('$O/bench_${w}_${v}_$rep.json').read().strip().splitlines()[-1]); print('$w grid=$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
  done
done
done
