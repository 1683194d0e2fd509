#!/bin/bash
# Round-2 A/B of the thread-per-element kernel's regular-block addressing (C4). NOTE: the
# ECM2_TPE_REG_OFF switch was removed after this run; the script is the recipe of
# profiles/r2_ab_treg.txt.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/ab_treg
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -2 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in off on; do
    if [ $v = off ]; then export ECM2_TPE_REG_OFF=1; else unset ECM2_TPE_REG_OFF; fi
    timeout -k 10 300 python3 bench.py --workload c4 --steps 50 --warmup 5 --no-cpu-baseline --full-layout 0 > "$O/bench_${v}_$rep.json" 2> "$O/bench_${v}_$rep.err" || exit $?
    python3 -c "import json; d=json.loads(open('$O/bench_${v}_$rep.json').read().strip().splitlines()[-1]); print('reg=$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
  done
done
