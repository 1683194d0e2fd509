#!/bin/bash
# GPU suite at the tree (brick kernel with the next-brick cache prefetch), then a same-box A/B of
# the prefetch distance on C5 (ECM2_BRICK_PFD = 0 off, 160, 320 bricks), alternating, twice
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r3pfd
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for pfd in 0 160 320 80; do
    ECM2_BRICK_PFD=$pfd timeout -k 10 300 python3 bench.py --workload c5 --steps 50 --warmup 5 --no-cpu-baseline --full-layout 0 > "$O/c5_pfd${pfd}_$rep.json" 2> "$O/c5_pfd${pfd}_$rep.err" || exit $?
    python3 -c "import json; d=json.loads(open('$O/c5_pfd${pfd}_$rep.json').read().strip().splitlines()[-1]); print('c5 pfd=$pfd rep $rep', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
  done
done
