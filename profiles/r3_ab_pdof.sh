#!/bin/bash
# GPU suite at the tree, then same-box A/Bs: b = 9601a19 minus the summation-pass change vs c = the
# summation pass issuing explicit-dof entries' dofs beside the descriptor staging (C4 with the
# reference's numbering, C3); then C5 with 2 x 2 x 2 bricks (ECM2_BRICKS=2) against 2 x 2 x 1
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r3pdof
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit $rc
bash profiles/ab_libs.sh pdof_c4e "libecm2pa_b.so libecm2pa_c.so" --workload c4 --steps 50 --warmup 5 --variants 0 --numbering entity || exit $?
bash profiles/ab_libs.sh pdof_c3 "libecm2pa_b.so libecm2pa_c.so" --workload c3 --steps 30 --warmup 5 || exit $?
for rep in 1 2; do
  for bz in 1 2; do
    ECM2_BRICKS=$bz timeout -k 10 300 python3 bench.py --workload c5 --steps 50 --warmup 5 --no-cpu-baseline --full-layout 0 > "$O/c5_bz${bz}_$rep.json" 2> "$O/c5_bz${bz}_$rep.err" || exit $?
    python3 -c "import json; d=json.loads(open('$O/c5_bz${bz}_$rep.json').read().strip().splitlines()[-1]); print('c5 bz=$bz rep $rep', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
  done
done
