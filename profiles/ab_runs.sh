#!/bin/bash
# A/B of the TPE partial-slot layout: contiguous per-dof runs (ECM2_PART_RUNS=1) vs dense
# slots through a slot list (default), C2 / C4 / C3.
set -eu
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
for w in ${WORKLOADS:-c2 c4 c3}; do
for r in 1 0; do
  steps=50; [ "$w" = c2 ] && steps=200; [ "$w" = c3 ] && steps=20
  ECM2_PART_RUNS=$r timeout -k 10 300 python3 bench.py --workload $w --steps $steps --warmup 5 --no-cpu-baseline > "$O/ab_runs_${w}_${r}.json"
  python3 -c "import json; d=json.load(open('$O/ab_runs_${w}_${r}.json')); r=d['roofline']; print('$w', 'runs=$r', d['value'], 'MDoF/s', d['ms_per_step'], 'ms/step', r['kernel_ms_avg'], 'ms', (d.get('pcg') or {}).get('mdof_iter_per_s'))"
done
done
