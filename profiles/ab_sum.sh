#!/bin/bash
# A/B of the second-pass list order (ECM2_SUM_ORDER: slot | dof) on C2 and C5
set -u
line() { python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$1', d['value'], 'MDoF/s', d['ms_per_step'], 'ms/step', r['kernel_ms_avg'], 'ms', r['achieved'], 'GB/s', r['frac'])"; }
for o in slot dof; do
  ECM2_SUM_ORDER=$o timeout -k 10 200 python3 bench.py --workload c2 --steps 100 --warmup 10 --no-cpu-baseline | line "c2 sum order $o"
  ECM2_SUM_ORDER=$o timeout -k 10 200 python3 bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline | line "c5 sum order $o"
done
