#!/bin/bash
# A/B of the brick traversal order (ECM2_BRICK_CURVE: lex | morton) on C2 and C4
set -u
line() { python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$1', d['value'], 'MDoF/s', d['ms_per_step'], 'ms/step', r['kernel_ms_avg'], 'ms', r['achieved'], 'GB/s', r['frac'])"; }
for c in lex morton; do
  ECM2_BRICK_CURVE=$c timeout -k 10 200 python3 bench.py --workload c2 --steps 100 --warmup 10 --no-cpu-baseline | line "c2 curve $c"
  ECM2_BRICK_CURVE=$c timeout -k 10 200 python3 bench.py --workload c4 --steps 30 --warmup 3 --no-cpu-baseline | line "c4 curve $c"
done
