#!/bin/bash
# A/B of the summation pass's XCD-contiguous block order (ECM2_SUM_XCD=1) on C2, C4, C5 (one call).
set -u
line() { python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$1', d['value'], 'MDoF/s', d['ms_per_step'], 'ms/step', r['kernel_ms_avg'], 'ms')"; }
for rep in 1 2; do for w in c2 c4 c5; do for v in 0 1; do
  ECM2_SUM_XCD=$v timeout -k 10 200 python3 bench.py --workload $w --steps 50 --warmup 5 --no-cpu-baseline | line "$w sum_xcd $v"
done; done; done
