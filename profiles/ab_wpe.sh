#!/bin/bash
# A/B of the workgroup-per-element kernel on C5 (p=4): ECM2_WPE_VARIANT 0 = default,
# 1 = plain stores (diagnostic, wrong y), 2 = qdata prefetch, 3 = both
set -u
for v in ${VARIANTS:-0 1 2 3}; do
  ECM2_WPE_VARIANT=$v timeout -k 10 200 python3 bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline "$@" \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('wpe variant', $v, d['value'], 'MDoF/s', d['ms_per_step'], 'ms/step', r['kernel_ms_avg'], 'ms', r['achieved'], 'GB/s', r['frac'])"
done
