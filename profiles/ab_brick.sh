#!/bin/bash
# A/B of the p >= 3 brick kernel on C5 (68^3, p = 4): ECM2_LINE_BRICK = 0 (per-element line
# kernel), 1 (2 x 2 x 1 elements per workgroup), 2 (2 x 2 x 2) x ECM2_BRICK_VARIANT
set -u
for bz in ${BRICKS:-0 1 2}; do
for v in ${VARIANTS:-0 1}; do
  ECM2_LINE_BRICK=$bz ECM2_BRICK_VARIANT=$v timeout -k 10 200 python3 bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline "$@" \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c5 bricks', $bz, 'variant', $v, d['value'], 'MDoF/s', d['ms_per_step'], 'ms/step', r['kernel_ms_avg'], 'ms', r['achieved'], 'GB/s', r['frac'])"
  if [ "$bz" = 0 ]; then break; fi
done
done
