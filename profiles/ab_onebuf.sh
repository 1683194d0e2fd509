#!/bin/bash
# A/B on C5 (p=4, 68^3, 20.3M DoF, AFFINE_E): brick kernel LDS / qdata-load variants
# (ECM2_BRICK_VARIANT bit 1: AFFINE_E pairs loaded in the z stage; bit 4: one LDS buffer per element)
set -u
for rep in 1 2; do
for v in ${VARIANTS:-0 1 4 5}; do
  ECM2_BRICK_VARIANT=$v timeout -k 10 200 python3 bench.py --workload c5 --steps 30 --warmup 5 --no-cpu-baseline "$@" \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c5 brick variant', '$v', d['value'], 'MDoF/s', d['ms_per_step'], 'ms/step', r['kernel_ms_avg'], 'ms kernel', r['frac'])"
done
done
