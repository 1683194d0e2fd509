#!/bin/bash
# A/B of k_apply_tpe variants on the C2 workload (ECM2_TPE_VARIANT experiment knob):
#   0 = row-loop kernel (default), 4 = LDS-X + register double-buffered rows,
#   +1 = plain stores instead of atomics (diagnostic; wrong y), +2 = default-policy loads
set -u
for o in ${ORDERS:-auto}; do
for v in ${VARIANTS:-0 4 5 6 7}; do
  ECM2_ELEMENT_ORDER=$o ECM2_TPE_VARIANT=$v timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline "$@" \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('order', '$o', 'variant', $v, d['value'], 'MDoF/s', r['kernel_ms_avg'], 'ms', r['achieved'], 'GB/s', r['frac'])"
done
done
