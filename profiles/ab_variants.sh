#!/bin/bash
# A/B on the C2 workload over element order x scatter x k_apply_tpe variant
# (ECM2_ELEMENT_ORDER / ECM2_SCATTER / ECM2_TPE_VARIANT experiment knobs):
#   variant 0 = row-loop kernel, 4 = LDS-X + double-buffered rows + in-wave face
#   assembly (default), +1 = plain stores only (diagnostic; wrong y), +8 = 2 waves/SIMD
set -u
for o in ${ORDERS:-auto}; do
for sc in ${SCATTERS:-partials}; do
for v in ${VARIANTS:-4}; do
  ECM2_ELEMENT_ORDER=$o ECM2_SCATTER=$sc ECM2_TPE_VARIANT=$v timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline "$@" \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('order', '$o', 'scatter', '$sc', 'variant', $v, d['value'], 'MDoF/s', d['ms_per_step'], 'ms/step', r['kernel_ms_avg'], 'ms', r['achieved'], 'GB/s', r['frac'])"
done
done
done
