#!/bin/bash
# A/B on C5 (p=4, 68^3, 20.3M DoF): kernel (line | wpe) x scatter (partials | atomic)
set -u
for k in ${KERNELS:-line wpe}; do
for sc in ${SCATTERS:-partials atomic}; do
  ECM2_SCATTER=$sc timeout -k 10 200 python3 bench.py --workload c5 --kernel $k --steps 20 --warmup 3 --no-cpu-baseline "$@" \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c5 kernel', '$k', 'scatter', '$sc', d['value'], 'MDoF/s', d['ms_per_step'], 'ms/step', r['kernel_ms_avg'], 'ms', r['achieved'], 'GB/s', r['frac'])"
done
done
