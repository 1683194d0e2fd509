#!/bin/bash
# A/B of the line kernel on C5: chunk length (ECM2_LINE_CHUNK) x qdata prefetch (ECM2_LINE_VARIANT)
set -u
for ch in ${CHUNKS:-1 2 4 8}; do
for v in ${VARIANTS:-0 2}; do
  ECM2_LINE_CHUNK=$ch ECM2_LINE_VARIANT=$v timeout -k 10 200 python3 bench.py --workload c5 --kernel line --steps 20 --warmup 3 --no-cpu-baseline "$@" \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c5 line chunk', $ch, 'variant', $v, d['value'], 'MDoF/s', d['ms_per_step'], 'ms/step', r['kernel_ms_avg'], 'ms', r['achieved'], 'GB/s', r['frac'])"
done
done
