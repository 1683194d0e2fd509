#!/bin/bash
# A/B of the XCD-contiguous workgroup order: TPE (C2, C4: ECM2_TPE_VARIANT 4 vs 20) and
# line kernel (C5: chunk length x ECM2_LINE_VARIANT 0/2/4).
set -u
line() { python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$1', d['value'], 'MDoF/s', d['ms_per_step'], 'ms/step', r['kernel_ms_avg'], 'ms', r['achieved'], 'GB/s', r['frac'])"; }
for w in c2 c4; do for v in 4 20; do
  ECM2_TPE_VARIANT=$v timeout -k 10 200 python3 bench.py --workload $w --steps 50 --warmup 5 --no-cpu-baseline | line "$w tpe variant $v"
done; done
for ch in ${CHUNKS:-1 8}; do for v in ${LVARIANTS:-0 2 4}; do
  ECM2_LINE_CHUNK=$ch ECM2_LINE_VARIANT=$v timeout -k 10 200 python3 bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline | line "c5 line chunk $ch variant $v"
done; done
