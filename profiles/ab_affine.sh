#!/bin/bash
# A/B of the AFFINE qdata layout (p <= 2 fused kernel): --geometry compressed (default) vs
# full, x ECM2_TPE_VARIANT (0 = default, 8 = two waves per SIMD bound, 2 = cached loads),
# on C2 / C4 (and C3 with its PCG).  One line per run.
set -eu
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
for w in ${WORKLOADS:-c2 c4}; do
for g in ${GEOMS:-compressed full}; do
for v in ${VARIANTS:-0}; do
  extra=""; steps=50
  if [ "$w" = c2 ]; then steps=200; fi
  if [ "$w" = c3 ]; then extra="--workload c3"; steps=20; fi
  [ "$w" = c2 ] || [ "$w" = c3 ] || extra="--workload $w"
  ECM2_TPE_VARIANT=$v timeout -k 10 300 python3 bench.py $extra --geometry $g --steps $steps --warmup 5 --no-cpu-baseline > "$O/ab_affine_${w}_${g}_${v}.json"
  python3 -c "import json,sys; d=json.load(open('$O/ab_affine_${w}_${g}_${v}.json')); r=d['roofline']; print('$w', '$g', 'var', $v, d['value'], 'MDoF/s', d['ms_per_step'], 'ms/step', r['kernel_ms_avg'], 'ms', r['achieved'], 'GB/s', r['frac'], d['config']['qdata_layout'], d.get('pcg'))"
done
done
done
