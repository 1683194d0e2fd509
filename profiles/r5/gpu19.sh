# round 5, call 19: the curved-mesh GPU tests (fichera-q2, -q3), then SQ counters at HEAD for the headline (c4), the drop-in configuration and C5
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k curved \
  > gpurun_out/r5/curved.txt 2>&1 || { tail -30 gpurun_out/r5/curved.txt; exit 1; }
tail -1 gpurun_out/r5/curved.txt
X="--steps 20 --warmup 3 --variants 0 --full-layout 0 --sdirk 0 --pcg-iters 0"
bash profiles/sq_pass.sh r5_c4 --workload c4 $X > /dev/null &&
bash profiles/sq_pass.sh r5_dropin --workload c4 --numbering entity --mesh trilinear --geometry-input jacobians $X > /dev/null &&
bash profiles/sq_pass.sh r5_c5 --workload c5 $X > /dev/null || exit 1
for t in r5_c4 r5_dropin r5_c5; do
  python3 -c "
import json,sys
d=json.load(open('gpurun_out/sq_$t/sq_summary.json'))['kernels']
for k,v in d.items():
    if v.get('dispatches',0) and ('apply' in k or 'sum' in k):
        print('$t', k[:40], {kk: round(v[kk],3) for kk in v if kk.endswith('_frac')}, 'VALU', v.get('SQ_INSTS_VALU'))
"
done
