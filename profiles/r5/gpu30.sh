# round 5, call 30: SQ counters at HEAD (after the XCD-contiguous order): headline, drop-in, C5
set -o pipefail
X="--steps 20 --warmup 3 --variants 0 --full-layout 0 --sdirk 0 --pcg-iters 0"
bash profiles/sq_pass.sh r5_c4 --workload c4 $X > /dev/null &&
bash profiles/sq_pass.sh r5_dropin --workload c4 --numbering entity --mesh trilinear --geometry-input jacobians $X > /dev/null &&
bash profiles/sq_pass.sh r5_c5 --workload c5 $X > /dev/null || exit 1
for t in r5_c4 r5_dropin r5_c5; do
  python3 -c "
import json
d=json.load(open('gpurun_out/sq_$t/sq_summary.json'))
for k,v in d.items():
    if v.get('dispatches',0) and ('apply' in k or 'sum' in k):
        print('$t', k[:24], {kk: round(v[kk],3) for kk in v if kk.endswith('_frac')})
"
done
