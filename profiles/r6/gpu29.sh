# round 6, call 29: SQ counters of the headline kernel and the C5 brick kernel at the final tree (diagonal flux)
set -o pipefail
O=gpurun_out/r6/gpu29
mkdir -p $O
export TMPDIR=/tmp
SQ_ARGS="--workload c4 --steps 20 --warmup 3 --variants 0 --full-layout 0 --sdirk 0 --pcg-iters 0"
bash profiles/sq_pass.sh r6_c4_final $SQ_ARGS > /dev/null && cp gpurun_out/sq_r6_c4_final/sq_summary.json $O/sq_c4_final.json || exit 1
SQ_ARGS="--workload c5 --steps 20 --warmup 3 --variants 0 --full-layout 0 --sdirk 0 --pcg-iters 0"
bash profiles/sq_pass.sh r6_c5_final $SQ_ARGS > /dev/null && cp gpurun_out/sq_r6_c5_final/sq_summary.json $O/sq_c5_final.json || exit 1
python3 -c "
import json
for f in ('$O/sq_c4_final.json', '$O/sq_c5_final.json'):
    d = json.load(open(f))
    for k, v in d.items():
        if 'tpe_ts' in k or 'sum_partials' in k or 'brick' in k: print(k[:70], {kk: round(v[kk], 3) if isinstance(v[kk], float) else v[kk] for kk in v})
"
