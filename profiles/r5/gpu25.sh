# round 5, call 25: the atomic scatter mode (ECM2_SCATTER=atomic: y zeroed, shared dofs added with FP64
# atomics, no partial slots and no summation pass) against the deterministic partials, same box,
# alternating, on C4 (snapshot kernel), C4 reference numbering and C5
set -o pipefail
O=gpurun_out/r5/gpu25
mkdir -p $O
X="--variants 0 --full-layout 0 --no-cpu-baseline --sdirk 0 --pcg-iters 0"
run() {  # tag scatter bench-args
  local tag=$1 sc=$2; shift 2
  ECM2_SCATTER=$sc timeout -k 10 300 python -u bench.py "$@" $X > $O/$tag.json 2> $O/$tag.err || return 1
  python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=b['roofline']; print(sys.argv[2], b['value'], 'MDoF/s', b['ms_per_step'], 'ms/Mult', 'kernel', r['kernel_ms_avg'], b['config']['qdata_layout'])" $O/$tag.json $tag
}
for rep in 1 2; do
  for sc in partials atomic; do
    run c4_${sc}_$rep $sc --workload c4 --steps 50 --warmup 5 &&
    run c4ent_${sc}_$rep $sc --workload c4 --numbering entity --steps 50 --warmup 5 &&
    run c5_${sc}_$rep $sc --workload c5 --steps 30 --warmup 5 || exit 1
  done
done
