# round 5 A/B on one box: the C5 (68^3, p = 4) Mult with the brick-grid summation pass vs the run plan,
# and with / without the brick kernel's coefficient snapshot; two repetitions each, interleaved.
set -o pipefail
mkdir -p gpurun_out/r5/ab_c5
O=gpurun_out/r5/ab_c5
run() {  # tag, env, flags
  env $2 timeout -k 10 300 python -u bench.py --workload c5 --steps 50 --warmup 5 --full-layout 0 --variants 0 \
    --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || return 1
  python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=b['roofline']; print(sys.argv[2], b['value'], 'MDoF/s', b['ms_per_step'], 'ms/Mult', 'kernel', r['kernel_ms_avg'], b['config']['qdata_layout'])" $O/$1.json $1
}
for rep in 1 2; do
  run grid_ts_$rep "ECM2_SUM_GRID=1" "" &&
  run plan_ts_$rep "ECM2_SUM_GRID=0" "" &&
  run grid_nots_$rep "ECM2_SUM_GRID=1" "--coefficient-snapshot 0" &&
  run plan_nots_$rep "ECM2_SUM_GRID=0" "--coefficient-snapshot 0" || exit 1
done
