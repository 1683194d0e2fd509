# round 5 A/B on one box (C5, 68^3, p = 4): the brick-grid summation pass with K = 2 / 4 / 8 items per
# thread against the run plan (ECM2_SUM_GRID=0); then the snapshot forms without a per-point stream
# (--variants 2: pennes, ex16) with the brick snapshot on (ECM2_BRICK_TS=1) and off (0)
set -o pipefail
O=gpurun_out/r5/ab_c5b
mkdir -p $O
run() {  # tag, env, flags
  env $2 timeout -k 10 300 python -u bench.py --workload c5 --steps 50 --warmup 5 --full-layout 0 \
    --no-cpu-baseline $3 > $O/$1.json 2> $O/$1.err || return 1
  python3 - $O/$1.json $1 <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = b["roofline"]
line = [sys.argv[2], b["value"], "MDoF/s", b["ms_per_step"], "ms/Mult", "kernel", r["kernel_ms_avg"], b["config"]["qdata_layout"]]
for k in ("pennes", "ex16"):
    if k in b:
        line += ["|", k, b[k]["value"], b[k]["ms_per_step"], b[k]["roofline"]["kernel_ms_avg"], b[k]["qdata_layout"]]
print(*line)
PY
}
for rep in 1 2; do
  run plan_$rep "ECM2_SUM_GRID=0" "--variants 0" &&
  run grid2_$rep "ECM2_SUM_GRID=2" "--variants 0" &&
  run grid4_$rep "ECM2_SUM_GRID=4" "--variants 0" &&
  run grid8_$rep "ECM2_SUM_GRID=8" "--variants 0" || exit 1
done
for rep in 1 2; do
  run laws_ts_$rep "ECM2_BRICK_TS=1" "--variants 2" &&
  run laws_nots_$rep "ECM2_BRICK_TS=0" "--variants 2" || exit 1
done
