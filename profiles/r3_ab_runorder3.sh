#!/bin/bash
# Round 3: chain run order (greedy line sharing) against dof order and the lines-touched choice (auto).
# against slot order; ECM2_PLAN_DUMP prints each form's decision.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/runorder3
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_distributed.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "full_size or c5 or lattice or slabs or member_rows" > "$O/pytest_auto.log" 2>&1 || { tail -30 "$O/pytest_auto.log"; exit 1; }
tail -1 "$O/pytest_auto.log"
run() {  # tag bench-args...
  local tag=$1; shift 1
  timeout -k 10 400 python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline \
    --full-layout 0 --variants 0 "$@" > "$O/$tag.json" 2> "$O/$tag.err" || { tail -5 "$O/$tag.err"; return 1; }
  grep "lines touched" "$O/$tag.err" | head -1 | sed "s/^/  $tag: /"
  python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=b['roofline']['kernel_ms_avg']; print(sys.argv[2], b['value'], 'MDoF/s', b['ms_per_step'], 'ms kernel', k, 'Mult-kernel us', round((b['ms_per_step']-k)*1e3,1))" "$O/$tag.json" "$tag"
}
for rep in 1 2; do
  for o in dof chain auto; do
    ro=$o; [ $o = auto ] && ro=
    ECM2_PLAN_DUMP=1 ECM2_RUN_ORDER=$ro run c5_${o}_$rep --workload c5 || exit 1
    ECM2_PLAN_DUMP=1 ECM2_RUN_ORDER=$ro run c4ent_${o}_$rep --workload c4 --numbering entity || exit 1
    ECM2_PLAN_DUMP=1 ECM2_RUN_ORDER=$ro run c3_${o}_$rep --workload c3 || exit 1
    ECM2_PLAN_DUMP=1 ECM2_RUN_ORDER=$ro run c4_${o}_$rep --workload c4 || exit 1
  done
done
