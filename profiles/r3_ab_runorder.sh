#!/bin/bash
# Round 3: summation-plan runs emitted by their smallest dof (ECM2_RUN_ORDER=dof) instead of by
# first partial slot, so neighbouring workgroups of the pass store neighbouring y lines.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/runorder
mkdir -p "$O"
ECM2_RUN_ORDER=dof timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "full_size or c5 or lattice or slabs" > "$O/pytest_dof.log" 2>&1 || { tail -30 "$O/pytest_dof.log"; exit 1; }
tail -1 "$O/pytest_dof.log"
run() {  # tag bench-args...
  local tag=$1; shift 1
  timeout -k 10 400 python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline \
    --full-layout 0 --variants 0 "$@" > "$O/$tag.json" 2> "$O/$tag.err" || { tail -5 "$O/$tag.err"; return 1; }
  python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=b['roofline']['kernel_ms_avg']; print(sys.argv[2], b['value'], 'MDoF/s', b['ms_per_step'], 'ms kernel', k, 'Mult-kernel us', round((b['ms_per_step']-k)*1e3,1))" "$O/$tag.json" "$tag"
}
for rep in 1 2; do
  for o in slot dof; do
    ECM2_RUN_ORDER=$o run c5_${o}_$rep --workload c5 || exit 1
    ECM2_RUN_ORDER=$o run c4ent_${o}_$rep --workload c4 --numbering entity || exit 1
    ECM2_RUN_ORDER=$o run c4_${o}_$rep --workload c4 || exit 1
    ECM2_RUN_ORDER=$o run c3_${o}_$rep --workload c3 || exit 1
  done
done
