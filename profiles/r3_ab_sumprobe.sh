#!/bin/bash
# Round 3: summation-pass timing probes (ECM2_SUM_PROBE; wrong results, timing only):
# 1 = every entry stored at y[entry index] (dense, whole lines); 2 = no partial reads (the value
# from the run lookup), stored at its dof as usual.  "Mult - kernel" = the pass + one launch gap.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/sumprobe
mkdir -p "$O"
run() {  # tag bench-args...
  local tag=$1; shift 1
  timeout -k 10 400 python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline \
    --full-layout 0 --variants 0 "$@" > "$O/$tag.json" 2> "$O/$tag.err" || { tail -5 "$O/$tag.err"; return 1; }
  python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=b['roofline']['kernel_ms_avg']; print(sys.argv[2], b['value'], 'MDoF/s', b['ms_per_step'], 'ms kernel', k, 'Mult-kernel us', round((b['ms_per_step']-k)*1e3,1))" "$O/$tag.json" "$tag"
}
for rep in 1 2; do
  for p in 0 1 2; do
    ECM2_SUM_PROBE=$p run c5_p${p}_$rep --workload c5 || exit 1
    ECM2_SUM_PROBE=$p run c4ent_p${p}_$rep --workload c4 --numbering entity || exit 1
    ECM2_SUM_PROBE=$p run c4_p${p}_$rep --workload c4 || exit 1
  done
done
