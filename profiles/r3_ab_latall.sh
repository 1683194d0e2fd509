#!/bin/bash
# Round 3: every p = 2 block on the latency kernel k_apply_tpe_pp (one workgroup per 64-element
# block, one quadrature plane per wave) instead of k_apply_tpe_sf (ECM2_LATENCY_ALL=1), for the
# one-round meshes (C2 50^3, an N = 8 rank of C4) and C4 on one GPU.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/latall
mkdir -p "$O"
ECM2_LATENCY_ALL=1 timeout -k 10 300 python3 -u -m pytest tests/test_distributed.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "(member_rows or group_matches or affine or tpe) and not reference_numbering and not full_size" > "$O/pytest_latall.log" 2>&1 || { tail -30 "$O/pytest_latall.log"; exit 1; }
tail -1 "$O/pytest_latall.log"
run() {  # tag bench-args...
  local tag=$1; shift 1
  timeout -k 10 400 python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline \
    --full-layout 0 --variants 0 "$@" > "$O/$tag.json" 2> "$O/$tag.err" || { tail -5 "$O/$tag.err"; return 1; }
  python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'N=%s' % b.get('emulated_n_gpus', 1), b.get('emulated_value', b.get('value')), 'MDoF/s slowest', b.get('slowest_member_ms', b.get('ms_per_step')), 'ms', b.get('member_ms', ''), 'kernel', b.get('roofline', {}).get('kernel_ms_avg', ''))" "$O/$tag.json" "$tag"
}
for rep in 1 2; do
  run c2_sf_$rep --workload c2 || exit 1
  ECM2_LATENCY_ALL=1 run c2_pp_$rep --workload c2 || exit 1
  run c4_sf_$rep --workload c4 || exit 1
  ECM2_LATENCY_ALL=1 run c4_pp_$rep --workload c4 || exit 1
done
run c4_n8_sf --workload c4 --loopback 8 --member -1 || exit 1
ECM2_LATENCY_ALL=1 run c4_n8_pp --workload c4 --loopback 8 --member -1 || exit 1
