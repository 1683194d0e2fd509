#!/bin/bash
# Round 3: latency-kernel tail in the serial schedule (ECM2_TAIL=R: blocks past the last whole round
# of R resident blocks go to k_apply_tpe_pp in a second launch), emulated per-rank C4 Mult.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/tail
mkdir -p "$O"
ECM2_TAIL=3 timeout -k 10 300 python3 -u -m pytest tests/test_distributed.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "member_rows or group_matches" > "$O/pytest_tail3.log" 2>&1 || { tail -30 "$O/pytest_tail3.log"; exit 1; }
tail -1 "$O/pytest_tail3.log"
run() {  # tag decomp bench-args...
  local tag=$1 dec=$2; shift 2
  ECM2_DECOMP=$dec timeout -k 10 400 python3 bench.py --workload c4 --steps 50 --warmup 5 --no-cpu-baseline \
    --full-layout 0 --variants 0 "$@" > "$O/$tag.json" 2> "$O/$tag.err" || { tail -5 "$O/$tag.err"; return 1; }
  python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'N=%s' % b.get('emulated_n_gpus', 1), b.get('emulated_value', b.get('value')), 'MDoF/s slowest', b.get('slowest_member_ms', b.get('ms_per_step')), 'ms', b.get('member_ms', ''))" "$O/$tag.json" "$tag"
}
run n1 overlap || exit 1
for N in 8 4; do
  for dec in overlap rap; do
    run ${dec}_n$N $dec --loopback $N --member -1 || exit 1
    ECM2_TAIL=2048 run ${dec}_tail2048_n$N $dec --loopback $N --member -1 || exit 1
  done
done
ECM2_TAIL=1024 run overlap_tail1024_n8 overlap --loopback 8 --member -1 || exit 1
