#!/bin/bash
# Round 3: emulated per-rank Mult of the partitioned C4 operator (bench.py --loopback N --member -1,
# serial schedule, direct launches): OVERLAP vs RAP, z-slabs vs 2 x 2 x 2 boxes (N = 8).
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/member_r3
mkdir -p "$O"
run() {  # tag decomp bench-args...
  local tag=$1 dec=$2; shift 2
  ECM2_DECOMP=$dec timeout -k 10 400 python3 bench.py --workload c4 --steps 50 --warmup 5 --no-cpu-baseline \
    --full-layout 0 --variants 0 "$@" > "$O/$tag.json" 2> "$O/$tag.err" || return 1
  python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'N=%s' % b.get('emulated_n_gpus', 1), b.get('emulated_value', b.get('value')), 'MDoF/s slowest', b.get('slowest_member_ms', b.get('ms_per_step')), 'ms', b.get('member_ms', ''))" "$O/$tag.json" "$tag"
}
run n1 overlap || exit 1
for N in 2 4 8; do
  run slabs_overlap_n$N overlap --loopback $N --member -1 || exit 1
  run slabs_rap_n$N rap --loopback $N --member -1 || exit 1
done
run boxes_overlap_n8 overlap --loopback 8 --member -1 --partition boxes || exit 1
run boxes_rap_n8 rap --loopback 8 --member -1 --partition boxes || exit 1
