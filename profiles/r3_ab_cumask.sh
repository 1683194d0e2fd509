#!/bin/bash
# Round 3: CU-partitioned overlapped schedule (ECM2_CU_SPLIT=k: the comm stream owns k CUs, the
# interior runs on a stream masked to the others) against the serial schedule, emulated per-rank
# Mult of the partitioned C4 operator (bench.py --loopback N --member -1, direct launches).
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/cumask
mkdir -p "$O"
ECM2_CU_SPLIT=32 timeout -k 10 300 python3 -u -m pytest tests/test_distributed.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "member_rows or overlapped_schedule or group_matches" > "$O/pytest_split32.log" 2>&1 || { tail -30 "$O/pytest_split32.log"; exit 1; }
tail -2 "$O/pytest_split32.log"
run() {  # tag decomp bench-args...
  local tag=$1 dec=$2; shift 2
  ECM2_DECOMP=$dec timeout -k 10 400 python3 bench.py --workload c4 --steps 50 --warmup 5 --no-cpu-baseline \
    --full-layout 0 --variants 0 "$@" > "$O/$tag.json" 2> "$O/$tag.err" || { tail -5 "$O/$tag.err"; return 1; }
  python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'N=%s' % b.get('emulated_n_gpus', 1), b.get('emulated_value', b.get('value')), 'MDoF/s slowest', b.get('slowest_member_ms', b.get('ms_per_step')), 'ms', b.get('member_ms', ''))" "$O/$tag.json" "$tag"
}
M="--loopback 8 --member -1"
run n1 overlap || exit 1
run serial_overlap_n8 overlap $M || exit 1
run serial_rap_n8 rap $M || exit 1
run ovl_nosplit_n8 overlap $M --schedule overlap --member-graph 0 || exit 1
for k in 32 64; do
  for mode in high stride; do
    ECM2_CU_SPLIT=$k ECM2_CU_SPLIT_MODE=$mode run ovl_s${k}_${mode}_n8 overlap $M --schedule overlap --member-graph 0 || exit 1
    ECM2_CU_SPLIT=$k ECM2_CU_SPLIT_MODE=$mode ECM2_BOUNDARY_KERNEL=tpe run ovl_s${k}_${mode}_tpe_n8 overlap $M --schedule overlap --member-graph 0 || exit 1
  done
done
ECM2_CU_SPLIT=32 run rap_s32_n8 rap $M --schedule overlap --member-graph 0 || exit 1
ECM2_CU_SPLIT=32 ECM2_BOUNDARY_KERNEL=tpe run rap_s32_tpe_n8 rap $M --schedule overlap --member-graph 0 || exit 1
