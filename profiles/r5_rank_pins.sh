#!/bin/bash
# Round 5: the per-rank PMC pins a `bench.py --gpus N` line reports as its traffic, re-collected at HEAD
# (one slowest member per N, C4 slabs, OVERLAP, serial schedule: kernel trace, FETCH pass, WRITE pass ->
# pmc_reduce.py -> pmc_pin.py).  Usage: COMMIT=<sha> bash profiles/r5_rank_pins.sh
set -uo pipefail
export PIN_SCRIPT=profiles/r5_rank_pins.sh TMPDIR=/tmp PIN_DATE=$(date -u +%Y-%m-%dT%H:%MZ)
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/rankpins
mkdir -p "$O"
for nm in "2 1" "4 2" "8 3"; do
  set -- $nm
  bash profiles/run_profile.sh c4_n$1_member$2 --workload c4 --loopback $1 --member $2 --steps 30 --warmup 5 \
    --full-layout 0 --variants 0 > /dev/null || exit $?
  python3 profiles/pmc_pin.py ${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/prof_c4_n$1_member$2 c4 apply > "$O/pmc_c4_n$1_affine.json" || exit $?
  echo "N=$1 member $2: $(python3 -c "import json,sys; p=json.load(open(sys.argv[1])); print(p['hbm_bytes_per_launch'], p['trace_avg_ns'])" "$O/pmc_c4_n$1_affine.json")"
done
