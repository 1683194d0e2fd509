#!/bin/bash
# Same-box A/B of several library builds on one workload, alternating, twice each.
# Usage: bash profiles/ab_libs.sh <tag> "<lib-a.so> <lib-b.so> ..." [bench args]
# (library paths relative to cardiac-ablation-ecm2_amd/lib/)
set -uo pipefail
TAG=${1:-ab}; LIBS=${2:?library list}; shift 2 || true
ARGS=${*:---workload c5 --steps 30 --warmup 5}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/ablibs_$TAG
mkdir -p "$O"
export TMPDIR=/tmp
for rep in 1 2; do
  for v in $LIBS; do
    L=cardiac-ablation-ecm2_amd/lib/$v
    timeout -k 10 300 python3 profiles/ab_lib.py $L $ARGS --no-cpu-baseline --full-layout 0 > "$O/${v}_$rep.json" 2> "$O/${v}_$rep.err" || exit $?
    python3 -c "import json; d=json.loads(open('$O/${v}_$rep.json').read().strip().splitlines()[-1]); print('$v rep $rep', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
  done
done
