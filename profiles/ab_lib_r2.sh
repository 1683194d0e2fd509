#!/bin/bash
# Same-box A/B of two library builds (lib/libecm2pa_ab.so = before, lib/libecm2pa.so = after)
# on one workload, alternating, twice each.  Usage: bash profiles/ab_lib_r2.sh <tag> [bench args]
set -uo pipefail
TAG=${1:-ab}; shift || true
ARGS=${*:---workload c4 --steps 50 --warmup 5}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/ablib_$TAG
mkdir -p "$O"
export TMPDIR=/tmp
for rep in 1 2; do
  for v in before after; do
    L=cardiac-ablation-ecm2_amd/lib/libecm2pa.so; [ $v = before ] && L=cardiac-ablation-ecm2_amd/lib/libecm2pa_ab.so
    timeout -k 10 300 python3 profiles/ab_lib.py $L $ARGS --no-cpu-baseline --full-layout 0 > "$O/$v$rep.json" 2> "$O/$v$rep.err" || exit $?
    python3 -c "import json; d=json.loads(open('$O/$v$rep.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
  done
done
