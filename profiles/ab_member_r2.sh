#!/bin/bash
# Same-box A/B of two library builds (lib/libecm2pa_ab.so = before, lib/libecm2pa.so = after) on the
# emulated per-rank Mult (bench.py --loopback N --member -1) and optionally a serial workload.
# Usage: bash profiles/ab_member_r2.sh <tag> [N ...]
set -uo pipefail
TAG=${1:-ab}; shift || true
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/abmember_$TAG
mkdir -p "$O"
for N in ${@:-8}; do
  for rep in 1 2; do
    for v in before after; do
      L=cardiac-ablation-ecm2_amd/lib/libecm2pa.so; [ $v = before ] && L=cardiac-ablation-ecm2_amd/lib/libecm2pa_ab.so
      timeout -k 10 300 python3 profiles/ab_lib.py $L --workload ${WL:-c4} --loopback $N --member -1 --steps 50 --warmup 5 \
        --no-cpu-baseline --full-layout 0 > "$O/$v$rep-n$N.json" 2> "$O/$v$rep-n$N.err" || exit $?
      python3 -c "import json; d=json.loads(open('$O/$v$rep-n$N.json').read().strip().splitlines()[-1]); print('N=$N $v', d['slowest_member_ms'], d['member_ms'])"
    done
  done
done
