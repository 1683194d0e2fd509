#!/bin/bash
# A/B (same box): qdata issued before the gather (b) vs after (a), C4 structured / entity / full layout
set -uo pipefail
for args in "--workload c4 --steps 50 --warmup 5 --variants 0" \
            "--workload c4 --steps 50 --warmup 5 --variants 0 --numbering entity" \
            "--workload c4 --steps 30 --warmup 5 --variants 0 --geometry full"; do
  tag=$(echo "$args" | tr -dc 'a-z0-9' | tail -c 24)
  echo "== $args"
  bash profiles/ab_libs.sh "pf_$tag" "libecm2pa_a.so libecm2pa_b.so" $args || exit $?
done
