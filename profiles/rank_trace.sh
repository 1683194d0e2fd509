#!/bin/bash
# Per-rank kernel durations of the partitioned Mult emulated on one GPU: bench.py --loopback N
# (N z-slab subdomains in one process) under rocprofv3 --kernel-trace, reduced by
# profiles/rank_trace.py (per kernel and grid size: the members' interior apply kernels run one
# after another on one stream, so each dispatch's duration is a rank's interior kernel alone).
# Usage: [EXTRA="--partition boxes"] [TAG=boxes] bash profiles/rank_trace.sh <workload> <N> [more N ...]
set -uo pipefail
WL=${1:-c4}; shift
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/rank_trace
mkdir -p "$O"
export TMPDIR=/tmp
for N in "$@"; do
  T=$WL${TAG:+-$TAG}-n$N
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/$T" -o run --output-format csv \
    -- python3 bench.py --workload $WL --loopback $N --steps 30 --warmup 5 --no-cpu-baseline --full-layout 0 ${EXTRA:-} \
    > "$O/$T.json" 2> "$O/$T.err" || exit $?
  python3 profiles/rank_trace.py "$O/$T" $N || exit $?
done
