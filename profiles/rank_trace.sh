#!/bin/bash
# Per-rank kernel durations of the partitioned Mult emulated on one GPU: bench.py --loopback N
# (N z-slab subdomains in one process) under rocprofv3 --kernel-trace, reduced by
# profiles/rank_trace.py (per kernel and grid size: the members' interior apply kernels run one
# after another on one stream, so each dispatch's duration is a rank's interior kernel alone).
# Usage: bash profiles/rank_trace.sh <workload> <N> [more N ...]
set -uo pipefail
WL=${1:-c4}; shift
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/rank_trace
mkdir -p "$O"
export TMPDIR=/tmp
for N in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/$WL-n$N" -o run --output-format csv \
    -- python3 bench.py --workload $WL --loopback $N --steps 30 --warmup 5 --no-cpu-baseline --full-layout 0 \
    > "$O/$WL-n$N.json" 2> "$O/$WL-n$N.err" || exit $?
  python3 profiles/rank_trace.py "$O/$WL-n$N" $N || exit $?
done
