#!/bin/bash
# One rocprofv3 SQ-counter pass (8 SQ slots, no TCC) over bench.py, reduced per kernel by
# profiles/sq_reduce.py: where the dominant kernels' wave cycles go (issue vs parked vs
# stalled), VALU / LDS instruction counts and LDS bank conflicts.
# Usage: bash profiles/sq_pass.sh <tag> [bench args...]
set -euo pipefail
TAG=${1:-c4}; shift || true
ARGS=${*:---workload c4 --steps 20 --warmup 3}
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/sq_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
C=${SQ_COUNTERS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT}
timeout -s KILL 120 rocprofv3 --pmc $C -T -d "$OUT" -o run --output-format csv \
  -- python3 bench.py $ARGS --no-cpu-baseline > "$OUT/bench.json"
python3 profiles/sq_reduce.py "$OUT" > "$OUT/sq_summary.json"
cat "$OUT/sq_summary.json"
