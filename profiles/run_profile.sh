#!/bin/bash
# Collects the rocprofv3 evidence for bench.py on the GPU box (run from the repo root):
#   1) --kernel-trace --stats  (per-kernel durations; must agree with bench's HIP-event timing)
#   2) --pmc FETCH_SIZE and 3) --pmc WRITE_SIZE in separate passes (TCC slots, MI355X_MICROARCH.md)
# then reduces them to per-launch HBM bytes of the dominant kernel (profiles/pmc_reduce.py).
# Usage: bash profiles/run_profile.sh <tag> [bench args...]
set -euo pipefail
TAG=${1:-c2}; shift || true
ARGS=${*:---steps 50 --warmup 5}
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/prof_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d "$OUT/trace" -o run --output-format csv \
  -- python3 bench.py $ARGS --no-cpu-baseline > "$OUT/bench_trace.json"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/fetch" -o run --output-format csv \
  -- python3 bench.py $ARGS --no-cpu-baseline > "$OUT/bench_fetch.json"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/write" -o run --output-format csv \
  -- python3 bench.py $ARGS --no-cpu-baseline > "$OUT/bench_write.json"
python3 profiles/pmc_reduce.py "$OUT" > "$OUT/pmc_summary.json"
cat "$OUT/pmc_summary.json"
