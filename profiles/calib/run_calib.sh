#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on the GPU box (run from the repo root after building
# profiles/calib/fetch_calib here: hipcc --offload-arch=gfx950 -O3 -o profiles/calib/fetch_calib
# profiles/calib/fetch_calib.hip).  Separate counter passes (TCC slots).
set -euo pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/calib
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/fetch" -o run --output-format csv -- ./profiles/calib/fetch_calib > "$OUT/known.json"
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/write" -o run --output-format csv -- ./profiles/calib/fetch_calib > /dev/null
timeout -s KILL 60 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- ./profiles/calib/fetch_calib > /dev/null
python3 profiles/calib/calib_reduce.py "$OUT" > "$OUT/calibration.json"
cat "$OUT/calibration.json"
