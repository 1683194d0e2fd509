#!/bin/bash
# GPU suite at the tree, then same-box A/B of the per-point-layout kernel: c = double buffer with a
# conditional prefetch + buffer copy vs d = three row buffers in rotation (groups of three rows)
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r3pf3
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit $rc
bash profiles/ab_libs.sh pf3_c4f "libecm2pa_c.so libecm2pa_d.so" --workload c4 --steps 30 --warmup 5 --variants 0 --geometry full || exit $?
timeout -k 10 300 python3 bench.py --workload c4 --numbering entity --steps 50 --warmup 5 --variants 0 --no-cpu-baseline --full-layout 0 > "$O/bench_c4ent.json" 2> "$O/bench_c4ent.err" || exit $?
tail -1 "$O/bench_c4ent.json" | cut -c1-1500
