#!/bin/bash
# Round 4, first GPU call: the GPU suite at the tree, the drop-in configuration's bench line
# (reference numbering + trilinear mesh + MFEM Jacobians), SQ counters of the TRILINEAR kernel
# on the trilinear C4 mesh and on the drop-in configuration.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r4p1
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --workload c4 --numbering entity --mesh trilinear --geometry-input jacobians \
  --steps 30 --warmup 5 --variants 0 --full-layout 0 --no-cpu-baseline > "$O/bench_drop.json" 2> "$O/bench_drop.err" || exit 1
tail -1 "$O/bench_drop.json" | cut -c1-400
bash profiles/sq_pass.sh c4tri --workload c4 --mesh trilinear --variants 0 --full-layout 0 --steps 20 --warmup 3 > "$O/sq_c4tri.txt" 2>&1 || exit 1
bash profiles/sq_pass.sh c4drop --workload c4 --numbering entity --mesh trilinear --geometry-input jacobians --variants 0 --full-layout 0 --steps 20 --warmup 3 > "$O/sq_c4drop.txt" 2>&1 || exit 1
bash profiles/sq_pass.sh c4 --workload c4 --variants 0 --full-layout 0 --steps 20 --warmup 3 > "$O/sq_c4.txt" 2>&1 || exit 1
echo done
