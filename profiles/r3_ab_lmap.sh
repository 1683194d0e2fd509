#!/bin/bash
# GPU suite at the tree (TRILINEAR layout), then same-box A/Bs: b = before lattice maps, c = with
# them (C4 entity, C3); c = per-point trilinear qdata vs d = TRILINEAR on-the-fly geometry
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r3lmap
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
bash profiles/ab_libs.sh lmap_c4e "libecm2pa_b.so libecm2pa_c.so" --workload c4 --steps 50 --warmup 5 --variants 0 --numbering entity || exit $?
bash profiles/ab_libs.sh lmap_c3 "libecm2pa_b.so libecm2pa_c.so" --workload c3 --steps 30 --warmup 5 || exit $?
[ $rc -eq 0 ] || exit $rc
bash profiles/ab_libs.sh tl_c4t "libecm2pa_c.so libecm2pa_d.so" --workload c4 --steps 30 --warmup 5 --variants 0 --mesh trilinear || exit $?
