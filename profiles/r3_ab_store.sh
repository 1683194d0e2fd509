#!/bin/bash
# GPU suite at the tree, then same-box A/Bs of b = HEAD before vs c = (1) all-lattice-map kernel
# (RM = 3: no treg row in the gather chain, face-grouped partial stride), (2) a lattice-map block's
# store entries loaded before the face merges, (3) longer explicit-dof summation runs preferred.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r3store
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit $rc
bash profiles/ab_libs.sh st_c4e "libecm2pa_b.so libecm2pa_c.so" --workload c4 --steps 50 --warmup 5 --variants 0 --numbering entity || exit $?
bash profiles/ab_libs.sh st_c4 "libecm2pa_b.so libecm2pa_c.so" --workload c4 --steps 50 --warmup 5 --variants 0 || exit $?
bash profiles/ab_libs.sh st_c3 "libecm2pa_b.so libecm2pa_c.so" --workload c3 --steps 30 --warmup 5 || exit $?
