#!/bin/bash
# GPU suite at the tree (TRILINEAR layout), then same-box A/B on the trilinear C4 mesh:
# c = per-point qdata (round-2 path), d = TRILINEAR with unrolled planes, e = TRILINEAR runtime planes
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r3tl
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
bash profiles/ab_libs.sh tl_c4t "libecm2pa_c.so libecm2pa_d.so libecm2pa_e.so" --workload c4 --steps 30 --warmup 5 --variants 0 --mesh trilinear || exit $?

bash profiles/r3_member_emul.sh
[ $rc -eq 0 ] || exit $rc
