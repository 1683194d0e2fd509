#!/bin/bash
# GPU suite at the tree, then same-box A/Bs of the summation pass: b = 432b12d (block row ->
# descriptor rows -> partials) vs c = fixed-size per-block records loaded at an address of the
# block index (one dependent global read less), on C5, C4 (both numberings) and C3
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r3rec
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit $rc
bash profiles/ab_libs.sh rec_c5 "libecm2pa_b.so libecm2pa_c.so" --workload c5 --steps 50 --warmup 5 || exit $?
bash profiles/ab_libs.sh rec_c4 "libecm2pa_b.so libecm2pa_c.so" --workload c4 --steps 50 --warmup 5 --variants 0 || exit $?
bash profiles/ab_libs.sh rec_c4e "libecm2pa_b.so libecm2pa_c.so" --workload c4 --steps 50 --warmup 5 --variants 0 --numbering entity || exit $?
bash profiles/ab_libs.sh rec_c3 "libecm2pa_b.so libecm2pa_c.so" --workload c3 --steps 30 --warmup 5 || exit $?
