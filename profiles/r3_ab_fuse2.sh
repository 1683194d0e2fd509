#!/bin/bash
# same-box A/B on C5: b = one brick launch (9601a19) vs d = two-colour schedule with the fused
# points' neighbour partials issued before the y transpose; kernel trace of d (launch times apart)
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r3fuse2
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread -k "c5 or C5" > "$O/pytest_c5.log" 2>&1
rc=$?
tail -2 "$O/pytest_c5.log"
[ $rc -eq 0 ] || exit $rc
bash profiles/ab_libs.sh fuse2_c5 "libecm2pa_b.so libecm2pa_d.so" --workload c5 --steps 50 --warmup 5 || exit $?
