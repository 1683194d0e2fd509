#!/bin/bash
# GPU suite at the tree (two-colour brick schedule on), then a same-box A/B on C5: b = 9601a19
# (one brick launch, every shared dof in the summation pass) vs c = two-colour schedule
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/r3fuse
mkdir -p "$O"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 200 --timeout-method thread -k "c5 or C5" > "$O/pytest_c5.log" 2>&1
rc=$?
tail -3 "$O/pytest_c5.log"; grep -E "FAILED|ERROR|Error" "$O/pytest_c5.log" | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"; grep -E "FAILED|ERROR" "$O/pytest_gpu.log" | head -20
[ $rc -eq 0 ] || exit $rc
bash profiles/ab_libs.sh fuse_c5 "libecm2pa_b.so libecm2pa_c.so" --workload c5 --steps 50 --warmup 5 || exit $?
