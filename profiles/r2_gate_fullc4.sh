#!/bin/bash
# the full-size 8-way C4 member parity test alone (timed)
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -v --timeout 500 --timeout-method thread -k "full_size" --durations=3 > "$O/pytest_fullc4.log" 2>&1
rc=$?
tail -8 "$O/pytest_fullc4.log"
exit $rc
