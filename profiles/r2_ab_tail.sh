#!/bin/bash
# A/B (experiment, source on branch exp/tail-pp) of the serial schedule's latency-kernel tail (ECM2_TAIL=k: the blocks past the apply kernel's last
# full round run in k_apply_tpe_pp when that takes <= k of its rounds) against one launch (ECM2_TAIL=0):
# parity with the tail on, then the emulated per-rank C4 Mult at N = 8, 4, 2, alternating.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/tail
mkdir -p "$O"
ECM2_TAIL=4 timeout -k 10 400 python3 -u -m pytest tests/test_distributed.py tests/test_gpu_configs.py tests/test_solvers.py \
  -m gpu -x -q --timeout 200 --timeout-method thread -k "not full_size" > "$O/parity_tail.log" 2>&1 || { tail -30 "$O/parity_tail.log"; exit 1; }
tail -1 "$O/parity_tail.log"
ECM2_TAIL=4 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "eight_way_members" > "$O/parity_tail_full.log" 2>&1 || { tail -30 "$O/parity_tail_full.log"; exit 1; }
tail -1 "$O/parity_tail_full.log"
for T in 0 1 4 0 1 4; do
  echo "-- ECM2_TAIL=$T"
  ECM2_TAIL=$T TAG=_t$T bash profiles/member_emul.sh 8 4 2 || exit $?
done
