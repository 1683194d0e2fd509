#!/bin/bash
# A/B of the 3-waves-per-SIMD p = 2 apply variant (ECM2_TPE_LO=1: 168 VGPRs with spills, 26 LDS x rows,
# alternating exchange regions) against the default (246 VGPRs, 2 waves/SIMD): parity first, then
# the emulated per-rank Mult at N = 2, 4, 8 and the one-GPU C4 line, both variants on one box.
set -uo pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/lo
mkdir -p "$O"
ECM2_TPE_LO=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_distributed.py tests/test_gpu_configs.py \
  -m gpu -x -q --timeout 200 --timeout-method thread -k "not full_size" > "$O/parity_lo.log" 2>&1 || { tail -30 "$O/parity_lo.log"; exit 1; }
tail -1 "$O/parity_lo.log"
for LO in 0 1 0 1; do
  echo "-- ECM2_TPE_LO=$LO"
  ECM2_TPE_LO=$LO TAG=_lo$LO bash profiles/member_emul.sh 8 4 2 || exit $?
done
